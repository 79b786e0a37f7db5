// flock_sc.hip — fused shared-critic DDPG update on gfx950 (C ABI: include/flock_learn.h, flock_sc_*).
//
// One Agent.learn() (learners/maddpg_shared_critic/agent_simple_shared_critic.py:115-150) is 12 launches instead
// of the ~130 small torch kernels of an autograd step:
//   critic phase (:118-141)                          actor phase (:144-150, through the UPDATED critic)
//   c1  rows: gather + fc1/LN/ReLU (3 paths)          a1  rows: actor fc1/LN/ReLU, critic fc1/LN/ReLU on s
//   c2  GEMM x3: fc2 of target actor / critic(s') /   a2  GEMM x2: actor fc2, critic fc2
//       critic(s)                                    a3  rows: LN2, mu, Q(s, mu), dQ/dmu, tanh + LN2 backward
//   c3  rows: LN2, heads, target y, MSE, backward    a4  GEMM: d fc1-out = dZ2 W2
//       through q / action_value / LN2               a5  rows: ReLU + LN1 backward
//   c4  GEMM: d fc1-out = dZ2 W2                     a6  grad + Adam (agent's slice, actor_steps[agent])
//   c5  rows: ReLU + LN1 backward
//   c6  grad + Adam: dW2 = dZ2^T H1 as a K=B GEMM with Adam in the epilogue; every other parameter is a
//       deterministic reduction over the B rows with Adam inline; the last block bumps the step counter.
//
// These launches are tiny (B = 256 rows) and each starts with a cold L2 (kernel-boundary writeback/invalidate of
// coarse-grained buffers), so their cost is the number of DEPENDENT memory round trips, not bytes or flops. Every
// kernel therefore issues all of its loads up front: parameters are flat contiguous regions (fc1 block, LN2 + head
// tail) staged into LDS in one round of 16-B loads; GEMM K-panels (<= 512 deep) are loaded whole into LDS in one
// round, then the four waves split K on v_mfma_f32_32x32x2_f32 (bit-for-bit a k-ordered fmaf chain) and combine
// their partial tiles in a fixed order.
// Row kernels: one wave64 per replay row (4 rows per 256-thread block), row vectors in registers (lane j holds
// features j, j+64, ...), LayerNorm statistics by xor-butterfly wave sums (bitwise identical in every lane).
// Numerics: the math of torch's fp32 ops in a different summation order (not bit-exact; tests use tolerances).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "flock_learn.h"
#include "learn_internal.h"

namespace {

using flock_learn_internal::fail;
using flock_learn_internal::launched;

constexpr int kRowsPerBlock = 4;
constexpr int kMaxAct = 4;
constexpr int kMaxIn = 64;
constexpr int kMaxFeat = 1024;
constexpr int kMaxFc1Block = 32768;  // fc1 (in + 3) floats staged in LDS per block
constexpr float kLnEps = 1e-5f;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------------------------------------------
// parameter and workspace layouts
struct CriticOff {
    int64_t W1, b1, g1, be1, W2, b2, g2, be2, Wa, ba, Wq, bq, total;
};
struct ActorOff {
    int64_t W1, b1, g1, be1, W2, b2, g2, be2, Wmu, bmu, total;
};
__host__ __device__ inline CriticOff critic_off(int in, int na, int H1, int H2) {
    CriticOff o;
    o.W1 = 0;
    o.b1 = o.W1 + (int64_t)H1 * in;
    o.g1 = o.b1 + H1;
    o.be1 = o.g1 + H1;
    o.W2 = o.be1 + H1;
    o.b2 = o.W2 + (int64_t)H2 * H1;
    o.g2 = o.b2 + H2;
    o.be2 = o.g2 + H2;
    o.Wa = o.be2 + H2;
    o.ba = o.Wa + (int64_t)H2 * na;
    o.Wq = o.ba + H2;
    o.bq = o.Wq + H2;
    o.total = o.bq + 1;
    return o;
}
__host__ __device__ inline ActorOff actor_off(int in, int na, int H1, int H2) {
    ActorOff o;
    o.W1 = 0;
    o.b1 = o.W1 + (int64_t)H1 * in;
    o.g1 = o.b1 + H1;
    o.be1 = o.g1 + H1;
    o.W2 = o.be1 + H1;
    o.b2 = o.W2 + (int64_t)H2 * H1;
    o.g2 = o.b2 + H2;
    o.be2 = o.g2 + H2;
    o.Wmu = o.be2 + H2;
    o.bmu = o.Wmu + (int64_t)na * H2;
    o.total = o.bmu + na;
    return o;
}
// LDS images of the flat tails [g2, be2, Wa, ba, Wq, bq] (critic) and [g2, be2, Wmu, bmu] (actor)
__host__ __device__ inline int crit_tail_len(int na, int H2) { return 2 * H2 + H2 * na + 2 * H2 + 1; }
__host__ __device__ inline int act_tail_len(int na, int H2) { return 2 * H2 + na * H2 + na; }
__host__ __device__ inline int round4(int n) { return (n + 3) & ~3; }

// workspace: [B, dim] row-major arrays
struct Ws {
    float *S, *A, *R, *T, *S2;             // gathered replay rows
    float *TH1, *NH1, *XH1, *RS1, *H1;     // fc1 outputs: target actor(s'), critic(s'), critic(s) xhat/rstd/h
    float* Z2;                             // [3][B][H2] fc2 pre-LN: target actor(s'), critic(s'), critic(s)
    float *XH2, *RS2, *HQ, *DZA, *DY2, *DZ2, *DQ, *LOSS;
    float *DH1, *DY1, *DZ1;
    float *AXH1, *ARS1, *AH1, *CH1;        // actor phase fc1: actor xhat/rstd/h, updated critic h
    float* Z2b;                            // [2][B][H2] actor fc2, critic fc2
    float *AXH2, *ARS2, *AH2, *DM, *ADY2, *ADZ2, *ALOSS;
    float *ADH1, *ADY1, *ADZ1;
};

int64_t ws_layout(int B, int in, int na, int H1, int H2, float* base, Ws* w) {
    int64_t off = 0;
    auto take = [&](int64_t per_row) {
        float* p = base ? base + off : nullptr;
        off += (int64_t)B * per_row;
        off = (off + 63) & ~(int64_t)63;  // 256-B aligned arrays
        return p;
    };
    Ws x;
    x.S = take(in); x.A = take(na); x.R = take(1); x.T = take(1); x.S2 = take(in);
    x.TH1 = take(H1); x.NH1 = take(H1); x.XH1 = take(H1); x.RS1 = take(1); x.H1 = take(H1);
    x.Z2 = take(3 * (int64_t)H2);
    x.XH2 = take(H2); x.RS2 = take(1); x.HQ = take(H2); x.DZA = take(H2); x.DY2 = take(H2); x.DZ2 = take(H2);
    x.DQ = take(1); x.LOSS = take(1);
    x.DH1 = take(H1); x.DY1 = take(H1); x.DZ1 = take(H1);
    x.AXH1 = take(H1); x.ARS1 = take(1); x.AH1 = take(H1); x.CH1 = take(H1);
    x.Z2b = take(2 * (int64_t)H2);
    x.AXH2 = take(H2); x.ARS2 = take(1); x.AH2 = take(H2); x.DM = take(na); x.ADY2 = take(H2); x.ADZ2 = take(H2);
    x.ALOSS = take(1);
    x.ADH1 = take(H1); x.ADY1 = take(H1); x.ADZ1 = take(H1);
    if (w) *w = x;
    return off;
}

// everything the row kernels read
struct RowArgs {
    int B, in, na, H1, H2;
    const int64_t* idx;
    const int64_t* agent;
    const float *rs, *rs2, *ra, *rr, *rt;  // ring
    const float* critic;
    const float* actors;
    const float* actors_target;
    int64_t stride;
    float gamma, invB;
};

// ---------------------------------------------------------------------------------------------------------------
// helpers
// wave64 all-reduce sum on DPP (quad_perm, row half-mirror, row mirror: every lane of a 16-lane row adds commutative
// pairs, so the row sum is bitwise identical in all of its lanes) + readlane of the four row sums (a scalar, so the
// result is identical in every lane). Replaces a 6-step ds_bpermute butterfly (LDS-path latency per step).
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_sum(float v) {
    v = dpp_add<0xB1>(v);   // quad_perm [1,0,3,2]
    v = dpp_add<0x4E>(v);   // quad_perm [2,3,0,1]
    v = dpp_add<0x141>(v);  // row_half_mirror
    v = dpp_add<0x140>(v);  // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}
__device__ __forceinline__ float relu(float x) { return x > 0.0f ? x : 0.0f; }
__device__ __forceinline__ float rsqrt_rn(float x) { return 1.0f / __builtin_sqrtf(x); }

// copy n floats global -> LDS (dst 16-B aligned) with every load of a round issued before any LDS store
__device__ __forceinline__ void stage(float* __restrict__ dst, const float* __restrict__ src, int n) {
    const int tid = threadIdx.x;
    if (((uintptr_t)src & 15) == 0) {
        const int n4 = n >> 2;
        const float4* s4 = reinterpret_cast<const float4*>(src);
        for (int base = 0; base < n4; base += 256 * 8) {
            float4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int t = base + tid + 256 * i;
                v[i] = t < n4 ? s4[t] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int t = base + tid + 256 * i;
                if (t < n4) reinterpret_cast<float4*>(dst)[t] = v[i];
            }
        }
        for (int t = 4 * n4 + tid; t < n; t += 256) dst[t] = src[t];
    } else {
        for (int base = 0; base < n; base += 256 * 16) {
            float v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = base + tid + 256 * i;
                v[i] = t < n ? src[t] : 0.0f;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = base + tid + 256 * i;
                if (t < n) dst[t] = v[i];
            }
        }
    }
}

// mean / rstd of a register row (biased variance, like nn.LayerNorm)
template <int C>
__device__ __forceinline__ void ln_stats(const float (&z)[C], int F, int lane, float& mean, float& rstd) {
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c)
        if (lane + 64 * c < F) s += z[c];
    mean = wave_sum(s) / (float)F;
    float q = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c)
        if (lane + 64 * c < F) {
            const float d = z[c] - mean;
            q = fmaf(d, d, q);
        }
    rstd = rsqrt_rn(wave_sum(q) / (float)F + kLnEps);
}

template <int C>
__device__ __forceinline__ void load_row(float (&v)[C], const float* p, int F, int lane) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        v[c] = j < F ? p[j] : 0.0f;
    }
}
template <int C>
__device__ __forceinline__ void store_row(float* p, const float (&v)[C], int F, int lane) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        if (j < F) p[j] = v[c];
    }
}

// fc1 from an LDS image [W1 (F x in), b1, g1, be1] and the input row xs (LDS): z = W x + b, LayerNorm -> xhat, rstd;
// h = ReLU(xhat g + be)
template <int C>
__device__ __forceinline__ void fc1_ln_relu(const float* xs, int in, const float* sp, int F, int lane,
                                            float (&xh)[C], float (&h)[C], float& rstd) {
    const float* b = sp + F * in;
    const float* g = b + F;
    const float* be = g + F;
    float z[C];
#pragma unroll
    for (int c = 0; c < C; ++c) z[c] = 0.0f;
    for (int i = 0; i < in; ++i) {
        const float xi = xs[i];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int j = lane + 64 * c;
            if (j < F) z[c] = fmaf(xi, sp[j * in + i], z[c]);
        }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        if (j < F) z[c] = z[c] + b[j];
    }
    float mean;
    ln_stats<C>(z, F, lane, mean, rstd);
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        xh[c] = (z[c] - mean) * rstd;
        h[c] = j < F ? relu(fmaf(xh[c], g[j], be[j])) : 0.0f;
    }
}

// y = LN(z) * g + be for a register row z (g, be in LDS)
template <int C>
__device__ __forceinline__ void ln_affine(const float (&z)[C], const float* g, const float* be, int F, int lane,
                                          float (&xh)[C], float (&y)[C], float& rstd) {
    float mean;
    ln_stats<C>(z, F, lane, mean, rstd);
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        xh[c] = (z[c] - mean) * rstd;
        y[c] = j < F ? fmaf(xh[c], g[j], be[j]) : 0.0f;
    }
}

// LayerNorm backward for one row: dz = rstd * (dxh - mean(dxh) - xh * mean(dxh * xh)), dxh = dy * g
template <int C>
__device__ __forceinline__ void ln_backward(const float (&dy)[C], const float (&xh)[C], const float (&g)[C],
                                            float rstd, int F, float (&dz)[C]) {
    float dxh[C], s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        dxh[c] = dy[c] * g[c];
        s1 += dxh[c];
        s2 = fmaf(dxh[c], xh[c], s2);
    }
    const float m1 = wave_sum(s1) / (float)F, m2 = wave_sum(s2) / (float)F;
#pragma unroll
    for (int c = 0; c < C; ++c) dz[c] = rstd * (dxh[c] - m1 - xh[c] * m2);
}

// ---------------------------------------------------------------------------------------------------------------
// c1 (grid.y = path): 0 target actor on s', 1 critic on s', 2 critic on s (+ the gathered minibatch rows)
template <int C>
__device__ __forceinline__ void c1_body(const Ws& w, const RowArgs& a, int bx, int path) {
    extern __shared__ float4 smem4[];
    float* xs = reinterpret_cast<float*>(smem4);  // [4 rows][kMaxIn] inputs, then the fc1 image
    float* sp = xs + kRowsPerBlock * kMaxIn;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r = bx * kRowsPerBlock + wv;
    const float* net = path == 0 ? a.actors_target + (*a.agent) * a.stride : a.critic;  // fc1 block at offset 0
    const bool live = r < a.B;
    if (live) {
        const int64_t ir = a.idx[r];
        const float* x = (path == 2 ? a.rs : a.rs2) + ir * a.in;
        if (lane < a.in) xs[wv * kMaxIn + lane] = x[lane];
        if (path == 2) {
            if (lane < a.in) {
                w.S[(int64_t)r * a.in + lane] = x[lane];
                w.S2[(int64_t)r * a.in + lane] = a.rs2[ir * a.in + lane];
            }
            if (lane < a.na) w.A[(int64_t)r * a.na + lane] = a.ra[ir * a.na + lane];
            if (lane == 0) {
                w.R[r] = a.rr[ir];
                w.T[r] = a.rt[ir];
            }
        }
    }
    stage(sp, net, a.H1 * (a.in + 3));
    __syncthreads();
    if (!live) return;
    float xh[C], h[C], rs;
    fc1_ln_relu<C>(xs + wv * kMaxIn, a.in, sp, a.H1, lane, xh, h, rs);
    const int64_t ro = (int64_t)r * a.H1;
    if (path == 0) {
        store_row<C>(w.TH1 + ro, h, a.H1, lane);
    } else if (path == 1) {
        store_row<C>(w.NH1 + ro, h, a.H1, lane);
    } else {
        store_row<C>(w.XH1 + ro, xh, a.H1, lane);
        store_row<C>(w.H1 + ro, h, a.H1, lane);
        if (lane == 0) w.RS1[r] = rs;
    }
}

// c3: heads, TD target, MSE and the critic backward down to the fc2 pre-activation
template <int C>
__device__ __forceinline__ void c3_body(const Ws& w, const RowArgs& a, int bx) {
    extern __shared__ float4 smem4[];
    float* ct = reinterpret_cast<float*>(smem4);  // critic tail
    const int H2 = a.H2, na = a.na;
    float* at = ct + round4(crit_tail_len(na, H2));  // target actor tail
    const int lane = threadIdx.x & 63;
    const int r = bx * kRowsPerBlock + (threadIdx.x >> 6);
    const bool live = r < a.B;
    const CriticOff co = critic_off(a.in, na, a.H1, H2);
    const ActorOff ao = actor_off(a.in, na, a.H1, H2);
    float zt[C], zn[C], zs[C];
    float rwd = 0.0f, term = 0.0f, act[kMaxAct];
    if (live) {
        load_row<C>(zt, w.Z2 + (int64_t)r * H2, H2, lane);
        load_row<C>(zn, w.Z2 + ((int64_t)a.B + r) * H2, H2, lane);
        load_row<C>(zs, w.Z2 + (2 * (int64_t)a.B + r) * H2, H2, lane);
        rwd = w.R[r];
        term = w.T[r];
#pragma unroll
        for (int o = 0; o < kMaxAct; ++o) act[o] = o < na ? w.A[(int64_t)r * na + o] : 0.0f;
    }
    stage(ct, a.critic + co.g2, crit_tail_len(na, H2));
    stage(at, a.actors_target + (*a.agent) * a.stride + ao.g2, act_tail_len(na, H2));
    __syncthreads();
    if (!live) return;
    const float *cg2 = ct, *cbe2 = ct + H2, *cWa = ct + 2 * H2, *cba = cWa + H2 * na, *cWq = cba + H2;
    const float cbq = cWq[H2];
    const float *tg2 = at, *tbe2 = at + H2, *tWmu = at + 2 * H2, *tbmu = tWmu + na * H2;
    float xh[C], y[C], rs;

    // target actor on s': mu' = tanh(Wmu ReLU(LN2(z)) + bmu)                    (:126, ddpg_network.py:134-140)
    ln_affine<C>(zt, tg2, tbe2, H2, lane, xh, y, rs);
    float ta[kMaxAct];
#pragma unroll
    for (int o = 0; o < kMaxAct; ++o) {
        ta[o] = 0.0f;
        if (o >= na) continue;
        float p = 0.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int j = lane + 64 * c;
            if (j < H2) p = fmaf(relu(y[c]), tWmu[o * H2 + j], p);
        }
        ta[o] = tanhf(wave_sum(p) + tbmu[o]);
    }
    // target critic (== critic) on (s', mu'): q' = Wq ReLU(LN2(z) + ReLU(Wa mu' + ba)) + bq          (:127)
    ln_affine<C>(zn, cg2, cbe2, H2, lane, xh, y, rs);
    float qp = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        if (j < H2) {
            float za = 0.0f;
#pragma unroll
            for (int o = 0; o < kMaxAct; ++o)
                if (o < na) za = fmaf(ta[o], cWa[j * na + o], za);
            za = za + cba[j];
            qp = fmaf(cWq[j], relu(y[c] + relu(za)), qp);
        }
    }
    const float qn = wave_sum(qp) + cbq;
    const float target = rwd + (a.gamma * qn) * term;  // :130 (terminal stored as 1 - done)

    // critic on (s, a), keeping what the backward needs                                                   (:128)
    ln_affine<C>(zs, cg2, cbe2, H2, lane, xh, y, rs);
    float za[C], u[C];
    qp = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        za[c] = 0.0f;
        u[c] = 0.0f;
        if (j < H2) {
            float acc = 0.0f;
#pragma unroll
            for (int o = 0; o < kMaxAct; ++o)
                if (o < na) acc = fmaf(act[o], cWa[j * na + o], acc);
            za[c] = acc + cba[j];
            u[c] = y[c] + relu(za[c]);
            qp = fmaf(cWq[j], relu(u[c]), qp);
        }
    }
    const float q = wave_sum(qp) + cbq;
    const float diff = target - q;
    const float dq = 2.0f * (q - target) * a.invB;  // d/dq mean((target - q)^2)                           (:139)
    if (lane == 0) {
        w.DQ[r] = dq;
        w.LOSS[r] = diff * diff;
    }
    float dy2[C], dz2[C], g2[C];
    const int64_t ro = (int64_t)r * H2;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        dy2[c] = 0.0f;
        g2[c] = 0.0f;
        if (j < H2) {
            const float du = u[c] > 0.0f ? dq * cWq[j] : 0.0f;  // through q and the outer ReLU
            dy2[c] = du;
            g2[c] = cg2[j];
            w.HQ[ro + j] = relu(u[c]);
            w.DZA[ro + j] = za[c] > 0.0f ? du : 0.0f;  // through ReLU(action_value)
        }
    }
    ln_backward<C>(dy2, xh, g2, rs, H2, dz2);
    store_row<C>(w.DY2 + ro, dy2, H2, lane);
    store_row<C>(w.XH2 + ro, xh, H2, lane);
    store_row<C>(w.DZ2 + ro, dz2, H2, lane);
    if (lane == 0) w.RS2[r] = rs;
}

// c5 / a5: ReLU + LN1 backward: dy = dh * [h > 0]; dz = LN backward(dy)
struct Ln1Args {
    int B, F;
    const float *DH, *XH, *RS, *H, *g_base;
    const int64_t* agent;  // g_base is agent-relative (+ stride * (*agent)) when non-NULL
    int64_t stride;
    float *DY, *DZ;
};
template <int C>
__device__ __forceinline__ void ln1_body(const Ln1Args& l, int bx) {
    const int lane = threadIdx.x & 63;
    const int r = bx * kRowsPerBlock + (threadIdx.x >> 6);
    const int F = l.F;
    if (r >= l.B) return;
    const float* g = l.g_base + (l.agent ? (*l.agent) * l.stride : 0);
    const int64_t ro = (int64_t)r * F;
    float dh[C], xh[C], h[C], gv[C], dy[C], dz[C];
    load_row<C>(dh, l.DH + ro, F, lane);
    load_row<C>(xh, l.XH + ro, F, lane);
    load_row<C>(h, l.H + ro, F, lane);
    load_row<C>(gv, g, F, lane);
    const float rs = l.RS[r];
#pragma unroll
    for (int c = 0; c < C; ++c) dy[c] = h[c] > 0.0f ? dh[c] : 0.0f;
    ln_backward<C>(dy, xh, gv, rs, F, dz);
    store_row<C>(l.DY + ro, dy, F, lane);
    store_row<C>(l.DZ + ro, dz, F, lane);
}

// a1 (grid.y = path): 0 the agent's actor fc1/LN/ReLU on s (saved for backward), 1 the updated critic's on s
template <int C>
__device__ __forceinline__ void a1_body(const Ws& w, const RowArgs& a, int bx, int path) {
    extern __shared__ float4 smem4[];
    float* xs = reinterpret_cast<float*>(smem4);
    float* sp = xs + kRowsPerBlock * kMaxIn;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r = bx * kRowsPerBlock + wv;
    const bool live = r < a.B;
    const float* net = path == 0 ? a.actors + (*a.agent) * a.stride : a.critic;
    if (live && lane < a.in) xs[wv * kMaxIn + lane] = w.S[(int64_t)r * a.in + lane];
    stage(sp, net, a.H1 * (a.in + 3));
    __syncthreads();
    if (!live) return;
    float xh[C], h[C], rs;
    fc1_ln_relu<C>(xs + wv * kMaxIn, a.in, sp, a.H1, lane, xh, h, rs);
    const int64_t ro = (int64_t)r * a.H1;
    if (path == 0) {
        store_row<C>(w.AXH1 + ro, xh, a.H1, lane);
        store_row<C>(w.AH1 + ro, h, a.H1, lane);
        if (lane == 0) w.ARS1[r] = rs;
    } else {
        store_row<C>(w.CH1 + ro, h, a.H1, lane);
    }
}

// a3: actor LN2/ReLU/mu/tanh, Q(s, mu) with the updated critic, actor loss -mean Q, and the backward through the
// critic's action branch (dQ/dmu) and the actor head down to the actor's fc2 pre-activation
template <int C>
__device__ __forceinline__ void a3_body(const Ws& w, const RowArgs& a, int bx) {
    extern __shared__ float4 smem4[];
    float* ct = reinterpret_cast<float*>(smem4);
    const int H2 = a.H2, na = a.na;
    float* at = ct + round4(crit_tail_len(na, H2));
    const int lane = threadIdx.x & 63;
    const int r = bx * kRowsPerBlock + (threadIdx.x >> 6);
    const bool live = r < a.B;
    const CriticOff co = critic_off(a.in, na, a.H1, H2);
    const ActorOff ao = actor_off(a.in, na, a.H1, H2);
    const int64_t ro = (int64_t)r * H2;
    float za2[C], zc2[C];
    if (live) {
        load_row<C>(za2, w.Z2b + ro, H2, lane);
        load_row<C>(zc2, w.Z2b + ((int64_t)a.B + r) * H2, H2, lane);
    }
    stage(ct, a.critic + co.g2, crit_tail_len(na, H2));
    stage(at, a.actors + (*a.agent) * a.stride + ao.g2, act_tail_len(na, H2));
    __syncthreads();
    if (!live) return;
    const float *cg2 = ct, *cbe2 = ct + H2, *cWa = ct + 2 * H2, *cba = cWa + H2 * na, *cWq = cba + H2;
    const float cbq = cWq[H2];
    const float *ag2 = at, *abe2 = at + H2, *aWmu = at + 2 * H2, *abmu = aWmu + na * H2;

    float xh[C], y[C], h2[C], rs;
    ln_affine<C>(za2, ag2, abe2, H2, lane, xh, y, rs);
#pragma unroll
    for (int c = 0; c < C; ++c) h2[c] = relu(y[c]);
    float mu[kMaxAct];
#pragma unroll
    for (int o = 0; o < kMaxAct; ++o) {
        mu[o] = 0.0f;
        if (o >= na) continue;
        float p = 0.0f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int j = lane + 64 * c;
            if (j < H2) p = fmaf(h2[c], aWmu[o * H2 + j], p);
        }
        mu[o] = tanhf(wave_sum(p) + abmu[o]);
    }
    float cxh[C], cy[C], crs;
    ln_affine<C>(zc2, cg2, cbe2, H2, lane, cxh, cy, crs);
    float za[C], u[C], qp = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        za[c] = 0.0f;
        u[c] = 0.0f;
        if (j < H2) {
            float acc = 0.0f;
#pragma unroll
            for (int o = 0; o < kMaxAct; ++o)
                if (o < na) acc = fmaf(mu[o], cWa[j * na + o], acc);
            za[c] = acc + cba[j];
            u[c] = cy[c] + relu(za[c]);
            qp = fmaf(cWq[j], relu(u[c]), qp);
        }
    }
    const float Q = wave_sum(qp) + cbq;
    if (lane == 0) w.ALOSS[r] = -Q;
    const float dQ = -a.invB;  // d/dQ mean(-Q)                                                         (:147-149)
    float dmu_p[kMaxAct];
#pragma unroll
    for (int o = 0; o < kMaxAct; ++o) dmu_p[o] = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        if (j < H2) {
            const float du = u[c] > 0.0f ? dQ * cWq[j] : 0.0f;
            const float dza = za[c] > 0.0f ? du : 0.0f;
#pragma unroll
            for (int o = 0; o < kMaxAct; ++o)
                if (o < na) dmu_p[o] = fmaf(cWa[j * na + o], dza, dmu_p[o]);
        }
    }
    float dm[kMaxAct];
#pragma unroll
    for (int o = 0; o < kMaxAct; ++o) {
        dm[o] = 0.0f;
        if (o >= na) continue;
        dm[o] = wave_sum(dmu_p[o]) * (1.0f - mu[o] * mu[o]);  // tanh backward
        if (lane == 0) w.DM[(int64_t)r * na + o] = dm[o];
    }
    float dy2[C], dz2[C], g2[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        float dh = 0.0f;
        g2[c] = 0.0f;
        if (j < H2) {
#pragma unroll
            for (int o = 0; o < kMaxAct; ++o)
                if (o < na) dh = fmaf(aWmu[o * H2 + j], dm[o], dh);
            g2[c] = ag2[j];
        }
        dy2[c] = h2[c] > 0.0f ? dh : 0.0f;
    }
    ln_backward<C>(dy2, xh, g2, rs, H2, dz2);
    store_row<C>(w.AXH2 + ro, xh, H2, lane);
    store_row<C>(w.AH2 + ro, h2, H2, lane);
    store_row<C>(w.ADY2 + ro, dy2, H2, lane);
    store_row<C>(w.ADZ2 + ro, dz2, H2, lane);
    if (lane == 0) w.ARS2[r] = rs;
}

// Merged row kernels of a learn() round (launch_round): the critic-phase job of one learn() and the actor-phase job of
// the previous one in ONE launch, picked by a block-uniform branch (either job may be absent: npc / nbc = 0, or no
// blocks past them).
template <int C>
__global__ __launch_bounds__(256) void sc_k1(Ws wc, RowArgs ac, int npc, Ws wa, RowArgs aa) {
    if ((int)blockIdx.y < npc)
        c1_body<C>(wc, ac, blockIdx.x, blockIdx.y);
    else
        a1_body<C>(wa, aa, blockIdx.x, blockIdx.y - npc);
}
template <int C>
__global__ __launch_bounds__(256) void sc_k3(Ws wc, RowArgs ac, int nbc, Ws wa, RowArgs aa) {
    if ((int)blockIdx.x < nbc)
        c3_body<C>(wc, ac, blockIdx.x);
    else
        a3_body<C>(wa, aa, blockIdx.x - nbc);
}
template <int C>
__global__ __launch_bounds__(256) void sc_ln1_bwd(Ln1Args l0, int nb0, Ln1Args l1) {
    if ((int)blockIdx.x < nb0)
        ln1_body<C>(l0, blockIdx.x);
    else
        ln1_body<C>(l1, blockIdx.x - nb0);
}

// ---------------------------------------------------------------------------------------------------------------
// f32 GEMM tile on MFMA: C[m, n] = sum_k A(m, k) B(k, n) for one 32x32 output tile; A(m, k) = A[m*sam + k*sak],
// B(k, n) = B[k*sbk + n*sbn]. K is processed in panels of up to kKC: the 32 x kc A panel and kc x 32 B panel are
// loaded whole into LDS (P[k][r], row pitch 33) in one round, the 4 waves each run v_mfma_f32_32x32x2_f32 over a
// quarter of the panel, and the 4 partial tiles are summed in a fixed order. Panel loaders are specialised on the
// operand layout (host-checked): 0 = k contiguous (float4 along k), 1 = rows contiguous (float4 along the rows),
// 2 = any strides (scalar).
constexpr int kT = 32;
constexpr int kKC = 512;
constexpr int kFwdKC = 200;   // forward / input-gradient GEMM K chunk (FLOCK_GEMM_KC overrides): 0.098 ms per config-3
                              // step vs 0.117 with whole 400-deep panels (lighter blocks co-run with the env kernel)
constexpr int kGradKC = 128;  // the gradient kernels share one launch with ~400 LDS-free reduction blocks: a 34-KB
                              // panel keeps 4 blocks per CU resident so the whole grid runs in one round
constexpr int kPitch = 33;
struct GemmP {
    const float* A;
    const float* B;
    float* C;
    const float* bias;
    int M, N, K, sam, sak, sbk, sbn, ldc;
    int64_t relB;  // B and bias are agent-relative: + relB * (*agent)
    const int64_t* agent;
    int tiles_n, tiles;
    int kchunk;  // K panel depth staged per round (<= kKC, multiple of 8)
};
constexpr int kMaxBatch = 5;  // a round's forward GEMMs: 3 (critic phase) + 2 (actor phase)
struct GemmBatch {
    GemmP p[kMaxBatch];
    int n;
};

__host__ __device__ inline int gemm_kc(int K, int chunk = kKC) {
    const int k = K < chunk ? K : chunk;
    return (k + 7) & ~7;
}
// A and B panels; the 4 partial tiles (4 x 16 x 64 floats) reuse the panel space once the MFMAs are done
__host__ __device__ inline size_t gemm_lds_bytes(int K, int chunk = kKC) {
    const int panels = 2 * gemm_kc(K, chunk) * kPitch, red = 4 * 16 * 64;
    return (size_t)(panels > red ? panels : red) * sizeof(float);
}

// P[kk][rr] = X(r0 + rr, k0 + kk) for rr < 32, kk < kc (zero outside R x Kd); X(r, k) = X[r*sr + k*sk]
template <int V>
__device__ __forceinline__ void load_panel(float* __restrict__ P, const float* __restrict__ X, int R, int Kd, int sr,
                                           int sk, int r0, int k0, int kc) {
    const int tid = threadIdx.x;
    if (V == 0) {  // k contiguous: float4 along k; item t -> row t / (kc/4), k-quad t % (kc/4)
        const int q = kc >> 2, items = 32 * q;
        for (int base = 0; base < items; base += 256 * 16) {
            float4 v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = base + tid + 256 * i;
                const int rr = t / q, k = k0 + 4 * (t - rr * q), rw = r0 + rr;
                v[i] = (t < items && rw < R && k < Kd) ? *reinterpret_cast<const float4*>(X + (int64_t)rw * sr + k)
                                                       : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = base + tid + 256 * i;
                if (t < items) {
                    const int rr = t / q, kk = 4 * (t - rr * q);
                    P[(kk + 0) * kPitch + rr] = v[i].x;
                    P[(kk + 1) * kPitch + rr] = v[i].y;
                    P[(kk + 2) * kPitch + rr] = v[i].z;
                    P[(kk + 3) * kPitch + rr] = v[i].w;
                }
            }
        }
    } else if (V == 1) {  // rows contiguous: float4 along r; item t -> k t / 8, row-quad t % 8
        const int items = 8 * kc;
        for (int base = 0; base < items; base += 256 * 16) {
            float4 v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = base + tid + 256 * i;
                const int kk = t >> 3, rr = 4 * (t & 7), k = k0 + kk, rw = r0 + rr;
                v[i] = (t < items && rw < R && k < Kd) ? *reinterpret_cast<const float4*>(X + (int64_t)k * sk + rw)
                                                       : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = base + tid + 256 * i;
                if (t < items) {
                    const int kk = t >> 3, rr = 4 * (t & 7);
                    float* d = P + kk * kPitch + rr;
                    d[0] = v[i].x;
                    d[1] = v[i].y;
                    d[2] = v[i].z;
                    d[3] = v[i].w;
                }
            }
        }
    } else {
        const int items = 32 * kc;
        for (int base = 0; base < items; base += 256 * 16) {
            float v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = base + tid + 256 * i;
                const int kk = t >> 5, rr = t & 31, k = k0 + kk, rw = r0 + rr;
                v[i] = (t < items && rw < R && k < Kd) ? X[(int64_t)rw * sr + (int64_t)k * sk] : 0.0f;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int t = base + tid + 256 * i;
                if (t < items) P[(t >> 5) * kPitch + (t & 31)] = v[i];
            }
        }
    }
}

// Split panel load for the vectorised layouts (V = 0, 1: one round of at most 16 float4 per thread, kc <= 512):
// panel_fetch issues the global loads into registers, panel_store writes them to LDS. gemm_tile fetches the A and
// B panels of a chunk together (one memory round trip instead of two) and the next chunk's panels before the
// current chunk's MFMAs.
template <int V, int NF>
__device__ __forceinline__ void panel_fetch(float4 (&v)[NF], const float* __restrict__ X, int R, int Kd, int sr,
                                            int sk, int r0, int k0, int kc) {
    const int tid = threadIdx.x;
    if (V == 0) {
        const int q = kc >> 2, items = 32 * q;
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int t = tid + 256 * i;
            const int rr = t / q, k = k0 + 4 * (t - rr * q), rw = r0 + rr;
            v[i] = (t < items && rw < R && k < Kd) ? *reinterpret_cast<const float4*>(X + (int64_t)rw * sr + k)
                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    } else {
        const int items = 8 * kc;
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int t = tid + 256 * i;
            const int kk = t >> 3, rr = 4 * (t & 7), k = k0 + kk, rw = r0 + rr;
            v[i] = (t < items && rw < R && k < Kd) ? *reinterpret_cast<const float4*>(X + (int64_t)k * sk + rw)
                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}
template <int V, int NF>
__device__ __forceinline__ void panel_store(float* __restrict__ P, const float4 (&v)[NF], int kc) {
    const int tid = threadIdx.x;
    if (V == 0) {
        const int q = kc >> 2, items = 32 * q;
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int t = tid + 256 * i;
            if (t < items) {
                const int rr = t / q, kk = 4 * (t - rr * q);
                P[(kk + 0) * kPitch + rr] = v[i].x;
                P[(kk + 1) * kPitch + rr] = v[i].y;
                P[(kk + 2) * kPitch + rr] = v[i].z;
                P[(kk + 3) * kPitch + rr] = v[i].w;
            }
        }
    } else {
        const int items = 8 * kc;
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int t = tid + 256 * i;
            if (t < items) {
                const int kk = t >> 3, rr = 4 * (t & 7);
                float* d = P + kk * kPitch + rr;
                d[0] = v[i].x;
                d[1] = v[i].y;
                d[2] = v[i].z;
                d[3] = v[i].w;
            }
        }
    }
}

// acc += the wave's K slice of the staged panels: operand k of MFMA kk/2 is a[kk * kPitch] / b[kk * kPitch]. The
// LDS reads of 8 MFMAs are issued together, so the loop pays one LDS latency per 8 MFMAs instead of one per MFMA;
// the accumulation order (and so every bit of the result) is the plain loop's.
__device__ __forceinline__ f32x16 mfma_panel(f32x16 acc, const float* a, const float* b, int kq) {
    int kk = 0;
    for (; kk + 16 <= kq; kk += 16) {
        float av[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            av[u] = a[(kk + 2 * u) * kPitch];
            bv[u] = b[(kk + 2 * u) * kPitch];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
    }
    for (; kk < kq; kk += 2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk * kPitch], b[kk * kPitch], acc, 0, 0, 0);
    return acc;
}

// the 4 outputs of thread (wave w, lane l): rows 8w + 4(l >> 5) + q (q < 4), column l & 31
template <int AV, int BV, int NF>
__device__ __forceinline__ void gemm_tile(const GemmP& g, const float* Bp, int tm, int tn, float* smem,
                                          float (&out)[4]) {
    const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
    const int kcmax = gemm_kc(g.K, g.kchunk);
    float* As = smem;
    float* Bs = smem + kcmax * kPitch;
    float* red = smem;  // after the last panel barrier
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.0f;
    if constexpr (AV != 2 && BV != 2) {
        float4 va[NF], vb[NF];
        int kc = gemm_kc(g.K, g.kchunk);
        panel_fetch<AV, NF>(va, g.A, g.M, g.K, g.sam, g.sak, tm * kT, 0, kc);
        panel_fetch<BV, NF>(vb, Bp, g.N, g.K, g.sbn, g.sbk, tn * kT, 0, kc);
        for (int k0 = 0; k0 < g.K; k0 += g.kchunk) {
            panel_store<AV, NF>(As, va, kc);
            panel_store<BV, NF>(Bs, vb, kc);
            __syncthreads();
            const int k1 = k0 + g.kchunk, kc1 = k1 < g.K ? gemm_kc(g.K - k1, g.kchunk) : 0;
            if (k1 < g.K) {  // the next chunk's loads fly during this chunk's MFMAs
                panel_fetch<AV, NF>(va, g.A, g.M, g.K, g.sam, g.sak, tm * kT, k1, kc1);
                panel_fetch<BV, NF>(vb, Bp, g.N, g.K, g.sbn, g.sbk, tn * kT, k1, kc1);
            }
            const int kq = kc >> 2;  // multiple of 2
            const float* a = As + (wv * kq + (l >> 5)) * kPitch + (l & 31);
            const float* b = Bs + (wv * kq + (l >> 5)) * kPitch + (l & 31);
            acc = mfma_panel(acc, a, b, kq);
            __syncthreads();
            kc = kc1;
        }
    } else {
        for (int k0 = 0; k0 < g.K; k0 += g.kchunk) {
            const int kc = gemm_kc(g.K - k0, g.kchunk);
            load_panel<AV>(As, g.A, g.M, g.K, g.sam, g.sak, tm * kT, k0, kc);
            load_panel<BV>(Bs, Bp, g.N, g.K, g.sbn, g.sbk, tn * kT, k0, kc);
            __syncthreads();
            const int kq = kc >> 2;  // multiple of 2
            const float* a = As + (wv * kq + (l >> 5)) * kPitch + (l & 31);
            const float* b = Bs + (wv * kq + (l >> 5)) * kPitch + (l & 31);
            acc = mfma_panel(acc, a, b, kq);
            __syncthreads();
        }
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) red[(wv * 16 + v) * 64 + l] = acc[v];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int v = 4 * wv + q;
        out[q] = ((red[(0 * 16 + v) * 64 + l] + red[(1 * 16 + v) * 64 + l]) + red[(2 * 16 + v) * 64 + l]) +
                 red[(3 * 16 + v) * 64 + l];
    }
}

// grid (max tiles, problems): block (x, y) computes tile x of problem y
template <int AV, int BV, int NF>
__global__ __launch_bounds__(256) void sc_gemm(GemmBatch gb) {
    extern __shared__ float4 smem4[];
    float* smem = reinterpret_cast<float*>(smem4);
    const GemmP& g = gb.p[blockIdx.y];
    const int t = blockIdx.x;
    if (t >= g.tiles) return;
    const int tm = t / g.tiles_n, tn = t - tm * g.tiles_n;
    const int64_t rel = g.relB ? g.relB * (*g.agent) : 0;
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int n = tn * kT + (l & 31);
    const float bias = (g.bias && n < g.N) ? g.bias[rel + n] : 0.0f;
    float out[4];
    gemm_tile<AV, BV, NF>(g, g.B + rel, tm, tn, smem, out);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int m = tm * kT + 8 * wv + 4 * (l >> 5) + q;
        if (m < g.M && n < g.N) g.C[(int64_t)m * g.ldc + n] = g.bias ? out[q] + bias : out[q];
    }
}

// ---------------------------------------------------------------------------------------------------------------
// gradients + Adam for one network. Blocks [0, tiles): the fc2.weight gradient (a K = B GEMM) with Adam in the
// epilogue; the next blocks: reduction red[q] (the last q with red[q].blk0 <= block) over the B rows, 16 elements per
// block (16 row groups per block):
//   mode 0: g[o] = sum_b D[b, o]         (biases, LayerNorm beta)
//   mode 1: g[o] = sum_b D[b, o] X[b, o] (LayerNorm gamma)
//   mode 2: g[o*in + i] = sum_b D[b, o] X[b, i]  (fc1 / action_value / head weights)
//   mode 3: loss = sum_b D[b] / B        (written to *loss, no Adam)
struct RedP {
    const float* D;
    const float* X;
    int ldd, ldx, mode, in, n, blk0;
    int64_t off;
};
constexpr int kMaxRed = 12;
constexpr int kRedElems = 16;
constexpr int kMaxRedBlocks = 4096;
struct GradAdam {
    GemmP g;  // C unused: the gradient goes to grad + w2_off
    int64_t w2_off;
    int nred, nblk, B, do_adam;
    RedP red[kMaxRed];
    float *p, *grad, *m, *v;
    int64_t rel;  // p/grad/m/v are agent-relative: + rel * (*agent)
    const int64_t* agent;
    int64_t* step;  // step[0], or step[*agent] when rel != 0
    unsigned* counter;
    float* loss;
    float lr, b1, b2, eps;
    // soft updates after the Adam step (actor kernel): target = tau p + (1 - tau) target for every updated
    // element, and the critic's self update (critic = tau c + (1 - tau) c) in soft_blocks extra blocks
    float* target;
    float* self_soft;
    int64_t self_n;
    int soft_rate, soft_blocks;
    float tau, one_minus_tau;
    // critic kernel with a view (FlockScUpdate.critic_view): the post-Adam value also goes to p_copy, and when
    // soft_count[*agent] (this learn's count) is a multiple of soft_rate, p receives the self soft update of it
    float* p_copy;
    const int64_t* soft_count;
};

struct AdamState {
    float p, m, v, t;
};
__device__ __forceinline__ AdamState adam_load(const GradAdam& ga, int64_t i) {
    return {ga.p[i], ga.m[i], ga.v[i], ga.target ? ga.target[i] : 0.0f};
}
// torch.optim.Adam single-tensor path, identical to adam_elem (flock_learn.hip)
__device__ __forceinline__ void adam_store(const GradAdam& ga, int64_t i, AdamState s, float gi, float neg_step,
                                           float bc2s, bool soft) {
    const float w1 = (float)(1.0 - (double)ga.b1), omb2 = (float)(1.0 - (double)ga.b2);
    float mi = s.m;
    mi = (w1 < 0.5f) ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.0f - w1);
    float vi = s.v * ga.b2;
    vi = vi + (omb2 * gi) * gi;
    const float denom = __builtin_sqrtf(vi) / bc2s + ga.eps;
    const float pn = s.p + (neg_step * mi) / denom;
    if (ga.p_copy) {  // critic with a view: view = post-Adam, p = its self soft update on soft learns
        ga.p_copy[i] = pn;
        ga.p[i] = soft ? ga.tau * pn + ga.one_minus_tau * pn : pn;
    } else {
        ga.p[i] = pn;
    }
    ga.m[i] = mi;
    ga.v[i] = vi;
    if (soft && ga.target) ga.target[i] = ga.tau * pn + ga.one_minus_tau * s.t;  // soft_update_kernel mode 1
}

// one job's blocks: bx in [0, nb), nb = g.tiles + nblk + soft_blocks
template <int AV, int BV, int NF>
__device__ __forceinline__ void grad_adam_body(const GradAdam& ga, int bx, int nb) {
    extern __shared__ float4 smem4[];
    float* smem = reinterpret_cast<float*>(smem4);
    __shared__ float sh[2];
    __shared__ int sh_soft;
    const int tid = threadIdx.x;
    const int64_t agent = ga.rel ? *ga.agent : 0;
    const int64_t base = ga.rel * agent;
    if (tid == 0) {
        const int64_t step0 = ga.do_adam ? ga.step[agent] : 0;
        const int64_t count = ga.soft_count ? ga.soft_count[*ga.agent] : step0;
        sh_soft = ga.do_adam && ga.soft_rate > 0 && (count % ga.soft_rate) == 0;  // this learn's count
        if (ga.do_adam) {
            const double st = (double)(step0 + 1);
            sh[0] = (float)(-(double)ga.lr / (1.0 - pow((double)ga.b1, st)));
            sh[1] = (float)sqrt(1.0 - pow((double)ga.b2, st));
        }
    }
    if (bx >= ga.g.tiles + ga.nblk) {  // critic self soft update blocks (after its Adam step)
        __syncthreads();
        if (sh_soft && ga.self_soft) {
            const int64_t b0 = (int64_t)(bx - ga.g.tiles - ga.nblk) * 1024;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t e = b0 + q * 256 + tid;
                if (e < ga.self_n) {
                    const float c = ga.self_soft[e];
                    ga.self_soft[e] = ga.tau * c + ga.one_minus_tau * c;
                }
            }
        }
    } else if (bx < ga.g.tiles) {
        {
            const int tm = bx / ga.g.tiles_n, tn = bx - tm * ga.g.tiles_n;
            const int wv = tid >> 6, l = tid & 63;
            const int nn = tn * kT + (l & 31);
            AdamState st[4];
            int64_t e[4];
            bool ok[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // prefetch the Adam state of this thread's 4 outputs
                const int mm = tm * kT + 8 * wv + 4 * (l >> 5) + q;
                ok[q] = mm < ga.g.M && nn < ga.g.N;
                e[q] = base + ga.w2_off + (int64_t)mm * ga.g.ldc + nn;
                st[q] = (ok[q] && ga.do_adam) ? adam_load(ga, e[q]) : AdamState{0.f, 0.f, 0.f, 0.f};
            }
            float out[4];
            gemm_tile<AV, BV, NF>(ga.g, ga.g.B, tm, tn, smem, out);  // (its barriers also publish sh[])
            const float neg_step = sh[0], bc2s = sh[1];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (ok[q]) {
                    ga.grad[e[q]] = out[q];
                    if (ga.do_adam) adam_store(ga, e[q], st[q], out[q], neg_step, bc2s, sh_soft != 0);
                }
        }
    } else {
        float* part = smem;  // [16 row groups][16 elements]
        const int b = bx - ga.g.tiles;
        int q0 = 0;  // descriptor of this block: a wave-uniform search over <= kMaxRed scalars
        for (int q = 1; q < ga.nred; ++q)
            if (b >= ga.red[q].blk0) q0 = q;
        const RedP& rp = ga.red[q0];
        const int el = tid & (kRedElems - 1), q = tid >> 4;
        const int e = (b - rp.blk0) * kRedElems + el;
        const bool live = e < rp.n;
        const int o = rp.mode == 2 ? e / rp.in : e;
        const int i = rp.mode == 2 ? e - o * rp.in : e;
        const bool prod = rp.mode == 1 || rp.mode == 2;
        const int64_t pe = base + rp.off + e;
        const AdamState st = (q == 0 && live && rp.mode != 3 && ga.do_adam) ? adam_load(ga, pe)
                                                                              : AdamState{0.f, 0.f, 0.f, 0.f};
        float acc = 0.0f;
        for (int r0 = q; r0 < ga.B; r0 += 16 * 16) {
            float dv[16], xv[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int r = r0 + 16 * k;
                const bool in = live && r < ga.B;
                dv[k] = in ? rp.D[(int64_t)r * rp.ldd + o] : 0.0f;
                xv[k] = (in && prod) ? rp.X[(int64_t)r * rp.ldx + i] : 0.0f;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) acc = prod ? fmaf(dv[k], xv[k], acc) : acc + dv[k];
        }
        part[q * kRedElems + el] = acc;
        __syncthreads();
        if (q == 0 && live) {
            float gsum = 0.0f;
#pragma unroll
            for (int k = 0; k < 16; ++k) gsum += part[k * kRedElems + el];
            if (rp.mode == 3) {
                *ga.loss = gsum * (1.0f / (float)ga.B);
            } else {
                ga.grad[pe] = gsum;
                if (ga.do_adam) adam_store(ga, pe, st, gsum, sh[0], sh[1], sh_soft != 0);
            }
        }
    }
    // the last block to arrive advances the step counter. No fence: every block's thread 0 consumed its load of
    // *step (the bias corrections) before its relaxed atomic add, and the increment only has to be visible to the
    // NEXT launch (kernel boundary). A device-scope fence here costs an L2 writeback per block on gfx950.
    if (ga.do_adam && tid == 0) {
        const unsigned prev = atomicAdd(ga.counter, 1u);
        if (prev == (unsigned)nb - 1u) {
            ga.step[agent] += 1;
            *ga.counter = 0u;
        }
    }
}

// a round's gradient + Adam launch: blocks [0, nb0) run job j0, the rest job j1 (when there are any)
struct GradAdam2 {
    GradAdam j0, j1;
    int nb0;
};
template <int AV, int BV, int NF>
__global__ __launch_bounds__(256) void sc_grad_adam(GradAdam2 gg) {
    if ((int)blockIdx.x < gg.nb0)
        grad_adam_body<AV, BV, NF>(gg.j0, blockIdx.x, gg.nb0);
    else
        grad_adam_body<AV, BV, NF>(gg.j1, blockIdx.x - gg.nb0, gridDim.x - gg.nb0);
}

// ---------------------------------------------------------------------------------------------------------------
// host side
// K-panel depth of the forward / input-gradient GEMMs: whole panels (kKC) by default; FLOCK_GEMM_KC (a multiple
// of 8 in [8, 512]) stages them in chunks (smaller LDS footprint per block; A/B diagnostics)
int kc_knob(const char* name, int dflt) {
    const char* e = getenv(name);
    const int v = e ? atoi(e) : 0;
    return (v >= 8 && v <= kKC && (v & 7) == 0) ? v : dflt;
}
int fwd_kc() {
    static const int kc = kc_knob("FLOCK_GEMM_KC", kFwdKC);
    return kc;
}
int grad_kc() {
    static const int kc = kc_knob("FLOCK_GRAD_KC", kGradKC);
    return kc;
}
// K chunk for a K-deep GEMM with at most kcmax per chunk: the chunks balanced, a multiple of 8
int balanced_kc(int K, int kcmax) {
    const int n = (K + kcmax - 1) / kcmax;
    const int kc = ((K + n - 1) / n + 7) & ~7;
    return kc < kcmax ? kc : kcmax;
}
// float4 registers per thread per operand of a chunk (kc <= 32 NF): the instantiated depths
int nf_of(int kc) { return kc <= 128 ? 4 : kc <= 224 ? 7 : kc <= 320 ? 10 : 16; }

GemmP gemm_p(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int sam, int sak,
             int sbk, int sbn, int ldc, int64_t relB, const int64_t* agent = nullptr) {
    GemmP g;
    g.A = A; g.B = B; g.C = C; g.bias = bias;
    g.M = M; g.N = N; g.K = K; g.sam = sam; g.sak = sak; g.sbk = sbk; g.sbn = sbn; g.ldc = ldc; g.relB = relB;
    g.agent = agent;
    g.tiles_n = (N + kT - 1) / kT;
    g.tiles = ((M + kT - 1) / kT) * g.tiles_n;
    g.kchunk = balanced_kc(K, fwd_kc());
    return g;
}

// panel-loader variant for an operand X(r, k) = X[r*sr + k*sk] with R rows (see load_panel); rel: agent stride
bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
int panel_variant(const float* X, int R, int K, int sr, int sk, int64_t rel) {
    if (!al16(X) || (rel & 3)) return 2;
    if (sk == 1 && (K & 3) == 0 && (sr & 3) == 0) return 0;
    if (sr == 1 && (R & 3) == 0 && (sk & 3) == 0) return 1;
    return 2;
}
int gemm_variant(const GemmP& g) {  // 0: (0,0)  1: (0,1)  2: (1,1)  3: (2,2)
    const int a = panel_variant(g.A, g.M, g.K, g.sam, g.sak, 0);
    const int b = panel_variant(g.B, g.N, g.K, g.sbn, g.sbk, g.relB);
    if (a == 0 && b == 0) return 0;
    if (a == 0 && b == 1) return 1;
    if (a == 1 && b == 1) return 2;
    return 3;
}

template <typename F>
int allow_lds(F* kernel, size_t bytes) {
    if (bytes > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes) != hipSuccess)
        return fail(-4, "flock_sc: cannot raise the dynamic LDS limit");
    return 0;
}

template <int AV, int BV, int NF>
int launch_gemm_v(hipStream_t st, const GemmBatch& gb, dim3 grid, size_t lds) {
    if (int rc = allow_lds(sc_gemm<AV, BV, NF>, lds)) return rc;
    hipLaunchKernelGGL((sc_gemm<AV, BV, NF>), grid, dim3(256), lds, st, gb);
    return launched();
}
template <int AV, int BV>
int launch_gemm_nf(hipStream_t st, const GemmBatch& gb, dim3 grid, size_t lds, int nf) {
    switch (nf) {
        case 4: return launch_gemm_v<AV, BV, 4>(st, gb, grid, lds);
        case 7: return launch_gemm_v<AV, BV, 7>(st, gb, grid, lds);
        case 10: return launch_gemm_v<AV, BV, 10>(st, gb, grid, lds);
        default: return launch_gemm_v<AV, BV, 16>(st, gb, grid, lds);
    }
}

int launch_gemm(hipStream_t st, const GemmBatch& gb) {
    int K = 0, kc = 8, tiles = 0, var = gemm_variant(gb.p[0]);
    for (int i = 0; i < gb.n; ++i) {
        K = gb.p[i].K > K ? gb.p[i].K : K;
        const int c = gemm_kc(gb.p[i].K, gb.p[i].kchunk);
        kc = c > kc ? c : kc;
        tiles = gb.p[i].tiles > tiles ? gb.p[i].tiles : tiles;
        if (gemm_variant(gb.p[i]) != var) var = 3;
    }
    const dim3 grid(tiles, gb.n);
    const size_t lds = gemm_lds_bytes(kc, kc);
    const int nf = nf_of(kc);
    switch (var) {
        case 0: return launch_gemm_nf<0, 0>(st, gb, grid, lds, nf);
        case 1: return launch_gemm_nf<0, 1>(st, gb, grid, lds, nf);
        case 2: return launch_gemm_nf<1, 1>(st, gb, grid, lds, nf);
        default: return launch_gemm_v<2, 2, 16>(st, gb, grid, lds);
    }
}

void add_red(GradAdam& ga, const float* D, int ldd, const float* X, int ldx, int mode, int in, int n, int64_t off) {
    const int j = ga.nred++;
    RedP& r = ga.red[j];
    r.D = D; r.X = X; r.ldd = ldd; r.ldx = ldx; r.mode = mode; r.in = in; r.n = n; r.off = off;
    r.blk0 = ga.nblk;
    ga.nblk += (n + kRedElems - 1) / kRedElems;
}
int grad_blocks(const GradAdam& ga) { return ga.g.tiles + ga.nblk + ga.soft_blocks; }
size_t grad_lds(const GradAdam& ga) {
    const size_t lds = gemm_lds_bytes(ga.g.K, ga.g.kchunk);
    return lds < 16 * kRedElems * sizeof(float) ? 16 * kRedElems * sizeof(float) : lds;
}

template <int AV, int BV, int NF>
int launch_grad_adam_v(hipStream_t st, const GradAdam2& gg, dim3 grid, size_t lds) {
    if (int rc = allow_lds(sc_grad_adam<AV, BV, NF>, lds)) return rc;
    hipLaunchKernelGGL((sc_grad_adam<AV, BV, NF>), grid, dim3(256), lds, st, gg);
    return launched();
}

int check(const FlockScUpdate* u) {
    if (!u) return fail(-3, "flock_sc: NULL argument");
    if (u->B < 1 || u->in_dim < 1 || u->n_actions < 1 || u->fc1 < 1 || u->fc2 < 1)
        return fail(-5, "flock_sc: sizes must be >= 1");
    if (u->in_dim > kMaxIn || u->n_actions > kMaxAct || u->fc1 > kMaxFeat || u->fc2 > kMaxFeat ||
        u->fc1 * (u->in_dim + 3) > kMaxFc1Block)
        return fail(-2, "flock_sc: in_dim <= 64, n_actions <= 4, fc1/fc2 <= 1024, fc1 * (in_dim + 3) <= 32768");
    if (!u->idx || !u->agent || !u->ring_state || !u->ring_new_state || !u->ring_action || !u->ring_reward ||
        !u->ring_terminal || !u->critic || !u->critic_grad || !u->actors || !u->actors_grad || !u->actors_target ||
        !u->losses || !u->workspace || !u->counters)
        return fail(-3, "flock_sc: NULL pointer");
    if (u->do_adam && (!u->critic_exp_avg || !u->critic_exp_avg_sq || !u->critic_step || !u->actors_exp_avg ||
                       !u->actors_exp_avg_sq || !u->actor_steps))
        return fail(-3, "flock_sc: NULL optimizer state");
    const ActorOff ao = actor_off(u->in_dim, u->n_actions, u->fc1, u->fc2);
    if (u->actor_stride < ao.total) return fail(-5, "flock_sc: actor_stride smaller than one actor");
    return 0;
}

int chunks(const FlockScUpdate* u) {
    const int F = u->fc1 > u->fc2 ? u->fc1 : u->fc2;
    const int c = (F + 63) / 64;
    return c <= 1 ? 1 : c <= 2 ? 2 : c <= 4 ? 4 : c <= 8 ? 8 : 16;
}

RowArgs row_args(const FlockScUpdate* u) {
    RowArgs a;
    a.B = u->B; a.in = u->in_dim; a.na = u->n_actions; a.H1 = u->fc1; a.H2 = u->fc2;
    a.idx = u->idx; a.agent = u->agent;
    a.rs = u->ring_state; a.rs2 = u->ring_new_state; a.ra = u->ring_action; a.rr = u->ring_reward;
    a.rt = u->ring_terminal;
    a.critic = u->critic; a.actors = u->actors; a.actors_target = u->actors_target; a.stride = u->actor_stride;
    a.gamma = u->gamma;
    a.invB = 1.0f / (float)u->B;
    return a;
}

size_t fc1_lds(int in, int H1) { return (size_t)(kRowsPerBlock * kMaxIn + round4(H1 * (in + 3))) * sizeof(float); }

size_t tails_lds(int na, int H2) {
    return (size_t)(round4(crit_tail_len(na, H2)) + round4(act_tail_len(na, H2))) * sizeof(float);
}

// One phase of one learn() as the arguments of the six launches of a round (launch_round):
//   1 rows: fc1 + LN + ReLU (critic c1: 3 paths, actor a1: 2 paths)   2 forward fc2 GEMMs (critic 3, actor 2)
//   3 rows: heads, losses, backward to the fc2 pre-activation (c3 / a3)   4 dH1 = dZ2 W2 GEMM
//   5 ReLU + LN1 backward   6 gradient + Adam (+ soft updates)
struct Job {
    Ws w;
    RowArgs a;
    int C, rb, B, in, na, H1, H2;
    size_t lds1, lds3;
    GemmP fwd[3];
    int nfwd;
    GemmP dh;
    Ln1Args l;
    GradAdam ga;
};

void job_common(const FlockScUpdate* u, Job& j) {
    j.B = u->B; j.in = u->in_dim; j.na = u->n_actions; j.H1 = u->fc1; j.H2 = u->fc2;
    ws_layout(j.B, j.in, j.na, j.H1, j.H2, u->workspace, &j.w);
    j.a = row_args(u);
    j.C = chunks(u);
    j.rb = (j.B + kRowsPerBlock - 1) / kRowsPerBlock;
    j.lds1 = fc1_lds(j.in, j.H1);
    j.lds3 = tails_lds(j.na, j.H2);
}

// critic phase (agent_simple_shared_critic.py:118-141)
void critic_job(const FlockScUpdate* u, Job& j) {
    job_common(u, j);
    const int B = j.B, in = j.in, na = j.na, H1 = j.H1, H2 = j.H2;
    const Ws& w = j.w;
    const CriticOff co = critic_off(in, na, H1, H2);
    const ActorOff ao = actor_off(in, na, H1, H2);
    // fc2 of target actor(s'), critic(s'), critic(s)
    j.fwd[0] = gemm_p(w.TH1, u->actors_target + ao.W2, w.Z2, u->actors_target + ao.b2, B, H2, H1, H1, 1, 1, H1, H2,
                      u->actor_stride, u->agent);
    j.fwd[1] = gemm_p(w.NH1, u->critic + co.W2, w.Z2 + (int64_t)B * H2, u->critic + co.b2, B, H2, H1, H1, 1, 1, H1,
                      H2, 0);
    j.fwd[2] = gemm_p(w.H1, u->critic + co.W2, w.Z2 + 2 * (int64_t)B * H2, u->critic + co.b2, B, H2, H1, H1, 1, 1,
                      H1, H2, 0);
    j.nfwd = 3;
    j.dh = gemm_p(w.DZ2, u->critic + co.W2, w.DH1, nullptr, B, H1, H2, H2, 1, H1, 1, H1, 0);  // dH1 = dZ2 W2
    j.l = Ln1Args{B, H1, w.DH1, w.XH1, w.RS1, w.H1, u->critic + co.g1, nullptr, 0, w.DY1, w.DZ1};
    GradAdam& ga = j.ga;
    ga.g = gemm_p(w.DZ2, w.H1, nullptr, nullptr, H2, H1, B, 1, H2, H1, 1, H1, 0);  // dW2 = dZ2^T H1
    ga.g.kchunk = balanced_kc(B, grad_kc());
    ga.w2_off = co.W2;
    ga.nred = 0;
    ga.nblk = 0;
    ga.B = B;
    ga.do_adam = u->do_adam;
    add_red(ga, w.DZ1, H1, w.S, in, 2, in, H1 * in, co.W1);
    add_red(ga, w.DZ1, H1, nullptr, 0, 0, 1, H1, co.b1);
    add_red(ga, w.DY1, H1, w.XH1, H1, 1, 1, H1, co.g1);
    add_red(ga, w.DY1, H1, nullptr, 0, 0, 1, H1, co.be1);
    add_red(ga, w.DZ2, H2, nullptr, 0, 0, 1, H2, co.b2);
    add_red(ga, w.DY2, H2, w.XH2, H2, 1, 1, H2, co.g2);
    add_red(ga, w.DY2, H2, nullptr, 0, 0, 1, H2, co.be2);
    add_red(ga, w.DZA, H2, w.A, na, 2, na, H2 * na, co.Wa);
    add_red(ga, w.DZA, H2, nullptr, 0, 0, 1, H2, co.ba);
    add_red(ga, w.DQ, 1, w.HQ, H2, 2, H2, H2, co.Wq);
    add_red(ga, w.DQ, 1, nullptr, 0, 0, 1, 1, co.bq);
    add_red(ga, w.LOSS, 1, nullptr, 0, 3, 1, 1, 0);
    ga.p = u->critic; ga.grad = u->critic_grad; ga.m = u->critic_exp_avg; ga.v = u->critic_exp_avg_sq;
    ga.rel = 0;
    ga.agent = u->agent;
    ga.step = u->critic_step;
    ga.counter = u->counters;
    ga.loss = u->losses + 1;
    ga.lr = u->beta; ga.b1 = u->beta1; ga.b2 = u->beta2; ga.eps = u->eps;
    ga.target = nullptr; ga.self_soft = nullptr; ga.self_n = 0; ga.soft_blocks = 0;
    // with a critic view the self soft update of this learn() rides in the critic's Adam (see FlockScUpdate)
    const bool view = u->do_adam && u->critic_view;
    ga.p_copy = view ? u->critic_view : nullptr;
    ga.soft_count = view ? u->actor_steps : nullptr;
    ga.soft_rate = view ? u->update_rate : 0;
    ga.tau = u->tau;
    ga.one_minus_tau = (float)(1.0 - (double)u->tau);
}

// actor phase (:144-150), through the UPDATED critic (critic_view when given)
void actor_job(const FlockScUpdate* u, Job& j) {
    job_common(u, j);
    const int B = j.B, in = j.in, na = j.na, H1 = j.H1, H2 = j.H2;
    const Ws& w = j.w;
    const bool view = u->do_adam && u->critic_view;
    float* const critic = view ? u->critic_view : u->critic;  // the critic this actor step sees (post-Adam)
    j.a.critic = critic;
    const CriticOff co = critic_off(in, na, H1, H2);
    const ActorOff ao = actor_off(in, na, H1, H2);
    // fc2 of the actor and of the updated critic
    j.fwd[0] = gemm_p(w.AH1, u->actors + ao.W2, w.Z2b, u->actors + ao.b2, B, H2, H1, H1, 1, 1, H1, H2,
                      u->actor_stride, u->agent);
    j.fwd[1] = gemm_p(w.CH1, critic + co.W2, w.Z2b + (int64_t)B * H2, critic + co.b2, B, H2, H1, H1, 1, 1, H1, H2,
                      0);
    j.nfwd = 2;
    j.dh = gemm_p(w.ADZ2, u->actors + ao.W2, w.ADH1, nullptr, B, H1, H2, H2, 1, H1, 1, H1, u->actor_stride,
                  u->agent);  // dH1 = dZ2 W2 (actor)
    j.l = Ln1Args{B, H1, w.ADH1, w.AXH1, w.ARS1, w.AH1, u->actors + ao.g1, u->agent, u->actor_stride, w.ADY1,
                  w.ADZ1};
    GradAdam& ga = j.ga;
    ga.g = gemm_p(w.ADZ2, w.AH1, nullptr, nullptr, H2, H1, B, 1, H2, H1, 1, H1, 0);
    ga.g.kchunk = balanced_kc(B, grad_kc());
    ga.w2_off = ao.W2;
    ga.nred = 0;
    ga.nblk = 0;
    ga.B = B;
    ga.do_adam = u->do_adam;
    add_red(ga, w.ADZ1, H1, w.S, in, 2, in, H1 * in, ao.W1);
    add_red(ga, w.ADZ1, H1, nullptr, 0, 0, 1, H1, ao.b1);
    add_red(ga, w.ADY1, H1, w.AXH1, H1, 1, 1, H1, ao.g1);
    add_red(ga, w.ADY1, H1, nullptr, 0, 0, 1, H1, ao.be1);
    add_red(ga, w.ADZ2, H2, nullptr, 0, 0, 1, H2, ao.b2);
    add_red(ga, w.ADY2, H2, w.AXH2, H2, 1, 1, H2, ao.g2);
    add_red(ga, w.ADY2, H2, nullptr, 0, 0, 1, H2, ao.be2);
    add_red(ga, w.DM, na, w.AH2, H2, 2, H2, na * H2, ao.Wmu);
    add_red(ga, w.DM, na, nullptr, 0, 0, 1, na, ao.bmu);
    add_red(ga, w.ALOSS, 1, nullptr, 0, 3, 1, 1, 0);
    ga.p = u->actors; ga.grad = u->actors_grad; ga.m = u->actors_exp_avg; ga.v = u->actors_exp_avg_sq;
    ga.rel = u->actor_stride;
    ga.agent = u->agent;
    ga.step = u->actor_steps;
    ga.counter = u->counters + 1;
    ga.loss = u->losses;
    ga.lr = u->alpha; ga.b1 = u->beta1; ga.b2 = u->beta2; ga.eps = u->eps;
    const bool soft = u->do_adam && u->update_rate > 0;
    ga.soft_rate = soft ? u->update_rate : 0;
    ga.target = soft ? u->actors_target : nullptr;  // agent-relative like p
    ga.self_soft = (soft && !view) ? u->critic : nullptr;  // with a view the critic kernel did it
    ga.self_n = co.total;
    ga.soft_blocks = (soft && !view) ? (int)((co.total + 1023) / 1024) : 0;
    ga.tau = u->tau;
    ga.one_minus_tau = (float)(1.0 - (double)u->tau);
    ga.p_copy = nullptr;
    ga.soft_count = nullptr;
}

// the C (features per lane / 64) instantiation of a row kernel launch
#define SC_C_SWITCH(C, ...)                  \
    switch (C) {                             \
        case 1: {                            \
            constexpr int CC = 1;            \
            __VA_ARGS__;                     \
        } break;                             \
        case 2: {                            \
            constexpr int CC = 2;            \
            __VA_ARGS__;                     \
        } break;                             \
        case 4: {                            \
            constexpr int CC = 4;            \
            __VA_ARGS__;                     \
        } break;                             \
        case 8: {                            \
            constexpr int CC = 8;            \
            __VA_ARGS__;                     \
        } break;                             \
        default: {                           \
            constexpr int CC = 16;           \
            __VA_ARGS__;                     \
        } break;                             \
    }

size_t zmax(size_t a, size_t b) { return a > b ? a : b; }

// One round: the critic phase of one learn() (jc) and the actor phase of another (ja) in six launches; either may be
// NULL. The two jobs share no written state when they are of different agents (the caller's guarantee), so the round
// computes exactly what the actor phase followed by the critic phase would.
int launch_round(hipStream_t st, const Job* jc, const Job* ja) {
    const Job& A = jc ? *jc : *ja;  // the first job (placeholder arguments for an absent one)
    const Job& Z = ja ? *ja : *jc;
    if (jc && ja && (jc->B != ja->B || jc->in != ja->in || jc->na != ja->na || jc->H1 != ja->H1 || jc->H2 != ja->H2))
        return fail(-5, "flock_sc_round: the two updates must have the same shapes");
    const int C = A.C, rb = A.rb;
    int rc = 0;
    {  // 1: fc1 rows
        const int npc = jc ? 3 : 0, npa = ja ? 2 : 0;
        const size_t lds = zmax(A.lds1, Z.lds1);
        const dim3 grid(rb, npc + npa);
        SC_C_SWITCH(C, if ((rc = allow_lds(sc_k1<CC>, lds))) return rc;
                    hipLaunchKernelGGL(sc_k1<CC>, grid, dim3(256), lds, st, A.w, A.a, npc, Z.w, Z.a))
        if ((rc = launched())) return rc;
    }
    {  // 2: forward fc2 GEMMs
        GemmBatch gb;
        gb.n = 0;
        if (jc)
            for (int i = 0; i < jc->nfwd; ++i) gb.p[gb.n++] = jc->fwd[i];
        if (ja)
            for (int i = 0; i < ja->nfwd; ++i) gb.p[gb.n++] = ja->fwd[i];
        if ((rc = launch_gemm(st, gb))) return rc;
    }
    {  // 3: heads, losses, backward to the fc2 pre-activation
        const int nbc = jc ? rb : 0;
        const size_t lds = zmax(A.lds3, Z.lds3);
        const dim3 grid(nbc + (ja ? rb : 0));
        SC_C_SWITCH(C, if ((rc = allow_lds(sc_k3<CC>, lds))) return rc;
                    hipLaunchKernelGGL(sc_k3<CC>, grid, dim3(256), lds, st, A.w, A.a, nbc, Z.w, Z.a))
        if ((rc = launched())) return rc;
    }
    {  // 4: dH1 = dZ2 W2
        GemmBatch gb;
        gb.n = 0;
        if (jc) gb.p[gb.n++] = jc->dh;
        if (ja) gb.p[gb.n++] = ja->dh;
        if ((rc = launch_gemm(st, gb))) return rc;
    }
    {  // 5: ReLU + LN1 backward
        const int two = (jc && ja) ? 2 : 1;
        const dim3 grid(rb * two);
        SC_C_SWITCH(C, hipLaunchKernelGGL(sc_ln1_bwd<CC>, grid, dim3(256), 0, st, A.l, rb, Z.l))
        if ((rc = launched())) return rc;
    }
    // 6: gradients + Adam
    GradAdam2 gg;
    gg.j0 = A.ga;
    gg.j1 = Z.ga;
    gg.nb0 = grad_blocks(A.ga);
    const int nb = gg.nb0 + ((jc && ja) ? grad_blocks(Z.ga) : 0);
    if (A.ga.nblk > kMaxRedBlocks || Z.ga.nblk > kMaxRedBlocks)
        return fail(-2, "flock_sc: too many reduction blocks (fc1 * in_dim too large)");
    const size_t lds = zmax(grad_lds(A.ga), grad_lds(Z.ga));
    const bool v11 = gemm_variant(A.ga.g) == 2 && gemm_variant(Z.ga.g) == 2;
    if (!v11) return launch_grad_adam_v<2, 2, 16>(st, gg, dim3(nb), lds);
    const int kc0 = gemm_kc(A.ga.g.K, A.ga.g.kchunk), kc1 = gemm_kc(Z.ga.g.K, Z.ga.g.kchunk);
    switch (nf_of(kc0 > kc1 ? kc0 : kc1)) {
        case 4: return launch_grad_adam_v<1, 1, 4>(st, gg, dim3(nb), lds);
        case 7: return launch_grad_adam_v<1, 1, 7>(st, gg, dim3(nb), lds);
        case 10: return launch_grad_adam_v<1, 1, 10>(st, gg, dim3(nb), lds);
        default: return launch_grad_adam_v<1, 1, 16>(st, gg, dim3(nb), lds);
    }
}

// learn() prologue: the agent index and the minibatch rows (Philox4x32-10, counter = (learn counter, row))
__device__ __forceinline__ uint4 philox4(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

__global__ __launch_bounds__(256) void sc_prep(int B, int64_t rows, uint64_t seed, uint64_t counter, int64_t* idx,
                                               int64_t* agent_out, int64_t agent) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r == 0) *agent_out = agent;
    if (idx && r < B) {
        const uint4 q = philox4(seed, (uint32_t)r, 0x5C5C5C5Cu, (uint32_t)counter, (uint32_t)(counter >> 32));
        const uint64_t u = ((uint64_t)q.x << 32) | q.y;
        idx[r] = (int64_t)(u % (uint64_t)rows);
    }
}

// learn() prologue with a minibatch snapshot: the sampled rows of every replay field are copied to staging rows
// 0..B-1, so the update can read the staging copy (with the identity index) while the next env step rewrites the ring
__global__ __launch_bounds__(256) void sc_prep_snapshot(int B, int64_t rows, uint64_t seed, uint64_t counter,
                                                        int64_t* idx_out, int64_t* agent_out, int64_t agent,
                                                        int in_dim, int n_actions, FlockScRows src,
                                                        FlockScRows dst) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r == 0) *agent_out = agent;
    if (r >= B) return;
    const uint4 q = philox4(seed, (uint32_t)r, 0x5C5C5C5Cu, (uint32_t)counter, (uint32_t)(counter >> 32));
    const uint64_t u = ((uint64_t)q.x << 32) | q.y;
    const int64_t row = (int64_t)(u % (uint64_t)rows);  // the row sc_prep samples for r
    if (idx_out) idx_out[r] = row;
    for (int c = 0; c < in_dim; ++c) {
        dst.state[(int64_t)r * in_dim + c] = src.state[row * in_dim + c];
        dst.new_state[(int64_t)r * in_dim + c] = src.new_state[row * in_dim + c];
    }
    for (int c = 0; c < n_actions; ++c) dst.action[(int64_t)r * n_actions + c] = src.action[row * n_actions + c];
    dst.reward[r] = src.reward[row];
    dst.terminal[r] = src.terminal[row];
}

}  // namespace

extern "C" {

int flock_sc_prep_snapshot(void* stream, int B, int64_t rows, uint64_t seed, uint64_t counter, int64_t* idx_out,
                           int64_t* agent_out, int64_t agent, int in_dim, int n_actions, const FlockScRows* ring,
                           const FlockScRows* staging) {
    if (!agent_out || !ring || !staging) return fail(-3, "flock_sc_prep_snapshot: NULL pointer");
    if (B < 1 || rows < 1 || in_dim < 1 || n_actions < 1)
        return fail(-5, "flock_sc_prep_snapshot: need B, rows, in_dim, n_actions >= 1");
    const FlockScRows* rs[2] = {ring, staging};
    for (const FlockScRows* x : rs)
        if (!x->state || !x->new_state || !x->action || !x->reward || !x->terminal)
            return fail(-3, "flock_sc_prep_snapshot: NULL field pointer");
    hipLaunchKernelGGL(sc_prep_snapshot, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, B, rows, seed,
                       counter, idx_out, agent_out, agent, in_dim, n_actions, *ring, *staging);
    return launched();
}

int flock_sc_prep(void* stream, int B, int64_t rows, uint64_t seed, uint64_t counter, int64_t* idx,
                  int64_t* agent_out, int64_t agent) {
    if (!agent_out) return fail(-3, "flock_sc_prep: NULL agent pointer");
    if (idx && (B < 1 || rows < 1)) return fail(-5, "flock_sc_prep: need B >= 1 and rows >= 1");
    const int blocks = idx ? (B + 255) / 256 : 1;
    hipLaunchKernelGGL(sc_prep, dim3(blocks), dim3(256), 0, (hipStream_t)stream, B, rows, seed, counter, idx,
                       agent_out, agent);
    return launched();
}

int64_t flock_sc_workspace_floats(int B, int in_dim, int n_actions, int fc1, int fc2) {
    return ws_layout(B, in_dim, n_actions, fc1, fc2, nullptr, nullptr);
}

int64_t flock_sc_update_size(void) { return (int64_t)sizeof(FlockScUpdate); }

int flock_sc_critic_update(void* stream, const FlockScUpdate* u) { return flock_sc_round(stream, u, nullptr); }

int flock_sc_actor_update(void* stream, const FlockScUpdate* u) { return flock_sc_round(stream, nullptr, u); }

int flock_sc_round(void* stream, const FlockScUpdate* critic_u, const FlockScUpdate* actor_u) {
    if (!critic_u && !actor_u) return fail(-3, "flock_sc_round: NULL argument");
    int rc = 0;
    if (critic_u && (rc = check(critic_u))) return rc;
    if (actor_u && (rc = check(actor_u))) return rc;
    Job jc, ja;
    if (critic_u) critic_job(critic_u, jc);
    if (actor_u) actor_job(actor_u, ja);
    return launch_round((hipStream_t)stream, critic_u ? &jc : nullptr, actor_u ? &ja : nullptr);
}


}  // extern "C"

// ---------------------------------------------------------------------------------------------------------------
// learn() pipeline: the config-3 loop's per-step learner work in one call (see include/flock_learn.h). Rounds are
// replayed from HIP graphs captured once: merged[s] = critic phase of slot s + actor phase of slot s - 1 (mod n),
// conly[s] / aonly[s] = one phase alone.
constexpr int kMaxSlots = 8;
struct FlockScPipeline {
    int n;
    FlockScUpdate u[kMaxSlots];
    FlockScRows ring, staging[kMaxSlots];
    hipGraphExec_t merged[kMaxSlots], conly[kMaxSlots], aonly[kMaxSlots];
    Job jc[kMaxSlots], ja[kMaxSlots];  // direct launches (graphs == false): the rounds' arguments, built once
    bool graphs;
    hipEvent_t snap_done[kMaxSlots], slot_free[kMaxSlots];
    bool used[kMaxSlots];
    int slot;
    int pending;  // slot of the learn() whose actor phase is not enqueued yet, or -1
    int64_t pending_agent;
};

namespace {
int capture_round(const FlockScUpdate* uc, const FlockScUpdate* ua, hipGraphExec_t* out) {
    hipStream_t cs;
    if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return fail(-4, "flock_sc_pipeline: stream");
    hipGraph_t g = nullptr;
    int rc = 0;
    if (hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        rc = fail(-4, "flock_sc_pipeline: begin capture");
    } else {
        rc = flock_sc_round(cs, uc, ua);
        const hipError_t e = hipStreamEndCapture(cs, &g);
        if (!rc && e != hipSuccess) rc = fail(-4, hipGetErrorString(e));
        if (!rc && hipGraphInstantiate(out, g, nullptr, nullptr, 0) != hipSuccess)
            rc = fail(-4, "flock_sc_pipeline: graph instantiate");
    }
    if (g) (void)hipGraphDestroy(g);
    (void)hipStreamDestroy(cs);
    return rc;
}
// one round of the pipeline on stream ls: critic phase of slot c and / or actor phase of slot a (-1: none)
int pipeline_round(FlockScPipeline* p, hipStream_t ls, int c, int a) {
    if (!p->graphs) return launch_round(ls, c >= 0 ? &p->jc[c] : nullptr, a >= 0 ? &p->ja[a] : nullptr);
    hipGraphExec_t g = c >= 0 && a >= 0 ? p->merged[c] : (c >= 0 ? p->conly[c] : p->aonly[a]);
    return hipGraphLaunch(g, ls) == hipSuccess ? 0 : fail(-4, "flock_sc_pipeline: graph launch failed");
}
}  // namespace

extern "C" {

FlockScPipeline* flock_sc_pipeline_create(int n_slots, const FlockScUpdate* slots, const FlockScRows* ring,
                                          const FlockScRows* staging) {
    if (!slots || !ring || !staging) {
        fail(-3, "flock_sc_pipeline_create: NULL argument");
        return nullptr;
    }
    if (n_slots < 2 || n_slots > kMaxSlots) {
        fail(-5, "flock_sc_pipeline_create: 2 <= n_slots <= 8");
        return nullptr;
    }
    for (int i = 0; i < n_slots; ++i) {
        if (check(&slots[i])) return nullptr;
        if (!slots[i].do_adam || !slots[i].critic_view) {
            fail(-5, "flock_sc_pipeline_create: each slot needs do_adam and a critic_view");
            return nullptr;
        }
        for (int j = 0; j < i; ++j)
            if (slots[i].critic_view == slots[j].critic_view || slots[i].workspace == slots[j].workspace) {
                fail(-5, "flock_sc_pipeline_create: each slot needs its own critic_view and workspace");
                return nullptr;
            }
    }
    FlockScPipeline* p = new FlockScPipeline();
    p->n = n_slots;
    p->ring = *ring;
    for (int i = 0; i < n_slots; ++i) {
        p->u[i] = slots[i];
        p->staging[i] = staging[i];
    }
    // rounds launched directly from arguments built here (6 hipLaunchKernel per round), or replayed as HIP graphs
    // (FLOCK_SC_PIPELINE_GRAPHS=1, read here once): config-3 step 0.117 ms direct vs 0.125 ms with graphs
    const char* ge = getenv("FLOCK_SC_PIPELINE_GRAPHS");
    p->graphs = ge && ge[0] == '1';
    int rc = 0;
    for (int i = 0; i < n_slots && !rc; ++i) {
        critic_job(&p->u[i], p->jc[i]);
        actor_job(&p->u[i], p->ja[i]);
        if (p->graphs) {
            rc = capture_round(&p->u[i], nullptr, &p->conly[i]);
            if (!rc) rc = capture_round(nullptr, &p->u[i], &p->aonly[i]);
            if (!rc) rc = capture_round(&p->u[i], &p->u[(i + n_slots - 1) % n_slots], &p->merged[i]);
        }
        hipEvent_t* evs[2] = {&p->snap_done[i], &p->slot_free[i]};
        for (hipEvent_t* e : evs)
            if (!rc && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess)
                rc = fail(-4, "flock_sc_pipeline_create: event");
        p->used[i] = false;
    }
    p->slot = 0;
    p->pending = -1;
    p->pending_agent = -1;
    if (rc) {
        flock_sc_pipeline_destroy(p);
        return nullptr;
    }
    return p;
}

int flock_sc_pipeline_learn(FlockScPipeline* p, void* env_stream, void* learner_stream, int64_t rows, uint64_t seed,
                            uint64_t counter, int64_t agent) {
    if (!p) return fail(-3, "flock_sc_pipeline_learn: NULL pipeline");
    hipStream_t es = (hipStream_t)env_stream, ls = (hipStream_t)learner_stream;
    const int s = p->slot, n = p->n;
    const FlockScUpdate& u = p->u[s];
    if (p->used[s] && hipStreamWaitEvent(es, p->slot_free[s], 0) != hipSuccess)
        return fail(-4, "flock_sc_pipeline_learn: wait");
    int rc = flock_sc_prep_snapshot(es, u.B, rows, seed, counter, nullptr, const_cast<int64_t*>(u.agent), agent,
                                    u.in_dim, u.n_actions, &p->ring, &p->staging[s]);
    if (rc) return rc;
    bool ok = hipEventRecord(p->snap_done[s], es) == hipSuccess && hipStreamWaitEvent(ls, p->snap_done[s], 0) == hipSuccess;
    if (!ok) return fail(-4, "flock_sc_pipeline_learn: stream operation failed");
    const int q = p->pending;
    if (q >= 0 && q == (s + n - 1) % n && p->pending_agent != agent) {
        // the actor phase of the previous learn() beside this critic phase (different agents: no shared state)
        if ((rc = pipeline_round(p, ls, s, q))) return rc;
        ok = hipEventRecord(p->slot_free[q], ls) == hipSuccess;
    } else {
        // same agent (this critic phase reads the target actor that actor phase soft-updates): one after the other
        if (q >= 0) {
            if ((rc = pipeline_round(p, ls, -1, q))) return rc;
            ok = hipEventRecord(p->slot_free[q], ls) == hipSuccess;
        }
        if (ok && (rc = pipeline_round(p, ls, s, -1))) return rc;
    }
    if (!ok) return fail(-4, "flock_sc_pipeline_learn: stream operation failed");
    p->pending = s;
    p->pending_agent = agent;
    p->used[s] = true;
    p->slot = (s + 1) % n;
    return 0;
}

int flock_sc_pipeline_flush(FlockScPipeline* p, void* learner_stream) {
    if (!p) return fail(-3, "flock_sc_pipeline_flush: NULL pipeline");
    const int q = p->pending;
    if (q < 0) return 0;
    hipStream_t ls = (hipStream_t)learner_stream;
    if (int rc = pipeline_round(p, ls, -1, q)) return rc;
    if (hipEventRecord(p->slot_free[q], ls) != hipSuccess)
        return fail(-4, "flock_sc_pipeline_flush: stream operation failed");
    p->pending = -1;
    return 0;
}

void flock_sc_pipeline_destroy(FlockScPipeline* p) {
    if (!p) return;
    for (int i = 0; i < p->n; ++i) {
        hipGraphExec_t* gs[3] = {&p->merged[i], &p->conly[i], &p->aonly[i]};
        for (hipGraphExec_t* g : gs)
            if (*g) (void)hipGraphExecDestroy(*g);
        hipEvent_t* evs[2] = {&p->snap_done[i], &p->slot_free[i]};
        for (hipEvent_t* e : evs)
            if (*e) (void)hipEventDestroy(*e);
    }
    delete p;
}

}  // extern "C"
