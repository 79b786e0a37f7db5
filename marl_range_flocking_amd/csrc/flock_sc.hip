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
#include "flock_mem.h"
#include "learn_internal.h"

namespace {

using flock_learn_internal::fail;
using flock_learn_internal::launched;

// replay rows per row-kernel block: one row per wave (round 4 measured 2 and 4 rows per wave 10-20 us per step slower
// beside the env kernel: DESIGN.md §3.3)
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
    float *DY1, *DXH1, *PS1;               // LN1 backward: dy, dxh = dy g1, row sums per dH tile [B][tiles][2]
    float *AXH1, *ARS1, *AH1, *CH1;        // actor phase fc1: actor xhat/rstd/h, updated critic h
    float* Z2b;                            // [2][B][H2] actor fc2, critic fc2
    float *AXH2, *ARS2, *AH2, *DM, *ADY2, *ADZ2, *ALOSS;
    float *ADY1, *ADXH1, *APS1;
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
    const int ps = 2 * ((H1 + 31) / 32);  // (sum dxh, sum dxh xh) per 32-column tile of a dH1 row
    x.DY1 = take(H1); x.DXH1 = take(H1); x.PS1 = take(ps);
    x.AXH1 = take(H1); x.ARS1 = take(1); x.AH1 = take(H1); x.CH1 = take(H1);
    x.Z2b = take(2 * (int64_t)H2);
    x.AXH2 = take(H2); x.ARS2 = take(1); x.AH2 = take(H2); x.DM = take(na); x.ADY2 = take(H2); x.ADZ2 = take(H2);
    x.ALOSS = take(1);
    x.ADY1 = take(H1); x.ADXH1 = take(H1); x.APS1 = take(ps);
    if (w) *w = x;
    return off;
}

// everything the row kernels read
struct RowArgs {
    int B, in, na, H1, H2;
    const int64_t* idx;
    const int64_t* agent;
    int64_t agent_v;  // >= 0: the agent index itself (the host's pipeline knows it), read instead of *agent
    const float *rs, *rs2, *ra, *rr, *rt;  // ring
    const float* critic;
    const float* actors;
    const float* actors_target;
    int64_t stride;
    float gamma, invB;
    // device-side snapshot gate (flock_sc_pipeline): the critic phase's row blocks wait until gate[0] >= gate_seq
    // (published by the snapshot kernel) instead of a cross-queue event wait; NULL: no wait
    unsigned long long* gate;
    unsigned long long gate_seq;
};
// the agent index of a job: the host's value when it has one (flock_sc_pipeline: no dependent load before the agent's
// parameter addresses), else the device word (graph-captured learns)
__device__ __forceinline__ int64_t agent_at(const int64_t* p, int64_t v) { return v >= 0 ? v : *p; }

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
// the replay row that minibatch row r of learn `counter` samples: Philox4x32-10(seed, (r, 0x5C5C5C5C, counter)) mod rows
// (uniform with replacement, ReplayBuffer.sample_buffer utils.py:65-76; sc_prep, the snapshot and the direct rounds'
// k1 rows all draw it this way)
__device__ __forceinline__ int64_t sample_row(uint64_t seed, uint64_t counter, int64_t rows, int r) {
    const uint4 q = philox4(seed, (uint32_t)r, 0x5C5C5C5Cu, (uint32_t)counter, (uint32_t)(counter >> 32));
    const uint64_t u = ((uint64_t)q.x << 32) | q.y;
    return (int64_t)(u % (uint64_t)rows);
}
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

// a register row from a [B][Fw] array (lane j holds features j, j + 64, ...; zero past Fw)
template <int C>
__device__ __forceinline__ void load_row(float (&v)[C], const float* p, int Fw, int lane) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = lane + 64 * c;
        v[c] = j < Fw ? p[j] : 0.0f;
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
template <int C, int HC>
__device__ __forceinline__ void c1_body(const Ws& w, const RowArgs& a, int bx, int path) {
    const int H1 = HC ? HC : a.H1;
    extern __shared__ float4 smem4[];
    float* xs = reinterpret_cast<float*>(smem4);  // [4 rows][kMaxIn] inputs, then the fc1 image
    float* sp = xs + kRowsPerBlock * kMaxIn;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r = bx * kRowsPerBlock + wv;
    // the staged replay rows and the agent index are read `sc1`: with the device-side gate (sc_k1) they are a
    // snapshot another queue's kernel has just written through (csrc/flock_mem.h); the index rows are constant
    using flock_mem::ld_sc1;
    const float* net = path == 0 ? a.actors_target + (a.agent_v >= 0 ? a.agent_v : ld_sc1(a.agent)) * a.stride : a.critic;  // fc1 block at offset 0
    const bool live = r < a.B;
    if (live) {
        const int64_t ir = a.idx[r];
        const float* x = (path == 2 ? a.rs : a.rs2) + ir * a.in;
        const float xv = lane < a.in ? ld_sc1(x + lane) : 0.0f;
        if (lane < a.in) xs[wv * kMaxIn + lane] = xv;
        if (path == 2) {
            if (lane < a.in) {
                w.S[(int64_t)r * a.in + lane] = xv;
                w.S2[(int64_t)r * a.in + lane] = ld_sc1(a.rs2 + ir * a.in + lane);
            }
            if (lane < a.na) w.A[(int64_t)r * a.na + lane] = ld_sc1(a.ra + ir * a.na + lane);
            if (lane == 0) {
                w.R[r] = ld_sc1(a.rr + ir);
                w.T[r] = ld_sc1(a.rt + ir);
            }
        }
    }
    stage(sp, net, H1 * (a.in + 3));
    __syncthreads();
    if (!live) return;
    float xh[C], h[C], rs;
    fc1_ln_relu<C>(xs + wv * kMaxIn, a.in, sp, H1, lane, xh, h, rs);
    const int64_t ro = (int64_t)r * H1;
    if (path == 0) {
        store_row<C>(w.TH1 + ro, h, H1, lane);
    } else if (path == 1) {
        store_row<C>(w.NH1 + ro, h, H1, lane);
    } else {
        store_row<C>(w.XH1 + ro, xh, H1, lane);
        store_row<C>(w.H1 + ro, h, H1, lane);
        if (lane == 0) w.RS1[r] = rs;
    }
}

// c3: heads, TD target, MSE and the critic backward down to the fc2 pre-activation
template <int C, int HC, int NAC>
__device__ __forceinline__ void c3_body(const Ws& w, const RowArgs& a, int bx) {
    extern __shared__ float4 smem4[];
    float* ct = reinterpret_cast<float*>(smem4);  // critic tail
    const int H2 = HC ? HC : a.H2, na = NAC ? NAC : a.na;
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
    stage(at, a.actors_target + agent_at(a.agent, a.agent_v) * a.stride + ao.g2, act_tail_len(na, H2));
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
// a1 (grid.y = path): 0 the agent's actor fc1/LN/ReLU on s (saved for backward), 1 the updated critic's on s
template <int C, int HC>
__device__ __forceinline__ void a1_body(const Ws& w, const RowArgs& a, int bx, int path) {
    const int H1 = HC ? HC : a.H1;
    extern __shared__ float4 smem4[];
    float* xs = reinterpret_cast<float*>(smem4);
    float* sp = xs + kRowsPerBlock * kMaxIn;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r = bx * kRowsPerBlock + wv;
    const bool live = r < a.B;
    const float* net = path == 0 ? a.actors + agent_at(a.agent, a.agent_v) * a.stride : a.critic;
    if (live && lane < a.in) xs[wv * kMaxIn + lane] = w.S[(int64_t)r * a.in + lane];
    stage(sp, net, H1 * (a.in + 3));
    __syncthreads();
    if (!live) return;
    float xh[C], h[C], rs;
    fc1_ln_relu<C>(xs + wv * kMaxIn, a.in, sp, H1, lane, xh, h, rs);
    const int64_t ro = (int64_t)r * H1;
    if (path == 0) {
        store_row<C>(w.AXH1 + ro, xh, H1, lane);
        store_row<C>(w.AH1 + ro, h, H1, lane);
        if (lane == 0) w.ARS1[r] = rs;
    } else {
        store_row<C>(w.CH1 + ro, h, H1, lane);
    }
}

// a3: actor LN2/ReLU/mu/tanh, Q(s, mu) with the updated critic, actor loss -mean Q, and the backward through the
// critic's action branch (dQ/dmu) and the actor head down to the actor's fc2 pre-activation
template <int C, int HC, int NAC>
__device__ __forceinline__ void a3_body(const Ws& w, const RowArgs& a, int bx) {
    extern __shared__ float4 smem4[];
    float* ct = reinterpret_cast<float*>(smem4);
    const int H2 = HC ? HC : a.H2, na = NAC ? NAC : a.na;
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
    stage(at, a.actors + agent_at(a.agent, a.agent_v) * a.stride + ao.g2, act_tail_len(na, H2));
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

// -DFLOCK_SC_PROF (diagnostics build, tools/sc_block_prof.py): per-block start / end times (s_memrealtime, 100 MHz)
// of the five round kernels (the start by thread 0, the end as the max over the block's waves), and phase marks of
// the forward GEMM blocks
#ifdef FLOCK_SC_PROF
__device__ unsigned long long g_scprof[5][4096][2];
struct ScProf {
    int k;
    unsigned long long t0;
    __device__ explicit ScProf(int kk) : k(kk), t0(__builtin_amdgcn_s_memrealtime()) {}
    __device__ ~ScProf() {
        const int b = blockIdx.x + gridDim.x * blockIdx.y;
        if (b < 4096 && (threadIdx.x & 63) == 0) {
            if (threadIdx.x == 0) g_scprof[k][b][0] = t0;
            atomicMax(&g_scprof[k][b][1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
        }
    }
};
#define SC_PROF(k) ScProf sc_prof_(k)
__device__ unsigned long long g_scmark[4096][8];
#define SC_MARK(MK, i)                                                                           \
    if (MK && threadIdx.x == 0 && blockIdx.x + gridDim.x * blockIdx.y < 4096)                   \
        g_scmark[blockIdx.x + gridDim.x * blockIdx.y][i] = __builtin_amdgcn_s_memrealtime();
#else
#define SC_PROF(k)
#define SC_MARK(MK, i)
#endif
// -DFLOCK_SC_PRIO=n (A/B builds only, tools/build_variant_sc.sh): the round kernels' waves raise their issue priority
// to n (s_setprio) over co-resident env waves
#ifdef FLOCK_SC_PRIO
#define SC_WAVE_PRIO() __builtin_amdgcn_s_setprio(FLOCK_SC_PRIO)
#else
#define SC_WAVE_PRIO()
#endif
// Merged row kernels of a learn() round (launch_round): the critic-phase job of one learn() and the actor-phase job of
// the previous one in ONE launch, picked by a block-uniform branch (either job may be absent: npc / nbc = 0, or no
// blocks past them).
// The device-side snapshot gate: gate[0] = the sequence number of the last published snapshot, gate[1] = error word
// (set by a waiter that gave up; flock_sc_pipeline_check reports it). One lane polls gate[0] with `sc1` loads until it
// reaches seq; the block's waves then read the snapshot rows with `sc1` loads after the barrier (the producer wrote
// them `sc1`, waited for every store, and set the flag after a workgroup barrier: csrc/flock_mem.h). A wait longer
// than kGateTimeoutTicks sets the error word and the block computes nothing (the host raises; no silent result).
// 2 s of s_memrealtime (100 MHz): the env stream may be held up by work enqueued on it before the learn() (an
// evaluation rollout, a long copy); 0.2 s failed a learn behind a 0.2-s kernel (tools/rccl_host_cost.py, round 5)
constexpr unsigned long long kGateTimeoutTicks = 200000000ull;
__device__ __forceinline__ bool gate_wait(unsigned long long* gate, unsigned long long seq,
                                          unsigned long long* err = nullptr,
                                          unsigned long long ticks = kGateTimeoutTicks) {
    __shared__ int ok;
    if (threadIdx.x == 0) {
        int good = 1;
        if ((long long)(flock_mem::ld_sc1(gate) - seq) < 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while ((long long)(flock_mem::ld_sc1(gate) - seq) < 0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                    __hip_atomic_store(err ? err : gate + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    good = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        ok = good;
    }
    __syncthreads();
    return ok != 0;
}

// XCD-aligned work order (speed only; every map here is a bijection of the block index, whatever the placement).
// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md: b and b + 8 share one), and lines an XCD's L2
// holds survive the kernel boundary (tools/ubench_l2_persist.hip: a same-XCD re-read in the next launch runs at the
// L2-hit time, 0.49 us, against 1.5 us from another XCD; profiles/r05/xcd/). With n a multiple of 8, block x takes
// work item (x mod 8) (n / 8) + x / 8: the items of group g = x mod 8 (row strip g of the minibatch: rows
// [g B / 8, (g + 1) B / 8)) run on one XCD in every launch of a round, so the fc1 rows k1 writes are L2 hits for the
// forward GEMM tiles of that strip (xcd_tile), its fc2 outputs for the k3 rows, and k1 / k3 rows for the bwd launch's
// dH1 tiles.
__device__ __forceinline__ int xcd_perm(int x, int n) { return (n & 7) == 0 ? (x & 7) * (n >> 3) + (x >> 3) : x; }

// Round 5 also had each XCD's k1 blocks pull the forward GEMM's fc2.weight panels into that XCD's L2 (one dword per
// 128-B line): it took the GEMM 18.1 -> 14.5 us in the loop while the rounds waited on a slot-free event between them;
// with the rounds back to back (round 6) the pull on k1's path cost more than it saved (same-box A/B, 200 steps
// 0.0743-0.0750 without against 0.0775-0.0790 ms per step, driver command 0.0825-0.0849 against 0.0838-0.0863;
// profiles/r06/nopull/) and was removed
template <int C, int HC>
__global__ __launch_bounds__(256) void sc_k1(Ws wc, RowArgs ac, int npc, Ws wa, RowArgs aa) {
    SC_PROF(0);
    SC_WAVE_PRIO();
    const bool crit = (int)blockIdx.y < npc;
    if (ac.gate && crit && !gate_wait(ac.gate, ac.gate_seq)) return;  // this learn's snapshot
    const int bx = xcd_perm(blockIdx.x, gridDim.x);
    if (crit)
        c1_body<C, HC>(wc, ac, bx, blockIdx.y);
    else
        a1_body<C, HC>(wa, aa, bx, blockIdx.y - npc);
}
template <int C, int HC, int NAC>
__global__ __launch_bounds__(256) void sc_k3(Ws wc, RowArgs ac, int nbc, Ws wa, RowArgs aa) {
    SC_PROF(2);
    SC_WAVE_PRIO();
    const int nba = (int)gridDim.x - nbc;
    if ((int)blockIdx.x < nbc)
        c3_body<C, HC, NAC>(wc, ac, (nbc & 7) == 0 ? xcd_perm(blockIdx.x, nbc) : (int)blockIdx.x);
    else
        a3_body<C, HC, NAC>(wa, aa, (nbc & 7) == 0 ? xcd_perm(blockIdx.x - nbc, nba) : (int)blockIdx.x - nbc);
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
#ifndef FLOCK_FWD_KC  // (A/B builds only, tools/build_variant_sc.sh)
#define FLOCK_FWD_KC 200
#endif
#ifndef FLOCK_GRAD_KC
#define FLOCK_GRAD_KC 128
#endif
constexpr int kFwdKC = FLOCK_FWD_KC;   // (round 5 with the XCD-aligned round: 0.0814-0.0822 ms per step against 0.0836-0.0843
                              // for 136-deep chunks and 0.098 for whole panels, profiles/r05/fwdkc/)
                              // forward / input-gradient GEMM K chunk: 0.098 ms per config-3 step vs 0.117 with whole
                              // 400-deep panels (lighter blocks co-run with the env kernel; tools/gpu_kc_sweep.sh)
constexpr int kGradKC = FLOCK_GRAD_KC;  // the gradient kernels share one launch with ~400 LDS-free reduction blocks: a 34-KB
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
    int64_t agent_v;  // >= 0: the agent index itself (RowArgs::agent_v)
    int tiles_n, tiles;
    int kchunk;  // K panel depth staged per round (<= kKC, multiple of 8)
};
constexpr int kMaxBatch = 5;  // a round's forward GEMMs: 3 (critic phase) + 2 (actor phase)
struct GemmBatch {
    GemmP p[kMaxBatch];
    int n;
    // the critic phase's snapshot consumed (its k1 launch, the only reader of the staging rows, has completed): block
    // (0, 0) stores done_seq to *done write-through for a snapshot kernel waiting to reuse the slot; NULL: none
    unsigned long long* done;
    unsigned long long done_seq;
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
template <int AV, int BV, int NF, int MK = 0>
__device__ __forceinline__ void gemm_tile(const GemmP& g, const float* Bp, int tm, int tn, float* smem,
                                          float (&out)[4]) {
    SC_MARK(MK, 0)
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
            SC_MARK(MK, (k0 ? 4 : 1))
            __syncthreads();
            SC_MARK(MK, (k0 ? 5 : 2))
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
            SC_MARK(MK, (k0 ? 6 : 3))
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
    SC_MARK(MK, 7)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int v = 4 * wv + q;
        out[q] = ((red[(0 * 16 + v) * 64 + l] + red[(1 * 16 + v) * 64 + l]) + red[(2 * 16 + v) * 64 + l]) +
                 red[(3 * 16 + v) * 64 + l];
    }
}

// XCD-aware tile order of a problem (blocks are dealt round-robin over the 8 XCDs: b and b + 8 share one; observed,
// used for speed only): with the grid's x extent equal to the problem's tile count and a multiple of 8, block x takes
// tile (x % 8) * (tiles / 8) + x / 8, so each XCD computes a contiguous run of tiles (at 8 row strips: one strip of
// A and all of B) and its L2 fetches ~1/8 of A from the Infinity Cache instead of nearly all of it
__device__ __forceinline__ int xcd_tile(int x, int tiles) {
    return (tiles & 7) == 0 && (int)gridDim.x == tiles ? (x & 7) * (tiles >> 3) + (x >> 3) : x;
}

// one forward GEMM tile: block x of problem y computes tile xcd_tile(x)
template <int AV, int BV, int NF>
__device__ __forceinline__ void gemm_block(const GemmBatch& gb, int y, int x) {
    extern __shared__ float4 smem4[];
    float* smem = reinterpret_cast<float*>(smem4);
    const GemmP& g = gb.p[y];
    if (x >= g.tiles) return;
    const int t = xcd_tile(x, g.tiles);
    const int tm = t / g.tiles_n, tn = t - tm * g.tiles_n;
    const int64_t rel = g.relB ? g.relB * agent_at(g.agent, g.agent_v) : 0;
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int n = tn * kT + (l & 31);
    const float bias = (g.bias && n < g.N) ? g.bias[rel + n] : 0.0f;
    float out[4];
    gemm_tile<AV, BV, NF, 1>(g, g.B + rel, tm, tn, smem, out);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int m = tm * kT + 8 * wv + 4 * (l >> 5) + q;
        if (m < g.M && n < g.N) g.C[(int64_t)m * g.ldc + n] = g.bias ? out[q] + bias : out[q];
    }
}

// grid (max tiles, problems): block (x, y) computes tile xcd_tile(x) of problem y
template <int AV, int BV, int NF>
__global__ __launch_bounds__(256) void sc_gemm(GemmBatch gb) {
    SC_PROF(1);
    SC_WAVE_PRIO();
    if (gb.done && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) flock_mem::st_sc1(gb.done, gb.done_seq);
    gemm_block<AV, BV, NF>(gb, blockIdx.y, blockIdx.x);
}

// ---------------------------------------------------------------------------------------------------------------
// Backward and update, the last two launches of a round.
//   bwd  (sc_bwd): dH1 = dZ2 W2 tiles with the ReLU + LN1-backward epilogue (dy = dH1 [h > 0], dxh = dy g1, and per
//        row and 32-column tile the partial sums of dxh and dxh xhat), the fc2.weight gradient dW2 = dZ2^T H1 tiles,
//        and the reductions whose inputs the row kernels already wrote (fc2.bias, LN2, heads, loss): gradients only.
//   late (sc_grad_adam): the fc1 / LN1 reductions, with dz = rstd (dxh - mean(dxh) - xhat mean(dxh xhat)) formed on
//        the fly from those row sums (no LN1-backward launch), Adam inline; Adam of the parameters whose gradients
//        the bwd launch wrote; the step counter; the critic's self soft update when it has no view.
// Reductions: red[q] (the last q with red[q].blk0 <= block) over the B rows, 16 elements per block (16 row groups):
//   mode 0: g[o] = sum_b D[b, o]         (biases, LayerNorm beta)
//   mode 1: g[o] = sum_b D[b, o] X[b, o] (LayerNorm gamma)
//   mode 2: g[o*in + i] = sum_b D[b, o] X[b, i]  (action_value / head weights)
//   mode 3: loss = sum_b D[b] / B        (written to *loss, no Adam)
//   mode 4: g[o*in + i] = sum_b dz[b, o] X[b, i], dz from D = dxh (fc1.weight)
//   mode 5: g[o] = sum_b dz[b, o]                  (fc1.bias)
struct RedP {
    const float* D;
    const float* X;
    int ldd, ldx, mode, in, n, blk0;
    int64_t off;
};
constexpr int kMaxRed = 12;
#ifndef FLOCK_RED_RB  // (A/B builds only, tools/build_variant_sc.sh)
#define FLOCK_RED_RB 8
#endif
// output elements per reduction block; the block's 256 threads are kRedElems elements x kRedGroups row groups (group q
// takes rows q, q + kRedGroups, ...; 8 and 4 elements per block measured slower in round 4: DESIGN.md §3.3)
constexpr int kRedElems = 16;
constexpr int kRedGroups = 256 / kRedElems;
constexpr int kMaxRedBlocks = 4096;

// LN1 row statistics for modes 4 / 5, from the bwd launch's per-tile row sums
struct DzArgs {
    const float *XH, *RS, *PS;  // xhat [B][F], rstd [B], row sums [B][ntn][2]
    int F, ntn;
};

// One block's reduction: the kRedElems-element slice of rp for block b (thread el = tid % kRedElems, row group
// q = tid / kRedElems);
// returns the sum in threads q == 0 (0 elsewhere). part: 256 floats of LDS; mst: [B][2] LDS (modes 4 / 5)
__device__ __forceinline__ float red_block(const RedP& rp, int b, int B, const DzArgs& dz, float* part, float* mst,
                                           int& e_out, bool& live_out) {
    const int tid = threadIdx.x;
    const bool dzm = rp.mode == 4 || rp.mode == 5;
    const int el = tid & (kRedElems - 1), q = tid / kRedElems;
    const int e = (b - rp.blk0) * kRedElems + el;
    const bool live = e < rp.n;
    const bool per_in = rp.mode == 2 || rp.mode == 4;
    const int o = per_in ? e / rp.in : e;
    const int i = per_in ? e - o * rp.in : e;
    const bool prod = rp.mode == 1 || rp.mode == 2 || rp.mode == 4;
    constexpr int kRB = FLOCK_RED_RB;  // rows per batch of loads (row group q takes rows q, q + kRedGroups, ...; 4 and 16 flat or
                            // slower in round 3)
    float dv[kRB], xv[kRB], xh[kRB], rs[kRB];
    auto load = [&](int r0) {
#pragma unroll
        for (int k = 0; k < kRB; ++k) {
            const int r = r0 + kRedGroups * k;
            const bool in = live && r < B;
            dv[k] = in ? rp.D[(int64_t)r * rp.ldd + o] : 0.0f;
            xv[k] = (in && prod) ? rp.X[(int64_t)r * rp.ldx + i] : 0.0f;
            xh[k] = (in && dzm) ? dz.XH[(int64_t)r * dz.F + o] : 0.0f;
            rs[k] = (in && dzm) ? dz.RS[r] : 0.0f;
        }
    };
    load(q);  // the first batch is in flight while the LN1 row statistics are formed
    if (dzm) {  // mean(dxh), mean(dxh xhat) of every row: its tiles' partial sums in a fixed order
        for (int r = tid; r < B; r += 256) {
            const float2* ps = reinterpret_cast<const float2*>(dz.PS + (int64_t)r * 2 * dz.ntn);
            float s1 = 0.0f, s2 = 0.0f;
            // the row's tile sums in batches of 16 independent loads (one memory round trip per batch; a plain loop
            // waited for each load in turn: 13 round trips at fc1 = 400), added in tile order
            constexpr int kPB = 16;
            for (int t0 = 0; t0 < dz.ntn; t0 += kPB) {
                float2 v[kPB];
#pragma unroll
                for (int u = 0; u < kPB; ++u)
                    v[u] = t0 + u < dz.ntn ? ps[t0 + u] : make_float2(0.0f, 0.0f);
#pragma unroll
                for (int u = 0; u < kPB; ++u)
                    if (t0 + u < dz.ntn) {
                        s1 += v[u].x;
                        s2 += v[u].y;
                    }
            }
            mst[2 * r] = s1 / (float)dz.F;
            mst[2 * r + 1] = s2 / (float)dz.F;
        }
        __syncthreads();
    }
    float acc = 0.0f;
    for (int r0 = q; r0 < B; r0 += kRedGroups * kRB) {
        if (r0 != q) load(r0);
        if (dzm) {
#pragma unroll
            for (int k = 0; k < kRB; ++k) {
                const int r = min(r0 + kRedGroups * k, B - 1);
                dv[k] = rs[k] * (dv[k] - mst[2 * r] - xh[k] * mst[2 * r + 1]);  // ln_backward's dz
            }
        }
#pragma unroll
        for (int k = 0; k < kRB; ++k) acc = prod ? fmaf(dv[k], xv[k], acc) : acc + dv[k];
    }
    part[q * kRedElems + el] = acc;
    __syncthreads();
    float gsum = 0.0f;
    if (q == 0 && live) {
#pragma unroll
        for (int k = 0; k < kRedGroups; ++k) gsum += part[k * kRedElems + el];
    }
    e_out = e;
    live_out = live && q == 0;
    return gsum;
}

struct BwdJob {
    GemmP dh;                    // dH1 = dZ2 W2 (B x H1, K = H2); W2 agent-relative through dh.relB / dh.agent
    GemmP dw;                    // dW2 = dZ2^T H1 (H2 x H1, K = B) -> grad + w2_off
    const float *H1, *XH1, *g1;  // LN1-backward epilogue of the dH tiles (g1 agent-relative like grad)
    float *DY1, *DXH1, *PS1;
    int F, ntn;
    int64_t w2_off;
    int nred, nblk, B;
    RedP red[kMaxRed];
    float* grad;
    int64_t rel;       // g1 is agent-relative: + rel * (*agent)
    int64_t grad_rel;  // grad is agent-relative: + grad_rel * (*agent) (0: FlockScUpdate.actor_grad_out)
    const int64_t* agent;
    int64_t agent_v;  // >= 0: the agent index itself
    float* loss;
};
__host__ __device__ inline int bwd_blocks(const BwdJob& j) { return j.dh.tiles + j.dw.tiles + j.nblk; }

// the 4 rows of thread (wave w, lane l) in a 32 x 32 tile: 8w + 4(l >> 5) + q; its column: l & 31
template <int AVH, int BVH, int AVW, int BVW, int NFH, int NFW>
__device__ __forceinline__ void bwd_body(const BwdJob& j, int bx) {
    extern __shared__ float4 smem4[];
    float* smem = reinterpret_cast<float*>(smem4);
    const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
    const int64_t base = j.rel ? j.rel * agent_at(j.agent, j.agent_v) : 0;
    const int64_t gbase = j.grad_rel ? j.grad_rel * agent_at(j.agent, j.agent_v) : 0;
    if (bx < j.dh.tiles) {
        const GemmP& g = j.dh;
        const int t = xcd_perm(bx, g.tiles);  // row strips on the XCDs of the k1 / k3 rows they read (xcd_perm)
        const int tm = t / g.tiles_n, tn = t - tm * g.tiles_n;
        const int64_t relB = g.relB ? g.relB * agent_at(g.agent, g.agent_v) : 0;
        const int n = tn * kT + (l & 31);
        const bool nok = n < g.N;
        // the epilogue's inputs, loaded before the GEMM
        const float gam = nok ? j.g1[base + n] : 0.0f;
        float hv[4], xv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int m = tm * kT + 8 * wv + 4 * (l >> 5) + q;
            const bool ok = m < g.M && nok;
            hv[q] = ok ? j.H1[(int64_t)m * j.F + n] : 0.0f;
            xv[q] = ok ? j.XH1[(int64_t)m * j.F + n] : 0.0f;
        }
        float out[4];
        gemm_tile<AVH, BVH, NFH>(g, g.B + relB, tm, tn, smem, out);
        float s1[4], s2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int m = tm * kT + 8 * wv + 4 * (l >> 5) + q;
            const bool ok = m < g.M && nok;
            const float dy = hv[q] > 0.0f ? out[q] : 0.0f;  // through the ReLU
            const float dxh = dy * gam;
            if (ok) {
                j.DY1[(int64_t)m * j.F + n] = dy;
                j.DXH1[(int64_t)m * j.F + n] = dxh;
            }
            s1[q] = ok ? dxh : 0.0f;
            s2[q] = ok ? dxh * xv[q] : 0.0f;
        }
        // row sums over the tile's 32 columns (the 32 lanes of a half-wave): xor butterfly, bitwise equal in all lanes
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                s1[q] += __shfl_xor(s1[q], off);
                s2[q] += __shfl_xor(s2[q], off);
            }
        if ((l & 31) == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int m = tm * kT + 8 * wv + 4 * (l >> 5) + q;
                if (m < g.M) {
                    j.PS1[((int64_t)m * j.ntn + tn) * 2] = s1[q];
                    j.PS1[((int64_t)m * j.ntn + tn) * 2 + 1] = s2[q];
                }
            }
        }
    } else if (bx < j.dh.tiles + j.dw.tiles) {
        const GemmP& g = j.dw;
        const int t = bx - j.dh.tiles;
        const int tm = t / g.tiles_n, tn = t - tm * g.tiles_n;
        float out[4];
        gemm_tile<AVW, BVW, NFW>(g, g.B, tm, tn, smem, out);
        const int nn = tn * kT + (l & 31);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int mm = tm * kT + 8 * wv + 4 * (l >> 5) + q;
            if (mm < g.M && nn < g.N) j.grad[gbase + j.w2_off + (int64_t)mm * g.ldc + nn] = out[q];
        }
    } else {
        const int b = bx - j.dh.tiles - j.dw.tiles;
        int q0 = 0;  // descriptor of this block: a wave-uniform search over <= kMaxRed scalars
        for (int q = 1; q < j.nred; ++q)
            if (b >= j.red[q].blk0) q0 = q;
        const RedP& rp = j.red[q0];
        int e;
        bool wr;
        const DzArgs none{nullptr, nullptr, nullptr, 0, 0};
        const float gsum = red_block(rp, b, j.B, none, smem, nullptr, e, wr);
        if (wr) {
            if (rp.mode == 3)
                *j.loss = gsum * (1.0f / (float)j.B);
            else
                j.grad[gbase + rp.off + e] = gsum;
        }
    }
}

struct Bwd2 {
    BwdJob j0, j1;
    int nb0;  // blocks of job j0, padded to a multiple of 8 (j1's dH1 tiles then start on XCD group 0 too)
    int n0;   // blocks job j0 uses
};
template <int AVH, int BVH, int AVW, int BVW, int NFH, int NFW>
__global__ __launch_bounds__(256) void sc_bwd(Bwd2 bb) {
    SC_PROF(3);
    SC_WAVE_PRIO();
    if ((int)blockIdx.x < bb.nb0) {
        if ((int)blockIdx.x < bb.n0) bwd_body<AVH, BVH, AVW, BVW, NFH, NFW>(bb.j0, blockIdx.x);
    } else {
        bwd_body<AVH, BVH, AVW, BVW, NFH, NFW>(bb.j1, blockIdx.x - bb.nb0);
    }
}

struct GradAdam {
    int nred, nblk, B, do_adam;
    RedP red[kMaxRed];
    DzArgs dz;
    int64_t adam_lo, adam_n;  // Adam-only region (gradients written by the bwd launch), relative to the agent base
    int adam_blocks;
    float *p, *grad, *m, *v;
    int64_t rel;       // p/m/v (and target) are agent-relative: + rel * (*agent)
    int64_t grad_rel;  // grad likewise: + grad_rel * (*agent) (0 with FlockScUpdate.actor_grad_out)
    const float* grad_scale;  // Adam-only blocks: gradient *= *grad_scale first (data-parallel 1 / world), or NULL
    const int64_t* agent;
    int64_t agent_v;  // >= 0: the agent index itself
    int64_t* step;  // step[0], or step[*agent] when rel != 0
    unsigned* counter;
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
__host__ __device__ inline int late_blocks(const GradAdam& ga) { return ga.nblk + ga.adam_blocks + ga.soft_blocks; }

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

// one job's blocks of the late launch: [0, nblk) reductions, [nblk, + adam_blocks) Adam of the bwd launch's
// gradients, then soft_blocks self soft update blocks
__device__ __forceinline__ void grad_adam_body(const GradAdam& ga, int bx, int nb) {
    extern __shared__ float4 smem4[];
    float* smem = reinterpret_cast<float*>(smem4);
    __shared__ float sh[2];
    __shared__ int sh_soft;
    const int tid = threadIdx.x;
    const int64_t agent = ga.rel ? agent_at(ga.agent, ga.agent_v) : 0;
    const int64_t base = ga.rel * agent, gbase = ga.grad_rel * agent;
    if (tid == 0) {
        const int64_t step0 = ga.do_adam ? ga.step[agent] : 0;
        const int64_t count = ga.soft_count ? ga.soft_count[agent_at(ga.agent, ga.agent_v)] : step0;
        sh_soft = ga.do_adam && ga.soft_rate > 0 && (count % ga.soft_rate) == 0;  // this learn's count
        if (ga.do_adam) {
            const double st = (double)(step0 + 1);
            sh[0] = (float)(-(double)ga.lr / (1.0 - pow((double)ga.b1, st)));
            sh[1] = (float)sqrt(1.0 - pow((double)ga.b2, st));
        }
    }
    const int adam0 = ga.nblk, soft0 = ga.nblk + ga.adam_blocks;
    if (bx >= soft0) {  // critic self soft update blocks (after its Adam step)
        __syncthreads();
        if (sh_soft && ga.self_soft) {
            const int64_t b0 = (int64_t)(bx - soft0) * 1024;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t e = b0 + q * 256 + tid;
                if (e < ga.self_n) {
                    const float c = ga.self_soft[e];
                    ga.self_soft[e] = ga.tau * c + ga.one_minus_tau * c;
                }
            }
        }
    } else if (bx >= adam0) {  // Adam of gradients the bwd launch wrote: every load first, then the updates
        const int64_t e0 = ga.adam_lo + (int64_t)(bx - adam0) * 1024, end = ga.adam_lo + ga.adam_n;
        AdamState st[4];
        float gi[4];
        const float gs = ga.grad_scale ? *ga.grad_scale : 1.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t e = e0 + q * 256 + tid;
            st[q] = e < end ? adam_load(ga, base + e) : AdamState{0.f, 0.f, 0.f, 0.f};
            gi[q] = e < end ? ga.grad[gbase + e] : 0.0f;
        }
        // the bias corrections of thread 0 (its step load and pow) after the loads are issued: one memory round trip
        // for the whole block instead of the step load's followed by the element loads'
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t e = e0 + q * 256 + tid;
            if (e < end) adam_store(ga, base + e, st[q], ga.grad_scale ? gi[q] * gs : gi[q], sh[0], sh[1], sh_soft != 0);
        }
    } else {
        const int b = bx;
        int q0 = 0;  // descriptor of this block: a wave-uniform search over <= kMaxRed scalars
        for (int q = 1; q < ga.nred; ++q)
            if (b >= ga.red[q].blk0) q0 = q;
        const RedP& rp = ga.red[q0];
        const int e1 = (b - rp.blk0) * kRedElems + (tid & (kRedElems - 1));
        const bool ad = tid / kRedElems == 0 && e1 < rp.n && rp.mode != 3 && ga.do_adam;
        const AdamState st = ad ? adam_load(ga, base + rp.off + e1) : AdamState{0.f, 0.f, 0.f, 0.f};
        int e;
        bool wr;
        const float gsum = red_block(rp, b, ga.B, ga.dz, smem, smem + 256, e, wr);
        if (wr) {
            ga.grad[gbase + rp.off + e] = gsum;
            if (ga.do_adam) adam_store(ga, base + rp.off + e, st, gsum, sh[0], sh[1], sh_soft != 0);
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

// a round's late launch: blocks [0, nb0) run job j0, the rest job j1 (when there are any)
struct GradAdam2 {
    GradAdam j0, j1;
    int nb0;
};
__global__ __launch_bounds__(256) void sc_grad_adam(GradAdam2 gg) {
    SC_PROF(4);
    SC_WAVE_PRIO();
    if ((int)blockIdx.x < gg.nb0)
        grad_adam_body(gg.j0, blockIdx.x, gg.nb0);
    else
        grad_adam_body(gg.j1, blockIdx.x - gg.nb0, gridDim.x - gg.nb0);
}

// ---------------------------------------------------------------------------------------------------------------
// host side
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
    g.agent_v = -1;
    g.tiles_n = (N + kT - 1) / kT;
    g.tiles = ((M + kT - 1) / kT) * g.tiles_n;
    g.kchunk = balanced_kc(K, kFwdKC);
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

// append reduction descriptor n elements (mode: see RedP) to a bwd or late job
template <typename J>
void add_red(J& ga, const float* D, int ldd, const float* X, int ldx, int mode, int in, int n, int64_t off) {
    const int j = ga.nred++;
    RedP& r = ga.red[j];
    r.D = D; r.X = X; r.ldd = ldd; r.ldx = ldx; r.mode = mode; r.in = in; r.n = n; r.off = off;
    r.blk0 = ga.nblk;
    ga.nblk += (n + kRedElems - 1) / kRedElems;
}
size_t red_lds(int B) { return (size_t)(256 + 2 * B) * sizeof(float); }  // part + LN1 row statistics
size_t bwd_lds(const BwdJob& j) {
    const size_t a = gemm_lds_bytes(j.dh.K, j.dh.kchunk), b = gemm_lds_bytes(j.dw.K, j.dw.kchunk);
    const size_t r = 256 * sizeof(float);
    return a > b ? (a > r ? a : r) : (b > r ? b : r);
}

template <int AVH, int BVH, int AVW, int BVW, int NFH, int NFW>
int launch_bwd_v(hipStream_t st, const Bwd2& bb, dim3 grid, size_t lds) {
    if (int rc = allow_lds(sc_bwd<AVH, BVH, AVW, BVW, NFH, NFW>, lds)) return rc;
    hipLaunchKernelGGL((sc_bwd<AVH, BVH, AVW, BVW, NFH, NFW>), grid, dim3(256), lds, st, bb);
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
    a.idx = u->idx; a.agent = u->agent; a.agent_v = -1;
    a.rs = u->ring_state; a.rs2 = u->ring_new_state; a.ra = u->ring_action; a.rr = u->ring_reward;
    a.rt = u->ring_terminal;
    a.critic = u->critic; a.actors = u->actors; a.actors_target = u->actors_target; a.stride = u->actor_stride;
    a.gamma = u->gamma;
    a.invB = 1.0f / (float)u->B;
    a.gate = nullptr;  // only flock_sc_pipeline_learn gates a critic phase on its snapshot
    a.gate_seq = 0;
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
    BwdJob bw;
    GradAdam ga;
    bool free_dev;  // gated critic phase whose slot is freed on the device (gate[2], sc_gemm): FlockScPipeline.gseq
};

void job_common(const FlockScUpdate* u, Job& j) {
    j.B = u->B; j.in = u->in_dim; j.na = u->n_actions; j.H1 = u->fc1; j.H2 = u->fc2;
    ws_layout(j.B, j.in, j.na, j.H1, j.H2, u->workspace, &j.w);
    j.a = row_args(u);
    j.C = chunks(u);
    j.rb = (j.B + kRowsPerBlock - 1) / kRowsPerBlock;
    j.lds1 = fc1_lds(j.in, j.H1);
    j.lds3 = tails_lds(j.na, j.H2);
    j.free_dev = false;
}

// the bwd launch's job: dH1 = dZ2 W2 (+ LN1 epilogue), dW2 = dZ2^T H1, then the caller's early reductions
void bwd_common(Job& j, const float* W2, int64_t rel_w2, const int64_t* agent, const float* H1, const float* XH1,
                const float* g1, float* DY1, float* DXH1, float* PS1, const float* DZ2, int64_t w2_off, float* grad,
                int64_t rel, float* loss) {
    const int B = j.B, H1n = j.H1, H2 = j.H2;
    BwdJob& bw = j.bw;
    bw.dh = gemm_p(DZ2, W2, nullptr, nullptr, B, H1n, H2, H2, 1, H1n, 1, H1n, rel_w2, agent);
    bw.dw = gemm_p(DZ2, H1, nullptr, nullptr, H2, H1n, B, 1, H2, H1n, 1, H1n, 0);
    bw.dw.kchunk = balanced_kc(B, kGradKC);
    bw.H1 = H1; bw.XH1 = XH1; bw.g1 = g1; bw.DY1 = DY1; bw.DXH1 = DXH1; bw.PS1 = PS1;
    bw.F = H1n; bw.ntn = bw.dh.tiles_n;
    bw.w2_off = w2_off;
    bw.nred = 0; bw.nblk = 0; bw.B = B;
    bw.grad = grad; bw.rel = rel; bw.grad_rel = rel; bw.agent = agent; bw.agent_v = -1; bw.loss = loss;
}

// the late launch's job: fc1 / LN1 reductions (+ Adam), Adam of [W2, total)
void late_common(Job& j, const FlockScUpdate* u, const float* DXH1, const float* DY1, const float* XH1,
                 const float* RS1, const float* PS1, int64_t W1, int64_t b1, int64_t g1, int64_t be1, int64_t W2,
                 int64_t total) {
    const int in = j.in, H1 = j.H1;
    GradAdam& ga = j.ga;
    ga.nred = 0;
    ga.nblk = 0;
    ga.B = j.B;
    ga.do_adam = u->do_adam;
    add_red(ga, DXH1, H1, j.w.S, in, 4, in, H1 * in, W1);
    add_red(ga, DXH1, H1, nullptr, 0, 5, 1, H1, b1);
    add_red(ga, DY1, H1, XH1, H1, 1, 1, H1, g1);
    add_red(ga, DY1, H1, nullptr, 0, 0, 1, H1, be1);
    ga.dz = DzArgs{XH1, RS1, PS1, H1, j.bw.ntn};
    ga.adam_lo = W2;
    ga.adam_n = total - W2;
    ga.adam_blocks = u->do_adam ? (int)((ga.adam_n + 1023) / 1024) : 0;
    ga.lr = 0.0f;
    ga.grad_scale = nullptr;
    ga.b1 = u->beta1; ga.b2 = u->beta2; ga.eps = u->eps;
    ga.tau = u->tau;
    ga.one_minus_tau = (float)(1.0 - (double)u->tau);
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
    BwdJob& bw = j.bw;
    bwd_common(j, u->critic + co.W2, 0, u->agent, w.H1, w.XH1, u->critic + co.g1, w.DY1, w.DXH1, w.PS1, w.DZ2, co.W2,
               u->critic_grad, 0, u->losses + 1);
    add_red(bw, w.DZ2, H2, nullptr, 0, 0, 1, H2, co.b2);
    add_red(bw, w.DY2, H2, w.XH2, H2, 1, 1, H2, co.g2);
    add_red(bw, w.DY2, H2, nullptr, 0, 0, 1, H2, co.be2);
    add_red(bw, w.DZA, H2, w.A, na, 2, na, H2 * na, co.Wa);
    add_red(bw, w.DZA, H2, nullptr, 0, 0, 1, H2, co.ba);
    add_red(bw, w.DQ, 1, w.HQ, H2, 2, H2, H2, co.Wq);
    add_red(bw, w.DQ, 1, nullptr, 0, 0, 1, 1, co.bq);
    add_red(bw, w.LOSS, 1, nullptr, 0, 3, 1, 1, 0);
    late_common(j, u, w.DXH1, w.DY1, w.XH1, w.RS1, w.PS1, co.W1, co.b1, co.g1, co.be1, co.W2, co.total);
    GradAdam& ga = j.ga;
    ga.p = u->critic; ga.grad = u->critic_grad; ga.m = u->critic_exp_avg; ga.v = u->critic_exp_avg_sq;
    ga.rel = 0;
    ga.grad_rel = 0;
    ga.agent = u->agent;
    ga.agent_v = -1;
    ga.step = u->critic_step;
    ga.counter = u->counters;
    ga.lr = u->beta;
    ga.target = nullptr; ga.self_soft = nullptr; ga.self_n = 0; ga.soft_blocks = 0;
    // with a critic view the self soft update of this learn() rides in the critic's Adam (see FlockScUpdate)
    const bool view = u->do_adam && u->critic_view;
    ga.p_copy = view ? u->critic_view : nullptr;
    ga.soft_count = view ? u->actor_steps : nullptr;
    ga.soft_rate = view ? u->update_rate : 0;
}

// actor phase (:144-150), through the UPDATED critic (critic_view when given)
void actor_job(const FlockScUpdate* u, Job& j) {
    job_common(u, j);
    const int B = j.B, in = j.in, na = j.na, H1 = j.H1, H2 = j.H2;
    const Ws& w = j.w;
    const bool view = u->do_adam && u->critic_view;
    // the critic this actor step sees (post-Adam): the view whenever one is given (the data-parallel rounds compute
    // gradients with do_adam = 0 after an earlier flock_sc_round_adam wrote the view)
    float* const critic = u->critic_view ? u->critic_view : u->critic;
    j.a.critic = critic;
    const CriticOff co = critic_off(in, na, H1, H2);
    const ActorOff ao = actor_off(in, na, H1, H2);
    // fc2 of the actor and of the updated critic
    j.fwd[0] = gemm_p(w.AH1, u->actors + ao.W2, w.Z2b, u->actors + ao.b2, B, H2, H1, H1, 1, 1, H1, H2,
                      u->actor_stride, u->agent);
    j.fwd[1] = gemm_p(w.CH1, critic + co.W2, w.Z2b + (int64_t)B * H2, critic + co.b2, B, H2, H1, H1, 1, 1, H1, H2,
                      0);
    j.nfwd = 2;
    BwdJob& bw = j.bw;
    bwd_common(j, u->actors + ao.W2, u->actor_stride, u->agent, w.AH1, w.AXH1, u->actors + ao.g1, w.ADY1, w.ADXH1,
               w.APS1, w.ADZ2, ao.W2, u->actors_grad, u->actor_stride, u->losses);
    if (u->actor_grad_out) {  // this actor's gradient into the caller's bucket (not agent-relative)
        bw.grad = u->actor_grad_out;
        bw.grad_rel = 0;
    }
    add_red(bw, w.ADZ2, H2, nullptr, 0, 0, 1, H2, ao.b2);
    add_red(bw, w.ADY2, H2, w.AXH2, H2, 1, 1, H2, ao.g2);
    add_red(bw, w.ADY2, H2, nullptr, 0, 0, 1, H2, ao.be2);
    add_red(bw, w.DM, na, w.AH2, H2, 2, H2, na * H2, ao.Wmu);
    add_red(bw, w.DM, na, nullptr, 0, 0, 1, na, ao.bmu);
    add_red(bw, w.ALOSS, 1, nullptr, 0, 3, 1, 1, 0);
    late_common(j, u, w.ADXH1, w.ADY1, w.AXH1, w.ARS1, w.APS1, ao.W1, ao.b1, ao.g1, ao.be1, ao.W2, ao.total);
    GradAdam& ga = j.ga;
    ga.p = u->actors; ga.grad = u->actors_grad; ga.m = u->actors_exp_avg; ga.v = u->actors_exp_avg_sq;
    ga.rel = u->actor_stride;
    ga.grad_rel = u->actor_stride;
    if (u->actor_grad_out) {
        ga.grad = u->actor_grad_out;
        ga.grad_rel = 0;
    }
    ga.agent = u->agent;
    ga.agent_v = -1;
    ga.step = u->actor_steps;
    ga.counter = u->counters + 1;
    ga.lr = u->alpha;
    const bool soft = u->do_adam && u->update_rate > 0;
    ga.soft_rate = soft ? u->update_rate : 0;
    ga.target = soft ? u->actors_target : nullptr;  // agent-relative like p
    ga.self_soft = (soft && !view) ? u->critic : nullptr;  // with a view the critic kernel did it
    ga.self_n = co.total;
    ga.soft_blocks = (soft && !view) ? (int)((co.total + 1023) / 1024) : 0;
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

// The reference's production widths (fc1 400, fc2 300, 2 actions: agent_simple_shared_critic.py / train_flock.py
// defaults) get row kernels with compile-time widths: every per-lane column mask and action loop folds away
// (sc_k3 ~40 % fewer instructions per wave). flock_set_diag("sc_no_spec", 1) forces the generic instantiations
// (the bitwise A/B of tests/test_gpu_learners.py).
bool g_sc_no_spec = false;  // set by flock_sc_diag_no_spec (flock_set_diag)
bool spec_shape(const Job& j) { return !g_sc_no_spec && j.H1 == 400 && j.H2 == 300 && j.na == 2; }

// the fc2.weight panels a job's forward GEMMs read: the first problem's (the target actor / actor of the agent) and
// the second's (the critic, or the critic view the actor phase reads; the critic phase's third problem shares it)

// One round: the critic phase of one learn() (jc) and the actor phase of another (ja) in five launches; either may be
// NULL. The two jobs share no written state when they are of different agents (the caller's guarantee), so the round
// computes exactly what the actor phase followed by the critic phase would.

// a callback between the bwd launch and the gradient / Adam launch (data-parallel pipelines: the all-reduce of the
// critic gradient the bwd launch completed starts there, beside the gradient launch)
struct MidHook {
    int (*fn)(void*);
    void* ctx;
};
int launch_round(hipStream_t st, const Job* jc, const Job* ja, const MidHook* mid = nullptr) {
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
        if (spec_shape(A)) {
            if ((rc = allow_lds(sc_k1<7, 400>, lds))) return rc;
            hipLaunchKernelGGL((sc_k1<7, 400>), grid, dim3(256), lds, st, A.w, A.a, npc, Z.w, Z.a);
        } else {
            SC_C_SWITCH(C, if ((rc = allow_lds(sc_k1<CC, 0>, lds))) return rc;
                        hipLaunchKernelGGL((sc_k1<CC, 0>), grid, dim3(256), lds, st, A.w, A.a, npc, Z.w, Z.a))
        }
        if ((rc = launched())) return rc;
    }
    {  // 2: forward fc2 GEMMs
        GemmBatch gb;
        gb.n = 0;
        gb.done = (jc && jc->a.gate && jc->free_dev) ? jc->a.gate + 2 : nullptr;
        gb.done_seq = jc ? jc->a.gate_seq : 0;
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
        if (spec_shape(A)) {
            if ((rc = allow_lds(sc_k3<5, 300, 2>, lds))) return rc;
            hipLaunchKernelGGL((sc_k3<5, 300, 2>), grid, dim3(256), lds, st, A.w, A.a, nbc, Z.w, Z.a);
        } else {
            SC_C_SWITCH(C, if ((rc = allow_lds(sc_k3<CC, 0, 0>, lds))) return rc;
                        hipLaunchKernelGGL((sc_k3<CC, 0, 0>), grid, dim3(256), lds, st, A.w, A.a, nbc, Z.w, Z.a))
        }
        if ((rc = launched())) return rc;
    }
    {  // 4: dH1 = dZ2 W2 with the LN1-backward epilogue, dW2, early reductions
        Bwd2 bb;
        bb.j0 = A.bw;
        bb.j1 = Z.bw;
        bb.n0 = bwd_blocks(A.bw);
        bb.nb0 = (jc && ja) ? (bb.n0 + 7) & ~7 : bb.n0;
        const int nb = bb.nb0 + ((jc && ja) ? bwd_blocks(Z.bw) : 0);
        const size_t lds = zmax(bwd_lds(A.bw), bwd_lds(Z.bw));
        bool fast = true;
        int kh = 8, kw = 8;
        for (const BwdJob* b : {&A.bw, &Z.bw}) {
            fast = fast && gemm_variant(b->dh) == 1 && gemm_variant(b->dw) == 2;
            const int ch = gemm_kc(b->dh.K, b->dh.kchunk), cw = gemm_kc(b->dw.K, b->dw.kchunk);
            kh = ch > kh ? ch : kh;
            kw = cw > kw ? cw : kw;
        }
        const int nfh = nf_of(kh), nfw = nf_of(kw);
        const dim3 grid(nb);
        if (!fast)
            rc = launch_bwd_v<2, 2, 2, 2, 16, 16>(st, bb, grid, lds);
        else if (nfw <= 4)
            rc = nfh <= 4 ? launch_bwd_v<0, 1, 1, 1, 4, 4>(st, bb, grid, lds)
                          : nfh <= 7 ? launch_bwd_v<0, 1, 1, 1, 7, 4>(st, bb, grid, lds)
                                     : launch_bwd_v<0, 1, 1, 1, 16, 4>(st, bb, grid, lds);
        else
            rc = nfh <= 7 ? launch_bwd_v<0, 1, 1, 1, 7, 16>(st, bb, grid, lds)
                          : launch_bwd_v<0, 1, 1, 1, 16, 16>(st, bb, grid, lds);
        if (rc) return rc;
    }
    if (mid && (rc = mid->fn(mid->ctx))) return rc;
    // 5: fc1 / LN1 gradients + every Adam step
    if (A.ga.nblk > kMaxRedBlocks || Z.ga.nblk > kMaxRedBlocks || A.bw.nblk > kMaxRedBlocks)
        return fail(-2, "flock_sc: too many reduction blocks (fc1 * in_dim too large)");
    GradAdam2 gg;
    gg.j0 = A.ga;
    gg.j1 = Z.ga;
    gg.nb0 = late_blocks(A.ga);
    const int nb = gg.nb0 + ((jc && ja) ? late_blocks(Z.ga) : 0);
    const size_t lds = red_lds(A.B);
    if ((rc = allow_lds(sc_grad_adam, lds))) return rc;
    hipLaunchKernelGGL(sc_grad_adam, dim3(nb), dim3(256), lds, st, gg);
    return launched();
}

__global__ __launch_bounds__(256) void sc_prep(int B, int64_t rows, uint64_t seed, uint64_t counter, int64_t* idx,
                                               int64_t* agent_out, int64_t agent) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r == 0) *agent_out = agent;
    if (idx && r < B) idx[r] = sample_row(seed, counter, rows, r);
}

// learn() prologue with a minibatch snapshot: the sampled rows of every replay field are copied to staging rows
// 0..B-1, so the update can read the staging copy (with the identity index) while the next env step rewrites the ring.
// SC1: every staging store write-through (the device-side gate's producer, csrc/flock_mem.h)
template <bool SC1>
__device__ __forceinline__ void snapshot_row(int64_t rows, uint64_t seed, uint64_t counter, int64_t* idx_out,
                                             int in_dim, int n_actions, const FlockScRows& src,
                                             const FlockScRows& dst, int vec, int r) {
    const int64_t row = sample_row(seed, counter, rows, r);  // the row sc_prep samples for r
    if (idx_out) idx_out[r] = row;
    auto st = [](auto* p, auto v) {
        if constexpr (SC1)
            flock_mem::st_sc1(p, v);
        else
            *p = v;
    };
    // every load of the row first, then the stores (src and dst may alias as far as the compiler knows: interleaved,
    // each store would wait for its load, one memory round trip per field)
    if (vec) {  // the v2 shapes (in_dim 4, n_actions 2) with aligned fields: 16-B / 8-B rows
        const float4 s0 = *reinterpret_cast<const float4*>(src.state + row * 4);
        const float4 ns = *reinterpret_cast<const float4*>(src.new_state + row * 4);
        const float2 ac = *reinterpret_cast<const float2*>(src.action + row * 2);
        const float rw = src.reward[row], te = src.terminal[row];
        st(reinterpret_cast<float4*>(dst.state + (int64_t)r * 4), s0);
        st(reinterpret_cast<float4*>(dst.new_state + (int64_t)r * 4), ns);
        st(reinterpret_cast<float2*>(dst.action + (int64_t)r * 2), ac);
        st(dst.reward + r, rw);
        st(dst.terminal + r, te);
        return;
    }
    for (int c = 0; c < in_dim; ++c) {
        const float a = src.state[row * in_dim + c], b = src.new_state[row * in_dim + c];
        st(dst.state + (int64_t)r * in_dim + c, a);
        st(dst.new_state + (int64_t)r * in_dim + c, b);
    }
    for (int c = 0; c < n_actions; ++c) st(dst.action + (int64_t)r * n_actions + c, src.action[row * n_actions + c]);
    const float rw = src.reward[row], te = src.terminal[row];
    st(dst.reward + r, rw);
    st(dst.terminal + r, te);
}

__global__ __launch_bounds__(64) void sc_prep_snapshot(int B, int64_t rows, uint64_t seed, uint64_t counter,
                                                        int64_t* idx_out, int64_t* agent_out, int64_t agent,
                                                        int in_dim, int n_actions, FlockScRows src,
                                                        FlockScRows dst, int vec) {
    const int r = blockIdx.x * 64 + threadIdx.x;
    if (r == 0) *agent_out = agent;
    if (r < B) snapshot_row<false>(rows, seed, counter, idx_out, in_dim, n_actions, src, dst, vec, r);
}

// the same snapshot as ONE block that publishes it through the device-side gate: rows and agent stored `sc1`, every
// wave's stores waited for, a workgroup barrier, then one lane's `sc1` store of gate[0] = seq (csrc/flock_mem.h).
// reuse > 0: the slot's previous snapshot (that sequence number) must have been consumed first: one lane polls gate[2]
// (stored by that round's sc_gemm after its k1 launch, the staging rows' only reader) with `sc1` loads for at most
// ticks (s_memrealtime); a snapshot that gives up sets the error word and writes nothing
__global__ __launch_bounds__(256) void sc_prep_snapshot_gate(int B, int64_t rows, uint64_t seed, uint64_t counter,
                                                             int64_t* agent_out, int64_t agent, int in_dim,
                                                             int n_actions, FlockScRows src, FlockScRows dst, int vec,
                                                             unsigned long long* gate, unsigned long long seq,
                                                             unsigned long long reuse, unsigned long long ticks) {
    if (reuse && !gate_wait(gate + 2, reuse, gate + 1, ticks)) return;
    if (threadIdx.x == 0) flock_mem::st_sc1(agent_out, agent);
    for (int r = threadIdx.x; r < B; r += 256)
        snapshot_row<true>(rows, seed, counter, nullptr, in_dim, n_actions, src, dst, vec, r);
    flock_mem::wait_vmem();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(gate, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// the "sc_no_spec" diagnostics knob of flock_set_diag (flock_env.hip)
void flock_sc_diag_no_spec(bool v) { g_sc_no_spec = v; }
void flock_sc_diag_event_system(bool v);  // below (the pipeline's event flags)

int round_adam(void* stream, const FlockScUpdate* critic_u, const FlockScUpdate* actor_u, const float* grad_scale,
               int64_t agent_c, int64_t agent_a);
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
    int vec = in_dim == 4 && n_actions == 2;
    for (const FlockScRows* x : rs)
        vec = vec && al16(x->state) && al16(x->new_state) && (((uintptr_t)x->action & 7) == 0);
    hipLaunchKernelGGL(sc_prep_snapshot, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, B, rows, seed,
                       counter, idx_out, agent_out, agent, in_dim, n_actions, *ring, *staging, vec);
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

int flock_sc_round_adam(void* stream, const FlockScUpdate* critic_u, const FlockScUpdate* actor_u,
                        const float* grad_scale) {
    return round_adam(stream, critic_u, actor_u, grad_scale, -1, -1);
}
}  // extern "C"

// flock_sc_round_adam with the learns' agent indices by value when >= 0 (the pipeline's data-parallel rounds: the
// slot's agent word may already hold a later learn's agent, written by a snapshot released at this round's GEMM)
int round_adam(void* stream, const FlockScUpdate* critic_u, const FlockScUpdate* actor_u, const float* grad_scale,
               int64_t agent_c, int64_t agent_a) {
    if (!critic_u && !actor_u) return fail(-3, "flock_sc_round_adam: NULL argument");
    int rc = 0;
    if (critic_u && (rc = check(critic_u))) return rc;
    if (actor_u && (rc = check(actor_u))) return rc;
    if ((critic_u && !critic_u->do_adam) || (actor_u && !actor_u->do_adam))
        return fail(-5, "flock_sc_round_adam: the updates must have do_adam = 1");
    Job jc, ja;
    GradAdam* js[2] = {nullptr, nullptr};
    int n = 0;
    if (critic_u) {
        critic_job(critic_u, jc);
        js[n++] = &jc.ga;
    }
    if (actor_u) {
        actor_job(actor_u, ja);
        js[n++] = &ja.ga;
    }
    for (int i = 0; i < n; ++i) {  // Adam-only: no reductions, the whole parameter range from the gradient buffer
        GradAdam& g = *js[i];
        g.nred = 0;
        g.nblk = 0;
        g.adam_lo = 0;
        g.grad_scale = grad_scale;
    }
    if (critic_u) {
        const CriticOff co = critic_off(critic_u->in_dim, critic_u->n_actions, critic_u->fc1, critic_u->fc2);
        jc.ga.adam_n = co.total;
        jc.ga.adam_blocks = (int)((co.total + 1023) / 1024);
    }
    if (actor_u) {
        const ActorOff ao = actor_off(actor_u->in_dim, actor_u->n_actions, actor_u->fc1, actor_u->fc2);
        ja.ga.adam_n = ao.total;
        ja.ga.adam_blocks = (int)((ao.total + 1023) / 1024);
    }
    if (critic_u) jc.ga.agent_v = agent_c;
    if (actor_u) ja.ga.agent_v = agent_a;
    GradAdam2 gg;
    gg.j0 = *js[0];
    gg.j1 = *js[n - 1];
    gg.nb0 = late_blocks(gg.j0);
    const int nb = gg.nb0 + (n == 2 ? late_blocks(gg.j1) : 0);
    hipLaunchKernelGGL(sc_grad_adam, dim3(nb), dim3(256), 0, (hipStream_t)stream, gg);
    return launched();
}
extern "C" {

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
// launched directly from arguments built once per slot (round = critic phase of slot s + actor phase of the previous
// learn's slot: five hipLaunchKernel; replaying the same rounds from HIP graphs measured 0.125 against 0.117 ms per
// config-3 step in round 2, so there is no graph path).
constexpr int kMaxSlots = 8;
struct FlockScPipeline {
    int n;
    FlockScUpdate u[kMaxSlots];
    FlockScRows ring, staging[kMaxSlots];
    Job jc[kMaxSlots], ja[kMaxSlots];  // the rounds' launch arguments, built once
    hipEvent_t snap_done[kMaxSlots];
    // device-side snapshot gate: gate[0] the published sequence number, gate[1] the error word of a waiter that gave
    // up; seq counts this pipeline's snapshots. gate_on: the critic phase's row blocks poll gate[0] (single GPU and
    // data-parallel rounds alike; never under counter collection); otherwise the learner stream waits for each snapshot
    // on a cross-queue event.
    unsigned long long* gate;
    unsigned long long seq;
    bool gate_on;
    // the gate's guard (flock_sc_pipeline_mark): a learn() is gated only when the caller marked the env stream since
    // the previous learn(): mark 2 = the round first waits (cross-queue, usually already complete) for mark_ev, recorded
    // behind everything the env stream held then; 1 = the caller declared that only its own env step was enqueued since
    // the previous snapshot; 0 = no mark: the event hand-off, so that no round ever spins on work of unknown length
    hipEvent_t mark_ev;
    int mark;
    int64_t gated_learns;  // learns that took the gate (the rest: the event hand-off)
    // slot reuse: the "free point" of a slot is where its last learn's actor phase has been enqueued on the learner
    // stream (one point per learn, in order); the env stream waits for it before the slot's next snapshot. An event is
    // recorded only at every free_every-th point (each record is a barrier packet between two rounds on the learner
    // stream, and each wait one on the env stream): a reuse waits for the first recorded point at or after its own,
    // which n_slots >= free_every + 1 guarantees is already enqueued (else a fresh event on the learner stream)
    int free_every;
    int64_t points;               // free points emitted so far
    int64_t slot_point[kMaxSlots];
    static constexpr int kRec = 16;
    hipEvent_t rec_ev[kRec];
    int64_t rec_pt[kRec];
    hipEvent_t fresh_ev;
    // slots freed on the device (single-GPU gated learns, g_sc_free_events off): gseq[s] = the snapshot sequence
    // number of slot s's last learn when that learn was gated (0: it took the event hand-off). Its round's sc_gemm
    // stores that number to gate[2] once its k1 launch, the only reader of the staging rows, has completed, and the
    // slot's next gated snapshot polls gate[2] before writing (sc_prep_snapshot_gate): no free-point event between
    // the rounds on the learner stream and no cross-queue wait on the env stream
    unsigned long long gseq[kMaxSlots];
    bool used[kMaxSlots];
    int slot;
    int pending;  // slot of the learn() whose actor phase is not enqueued yet, or -1
    int64_t pending_agent;
    // data-parallel rounds (flock_sc_pipeline_set_dp): gradients into the bucket, the caller's all-reduce of the part a
    // round wrote, then the Adam launch with grad_scale
    bool dp;
    FlockScUpdate ug[kMaxSlots], uadam[kMaxSlots];
    Job jgc[kMaxSlots], jga[kMaxSlots];  // the gradient rounds' launch arguments (ug), built once
    float* bucket;
    int64_t actor_off, bucket_floats, critic_floats;
    const float* grad_scale;
    FlockAllreduceFn allreduce;
    void* allreduce_ctx;
    // the actor half off the learner chain (flock_sc_pipeline_set_dp_actor): each slot's actor gradient in a buffer of
    // its own, all-reduced and stepped on actor_stream through the second callback
    bool split;
    hipStream_t actor_stream;
    hipEvent_t grads_done[kMaxSlots], actor_done[kMaxSlots], actor_joined;
    // split rounds: the critic gradient's [fc2.weight .. q.bias] part (complete after the bwd launch) is all-reduced on
    // comm_stream beside the gradient launch; only the fc1 / LN1 part ([0, critic_w2)) follows the gradient launch
    hipStream_t comm_stream;
    hipEvent_t bwd_done, ar_done;
    int64_t critic_w2;
    bool actor_used[kMaxSlots];
    int64_t actor_floats;
    FlockAllreduceFn actor_allreduce;
    void* actor_ctx;
    int n_agents;
    int* last_actor_slot;  // [n_agents]: the slot of the agent's last actor step on actor_stream, -1: none
};

namespace {
// The pipeline's events order work between its streams on ONE device (slot reuse, snapshot hand-offs, the guard
// mark, the split rounds' actor stream): a device-scope release is all they need. HIP's default event is a system-scope
// sequentially consistent fence when it is recorded (a cache writeback and invalidation behind the round the event
// follows: the next round's kernels then start from a cold L2). flock_set_diag("sc_event_system_scope", 1) restores the
// default for A/B (read when a pipeline is created).
bool g_sc_event_system = false;
// flock_set_diag("sc_free_events", 1): every slot freed by a learner-stream event (the round-5 scheme; A/B)
bool g_sc_free_events = false;
unsigned pipeline_event_flags() {
    return hipEventDisableTiming | (g_sc_event_system ? 0u : (unsigned)hipEventReleaseToDevice);
}
bool counter_collection() {  // rocprofv3 counter collection serialises dispatches: no spinning consumers under it
    const char* pmc = getenv("ROCPROF_COUNTER_COLLECTION");
    return pmc && pmc[0] && pmc[0] != '0';
}

// the learner stream waits for an event unless the host already sees it complete (a completed event's writes are
// visible to every later launch: the producer kernel's end released them)
int wait_unless_done(hipStream_t st, hipEvent_t ev) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return fail(-4, "flock_sc_pipeline: event query");
    return hipStreamWaitEvent(st, ev, 0) == hipSuccess ? 0 : fail(-4, "flock_sc_pipeline: stream wait");
}

// the actor step of `agent` that is still in flight on actor_stream (split data-parallel rounds): every reader of
// that agent's actor, target actor, moments or step count on the learner stream waits for it
int wait_actor(FlockScPipeline* p, hipStream_t ls, int64_t agent) {
    if (!p->last_actor_slot || agent < 0 || agent >= p->n_agents) return 0;
    const int s = p->last_actor_slot[agent];
    return s >= 0 ? wait_unless_done(ls, p->actor_done[s]) : 0;
}

// one round of the pipeline on stream ls: critic phase of slot c and / or actor phase of slot a (-1: none);
// agents: the learns' agent indices (split data-parallel rounds)
// the early part of a split round's critic all-reduce (MidHook): the bwd launch has completed the critic gradient's
// [fc2.weight, total) part; it is all-reduced on comm_stream while the gradient launch runs on the learner stream
struct EarlyAr {
    FlockScPipeline* p;
    hipStream_t ls;
};
int early_critic_allreduce(void* ctx) {
    const EarlyAr& e = *static_cast<EarlyAr*>(ctx);
    FlockScPipeline* p = e.p;
    if (hipEventRecord(p->bwd_done, e.ls) != hipSuccess || hipStreamWaitEvent(p->comm_stream, p->bwd_done, 0) != hipSuccess)
        return fail(-4, "flock_sc_pipeline: stream operation failed");
    if (int rc = p->allreduce(p->allreduce_ctx, p->bucket + p->critic_w2, p->critic_floats - p->critic_w2, p->comm_stream))
        return fail(rc < 0 ? rc : -4, "flock_sc_pipeline: the all-reduce callback failed");
    return hipEventRecord(p->ar_done, p->comm_stream) == hipSuccess ? 0 : fail(-4, "flock_sc_pipeline: event record");
}

// a job with its agent index as a value (the pipeline's learns know theirs: every kernel of the round computes the
// agent's parameter addresses without first loading the index). Same-box A/B against the device-word reads
// (profiles/r05/agentv/): driver command 0.0897-0.0904 vs 0.0908-0.0920, 200 steps 0.0809-0.0819 vs 0.0803-0.0815 ms
// per step: within the noise either way
Job with_agent(const Job& j0, int64_t agent) {
    Job j = j0;
    j.a.agent_v = agent;
    for (int i = 0; i < j.nfwd; ++i) j.fwd[i].agent_v = agent;
    j.bw.dh.agent_v = agent;
    j.bw.dw.agent_v = agent;
    j.bw.agent_v = agent;
    j.ga.agent_v = agent;
    return j;
}

// one round of the pipeline on stream ls: critic phase of slot c and / or actor phase of slot a (-1: none);
// agents: the learns' agent indices (split data-parallel rounds)
int pipeline_round(FlockScPipeline* p, hipStream_t ls, int c, int a, int64_t agent_c, int64_t agent_a) {
    if (!p->dp) {
        Job jc, ja;
        if (c >= 0) jc = with_agent(p->jc[c], agent_c);
        if (a >= 0) ja = with_agent(p->ja[a], agent_a);
        return launch_round(ls, c >= 0 ? &jc : nullptr, a >= 0 ? &ja : nullptr);
    }
    int rc = 0;
    Job jgc, jga;
    if (c >= 0) jgc = with_agent(p->jgc[c], agent_c);
    if (a >= 0) jga = with_agent(p->jga[a], agent_a);
    const Job* gc = c >= 0 ? &jgc : nullptr;
    const Job* ga = a >= 0 ? &jga : nullptr;
    if (!p->split) {
        // gradients only (do_adam = 0) into the bucket, ONE all-reduce (sum) of the part they wrote, then the Adam
        // launch (gradients scaled by *grad_scale): SharedCriticLearner._dp_round
        if ((rc = launch_round(ls, gc, ga))) return rc;
        const int64_t lo = c >= 0 ? 0 : p->actor_off, hi = a >= 0 ? p->bucket_floats : p->critic_floats;
        if ((rc = p->allreduce(p->allreduce_ctx, p->bucket + lo, hi - lo, ls)))
            return fail(rc < 0 ? rc : -4, "flock_sc_pipeline: the all-reduce callback failed");
        return round_adam(ls, c >= 0 ? &p->uadam[c] : nullptr, a >= 0 ? &p->uadam[a] : nullptr, p->grad_scale,
                          agent_c, agent_a);
    }
    // split: the critic half stays on the learner chain (the next critic phase needs this critic step), its larger
    // part all-reduced beside the gradient launch; the actor half is all-reduced and stepped on actor_stream (that
    // actor is read again only by its agent's next learn)
    if ((rc = wait_actor(p, ls, agent_c))) return rc;
    if (a >= 0 && p->actor_used[a] && (rc = wait_unless_done(ls, p->actor_done[a]))) return rc;  // slot a's buffer
    EarlyAr ear{p, ls};
    const MidHook mid{&early_critic_allreduce, &ear};
    if ((rc = launch_round(ls, gc, ga, c >= 0 ? &mid : nullptr))) return rc;
    if (a >= 0) {
        hipStream_t as = p->actor_stream;
        if (hipEventRecord(p->grads_done[a], ls) != hipSuccess || hipStreamWaitEvent(as, p->grads_done[a], 0) != hipSuccess)
            return fail(-4, "flock_sc_pipeline: stream operation failed");
        if ((rc = p->actor_allreduce(p->actor_ctx, p->ug[a].actor_grad_out, p->actor_floats, as)))
            return fail(rc < 0 ? rc : -4, "flock_sc_pipeline: the actor all-reduce callback failed");
        if ((rc = flock_sc_round_adam(as, nullptr, &p->uadam[a], p->grad_scale))) return rc;
        if (hipEventRecord(p->actor_done[a], as) != hipSuccess) return fail(-4, "flock_sc_pipeline: event record");
        p->actor_used[a] = true;
        p->last_actor_slot[agent_a] = a;
    }
    if (c >= 0) {
        if ((rc = p->allreduce(p->allreduce_ctx, p->bucket, p->critic_w2, ls)))
            return fail(rc < 0 ? rc : -4, "flock_sc_pipeline: the all-reduce callback failed");
        if (hipStreamWaitEvent(ls, p->ar_done, 0) != hipSuccess) return fail(-4, "flock_sc_pipeline: stream wait");
        if ((rc = flock_sc_round_adam(ls, &p->uadam[c], nullptr, p->grad_scale))) return rc;
    }
    return 0;
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
    int rc = 0;
    for (int i = 0; i < n_slots && !rc; ++i) {
        p->u[i] = slots[i];
        p->staging[i] = staging[i];
        critic_job(&p->u[i], p->jc[i]);
        actor_job(&p->u[i], p->ja[i]);
        hipEvent_t* evs[3] = {&p->snap_done[i], &p->grads_done[i], &p->actor_done[i]};
        for (hipEvent_t* e : evs)
            if (!rc && hipEventCreateWithFlags(e, pipeline_event_flags()) != hipSuccess)
                rc = fail(-4, "flock_sc_pipeline_create: event");
        p->used[i] = false;
        p->actor_used[i] = false;
    }
    p->slot = 0;
    p->pending = -1;
    p->pending_agent = -1;
    p->dp = false;
    p->split = false;
    p->actor_stream = nullptr;
    p->actor_joined = nullptr;
    p->comm_stream = nullptr;
    p->bwd_done = p->ar_done = nullptr;
    p->critic_w2 = 0;
    p->last_actor_slot = nullptr;
    p->n_agents = 0;
    p->gate = nullptr;
    p->seq = 0;
    p->gate_on = false;
    p->mark = 0;
    p->gated_learns = 0;
    p->mark_ev = nullptr;
    p->free_every = n_slots >= 5 ? (n_slots - 1) / 2 : 1;
    p->points = 0;
    p->fresh_ev = nullptr;
    for (int i = 0; i < kMaxSlots; ++i) {
        p->slot_point[i] = -1;
        p->gseq[i] = 0;
    }
    for (int i = 0; i < FlockScPipeline::kRec; ++i) {
        p->rec_ev[i] = nullptr;
        p->rec_pt[i] = -1;
        if (!rc && hipEventCreateWithFlags(&p->rec_ev[i], pipeline_event_flags()) != hipSuccess)
            rc = fail(-4, "flock_sc_pipeline_create: event");
    }
    if (!rc && hipEventCreateWithFlags(&p->fresh_ev, pipeline_event_flags()) != hipSuccess)
        rc = fail(-4, "flock_sc_pipeline_create: event");
    if (!rc && hipEventCreateWithFlags(&p->mark_ev, pipeline_event_flags()) != hipSuccess)
        rc = fail(-4, "flock_sc_pipeline_create: event");
    if (!rc && (hipMalloc(&p->gate, 4 * sizeof(unsigned long long)) != hipSuccess ||
                hipMemset(p->gate, 0, 4 * sizeof(unsigned long long)) != hipSuccess ||
                hipDeviceSynchronize() != hipSuccess))
        rc = fail(-4, "flock_sc_pipeline_create: gate");
    if (!rc) (void)flock_sc_pipeline_set_gate(p, 1);  // the default hand-off
    if (rc) {
        flock_sc_pipeline_destroy(p);
        return nullptr;
    }
    return p;
}

int flock_sc_pipeline_set_gate(FlockScPipeline* p, int on) {
    if (!p) return fail(-3, "flock_sc_pipeline_set_gate: NULL pipeline");
    p->gate_on = on != 0 && p->gate && !counter_collection();
    return p->gate_on ? 1 : 0;
}

int flock_sc_pipeline_mark(FlockScPipeline* p, void* env_stream, int wait) {
    if (!p) return fail(-3, "flock_sc_pipeline_mark: NULL pipeline");
    if (wait) {
        if (hipEventRecord(p->mark_ev, (hipStream_t)env_stream) != hipSuccess)
            return fail(-4, "flock_sc_pipeline_mark: event record");
        p->mark = 2;
    } else if (p->mark == 0) {
        p->mark = 1;
    }
    return 0;
}

namespace {
// slot q is free once everything enqueued on ls so far has run (its last learn's actor phase is enqueued): one free
// point; an event on every free_every-th point only
int emit_free_point(FlockScPipeline* p, hipStream_t ls, int q) {
    const int64_t j = p->points++;
    p->slot_point[q] = j;
    if (j % p->free_every != p->free_every - 1) return 0;
    const int k = (int)((j / p->free_every) % FlockScPipeline::kRec);
    p->rec_pt[k] = j;
    return hipEventRecord(p->rec_ev[k], ls) == hipSuccess ? 0 : fail(-4, "flock_sc_pipeline: event record");
}
// the env stream waits until slot s is free: for the first recorded free point at or after the slot's, or (none
// recorded yet) for everything the learner stream holds now
int wait_slot_free(FlockScPipeline* p, hipStream_t es, hipStream_t ls, int s) {
    const int64_t P = p->slot_point[s];
    if (P < 0) return 0;
    const int64_t j = P + (p->free_every - 1 - P % p->free_every);  // the first recorded point >= P
    const int k = (int)((j / p->free_every) % FlockScPipeline::kRec);
    hipEvent_t ev = p->fresh_ev;
    if (j < p->points && p->rec_pt[k] == j)
        ev = p->rec_ev[k];
    else if (hipEventRecord(p->fresh_ev, ls) != hipSuccess)
        return fail(-4, "flock_sc_pipeline: event record");
    return hipStreamWaitEvent(es, ev, 0) == hipSuccess ? 0 : fail(-4, "flock_sc_pipeline_learn: wait");
}

// the rounds of a learn() whose critic phase (slot s) reads inputs the learner stream can use (after its event wait
// or its row blocks' gate): the critic phase of s beside the actor phase of the previous learn, or one after the other
// (same agent)
int enqueue_rounds(FlockScPipeline* p, hipStream_t ls, int s, int64_t agent) {
    const int n = p->n;
    int rc = 0;
    const int q = p->pending;
    if (q >= 0 && q == (s + n - 1) % n && p->pending_agent != agent) {
        // the actor phase of the previous learn() beside this critic phase (different agents: no shared state)
        if ((rc = pipeline_round(p, ls, s, q, agent, p->pending_agent))) return rc;
        if (!p->gseq[q] && (rc = emit_free_point(p, ls, q))) return rc;
    } else {
        // same agent (this critic phase reads the target actor that actor phase soft-updates): one after the other
        if (q >= 0) {
            if ((rc = pipeline_round(p, ls, -1, q, -1, p->pending_agent))) return rc;
            if (!p->gseq[q] && (rc = emit_free_point(p, ls, q))) return rc;
        }
        if ((rc = pipeline_round(p, ls, s, -1, agent, -1))) return rc;
    }
    p->pending = s;
    p->pending_agent = agent;
    p->used[s] = true;
    p->slot = (s + 1) % n;
    return 0;
}
}  // namespace

int flock_sc_pipeline_learn(FlockScPipeline* p, void* env_stream, void* learner_stream, int64_t rows, uint64_t seed,
                            uint64_t counter, int64_t agent) {
    if (!p) return fail(-3, "flock_sc_pipeline_learn: NULL pipeline");
    if (rows < 1 || agent < 0) return fail(-5, "flock_sc_pipeline_learn: need rows >= 1 and an agent");
    if (p->last_actor_slot && agent >= p->n_agents) return fail(-5, "flock_sc_pipeline_learn: agent out of range");
    hipStream_t es = (hipStream_t)env_stream, ls = (hipStream_t)learner_stream;
    const int s = p->slot;
    const FlockScUpdate& u = p->u[s];
    int rc = 0;
    const int mark = p->mark;
    p->mark = 0;
    const bool gated = p->gate_on && mark;
    // slot reuse (the previous learn's snapshot in this slot consumed): on the device when both learns are gated,
    // else an event (and always an event for split data-parallel rounds, whose actor halves run on a stream of their
    // own). Every launch of a round after its k1 launch gets the learns' agent indices by value (with_agent, and
    // round_adam for the data-parallel Adam launch), since the snapshot released at the GEMM rewrites the slot's agent
    // word. Data-parallel rounds: the consuming round's GEMM may sit behind an all-reduce that waits for the other
    // ranks, so the poll's bound is 60 s there (a collective that never completes hangs the ranks anyway)
    const bool dev_free = gated && !g_sc_free_events && !(p->dp && p->split);
    const unsigned long long ticks = p->dp ? 30 * kGateTimeoutTicks : kGateTimeoutTicks;
    const unsigned long long reuse = (p->used[s] && dev_free) ? p->gseq[s] : 0;
    if (p->used[s] && !reuse) {
        if (p->gseq[s]) {  // a gated learn freed on the device, reused now by the event path: everything enqueued so far
            if (hipEventRecord(p->fresh_ev, ls) != hipSuccess || hipStreamWaitEvent(es, p->fresh_ev, 0) != hipSuccess)
                return fail(-4, "flock_sc_pipeline_learn: stream operation failed");
        } else if ((rc = wait_slot_free(p, es, ls, s))) {
            return rc;
        }
    }
    p->gseq[s] = 0;
    if (gated) {
        // the snapshot publishes gate[0] = seq after its write-through stores; this learn's critic row blocks wait
        // for it on the device. No deadlock whatever the streams' hardware queues: the snapshot is enqueued before
        // the round that waits for it, and nothing on the env stream waits for that round. The guard: the learner
        // stream first waits (cross-queue, without occupying a CU) for the caller's mark, so the row blocks spin only
        // over the env work enqueued since the mark (the caller's own env step), never behind a backlog of unknown
        // length; with mark 1 the caller declared that nothing else was enqueued since the previous snapshot
        if (mark == 2 && (rc = wait_unless_done(ls, p->mark_ev))) return rc;
        ++p->gated_learns;
        const FlockScRows& src = p->ring;
        const FlockScRows& dst = p->staging[s];
        int vec = u.in_dim == 4 && u.n_actions == 2;
        for (const FlockScRows* x : {&src, &dst})
            vec = vec && al16(x->state) && al16(x->new_state) && (((uintptr_t)x->action & 7) == 0);
        const unsigned long long seq = ++p->seq;
        hipLaunchKernelGGL(sc_prep_snapshot_gate, dim3(1), dim3(256), 0, es, u.B, rows, seed, counter,
                           const_cast<int64_t*>(u.agent), agent, u.in_dim, u.n_actions, src, dst, vec, p->gate, seq,
                           reuse, ticks);
        if ((rc = launched())) return rc;
        p->jc[s].a.gate = p->jgc[s].a.gate = p->gate;
        p->jc[s].a.gate_seq = p->jgc[s].a.gate_seq = seq;
        p->jc[s].free_dev = p->jgc[s].free_dev = dev_free;
        if (dev_free) p->gseq[s] = seq;
    } else {
        if ((rc = flock_sc_prep_snapshot(es, u.B, rows, seed, counter, nullptr, const_cast<int64_t*>(u.agent), agent,
                                         u.in_dim, u.n_actions, &p->ring, &p->staging[s])))
            return rc;
        p->jc[s].a.gate = p->jgc[s].a.gate = nullptr;
        p->jc[s].free_dev = p->jgc[s].free_dev = false;
        if (hipEventRecord(p->snap_done[s], es) != hipSuccess || hipStreamWaitEvent(ls, p->snap_done[s], 0) != hipSuccess)
            return fail(-4, "flock_sc_pipeline_learn: stream operation failed");
    }
    return enqueue_rounds(p, ls, s, agent);
}

int flock_sc_pipeline_set_dp(FlockScPipeline* p, float* bucket, int64_t critic_floats, int64_t actor_offset,
                             int64_t bucket_floats, const float* grad_scale, FlockAllreduceFn allreduce, void* ctx) {
    if (!p || !bucket || !allreduce) return fail(-3, "flock_sc_pipeline_set_dp: NULL argument");
    if (p->used[0] || p->pending >= 0) return fail(-5, "flock_sc_pipeline_set_dp: the pipeline has already learned");
    const FlockScUpdate& u0 = p->u[0];
    const int64_t ct = critic_off(u0.in_dim, u0.n_actions, u0.fc1, u0.fc2).total;
    const int64_t at = actor_off(u0.in_dim, u0.n_actions, u0.fc1, u0.fc2).total;
    if (critic_floats < ct || actor_offset < critic_floats || bucket_floats < actor_offset + at)
        return fail(-5, "flock_sc_pipeline_set_dp: the bucket must hold [critic gradient | actor gradient]");
    if (((uintptr_t)(bucket + actor_offset) & 15) != 0)
        return fail(-5, "flock_sc_pipeline_set_dp: the actor part of the bucket must be 16-B aligned");
    p->dp = true;
    p->bucket = bucket;
    p->critic_floats = critic_floats;
    p->actor_off = actor_offset;
    p->bucket_floats = bucket_floats;
    p->grad_scale = grad_scale;
    p->allreduce = allreduce;
    p->allreduce_ctx = ctx;
    for (int i = 0; i < p->n; ++i) {
        FlockScUpdate a = p->u[i];
        a.critic_grad = bucket;
        a.actor_grad_out = bucket + actor_offset;
        p->uadam[i] = a;  // do_adam = 1, the slot's update_rate: flock_sc_round_adam
        a.do_adam = 0;
        a.update_rate = 0;
        p->ug[i] = a;  // the gradient round
        critic_job(&p->ug[i], p->jgc[i]);
        actor_job(&p->ug[i], p->jga[i]);
    }
    return 0;
}

int flock_sc_pipeline_set_dp_actor(FlockScPipeline* p, float* const* actor_grads, int n_agents,
                                   FlockAllreduceFn allreduce, void* ctx) {
    if (!p || !actor_grads || !allreduce) return fail(-3, "flock_sc_pipeline_set_dp_actor: NULL argument");
    if (!p->dp) return fail(-5, "flock_sc_pipeline_set_dp_actor: call flock_sc_pipeline_set_dp first");
    if (p->used[0] || p->pending >= 0) return fail(-5, "flock_sc_pipeline_set_dp_actor: the pipeline has already learned");
    if (n_agents < 1) return fail(-5, "flock_sc_pipeline_set_dp_actor: n_agents >= 1");
    const FlockScUpdate& u0 = p->u[0];
    for (int i = 0; i < p->n; ++i) {
        if (!actor_grads[i] || ((uintptr_t)actor_grads[i] & 15) != 0)
            return fail(-5, "flock_sc_pipeline_set_dp_actor: one 16-B aligned actor gradient buffer per slot");
        for (int j = 0; j < i; ++j)
            if (actor_grads[i] == actor_grads[j])
                return fail(-5, "flock_sc_pipeline_set_dp_actor: the slots' buffers must differ");
    }
    if (!p->actor_stream && (hipStreamCreateWithFlags(&p->actor_stream, hipStreamNonBlocking) != hipSuccess ||
                             hipEventCreateWithFlags(&p->actor_joined, pipeline_event_flags()) != hipSuccess))
        return fail(-4, "flock_sc_pipeline_set_dp_actor: stream");
    delete[] p->last_actor_slot;
    p->last_actor_slot = new int[n_agents];
    for (int i = 0; i < n_agents; ++i) p->last_actor_slot[i] = -1;
    p->n_agents = n_agents;
    p->actor_floats = actor_off(u0.in_dim, u0.n_actions, u0.fc1, u0.fc2).total;
    if (!p->comm_stream && (hipStreamCreateWithFlags(&p->comm_stream, hipStreamNonBlocking) != hipSuccess ||
                            hipEventCreateWithFlags(&p->bwd_done, pipeline_event_flags()) != hipSuccess ||
                            hipEventCreateWithFlags(&p->ar_done, pipeline_event_flags()) != hipSuccess))
        return fail(-4, "flock_sc_pipeline_set_dp_actor: stream");
    p->critic_w2 = critic_off(u0.in_dim, u0.n_actions, u0.fc1, u0.fc2).W2;
    for (int i = 0; i < p->n; ++i) {
        p->ug[i].actor_grad_out = actor_grads[i];
        p->uadam[i].actor_grad_out = actor_grads[i];
        actor_job(&p->ug[i], p->jga[i]);
    }
    p->actor_allreduce = allreduce;
    p->actor_ctx = ctx;
    p->split = true;
    return 0;
}

int flock_sc_pipeline_flush(FlockScPipeline* p, void* learner_stream) {
    if (!p) return fail(-3, "flock_sc_pipeline_flush: NULL pipeline");
    hipStream_t ls = (hipStream_t)learner_stream;
    const int q = p->pending;
    if (q >= 0) {
        if (int rc = pipeline_round(p, ls, -1, q, -1, p->pending_agent)) return rc;
        if (int rc = p->gseq[q] ? 0 : emit_free_point(p, ls, q)) return rc;
        p->pending = -1;
    }
    // split rounds: the learner stream joins the actor stream, so synchronising the learner stream covers every step
    if (p->split && (hipEventRecord(p->actor_joined, p->actor_stream) != hipSuccess ||
                     hipStreamWaitEvent(ls, p->actor_joined, 0) != hipSuccess))
        return fail(-4, "flock_sc_pipeline_flush: stream operation failed");
    return 0;
}

#ifdef FLOCK_SC_PROF
// diagnostics build only: copy out the per-block times of the last launch of each round kernel / the GEMM marks
int flock_sc_prof_read(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_scprof), sizeof(g_scprof)) != hipSuccess;
}
int flock_sc_mark_read(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_scmark), sizeof(g_scmark)) != hipSuccess;
}
#endif

int flock_sc_pipeline_check(FlockScPipeline* p) {
    if (!p) return fail(-3, "flock_sc_pipeline_check: NULL pipeline");
    if (!p->gate) return 0;
    unsigned long long flag = 0;
    if (hipMemcpy(&flag, p->gate + 1, sizeof(flag), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(-4, "flock_sc_pipeline_check: copy failed");
    return flag ? fail(-6, "flock_sc_pipeline: a learn() round gave up waiting for its minibatch snapshot (device gate "
                           "timeout); its results are invalid")
                : 0;
}

int flock_sc_pipeline_gated(const FlockScPipeline* p) { return p && p->gate_on ? 1 : 0; }

}  // extern "C"
void flock_sc_diag_event_system(bool v) { g_sc_event_system = v; }
void flock_sc_diag_free_events(bool v) { g_sc_free_events = v; }
extern "C" {

void* flock_sc_pipeline_comm_stream(const FlockScPipeline* p) { return p ? (void*)p->comm_stream : nullptr; }

int64_t flock_sc_pipeline_gated_learns(const FlockScPipeline* p) { return p ? p->gated_learns : 0; }

void flock_sc_pipeline_destroy(FlockScPipeline* p) {
    if (!p) return;
    if (p->gate) (void)hipFree(p->gate);
    if (p->actor_stream) (void)hipStreamDestroy(p->actor_stream);
    if (p->actor_joined) (void)hipEventDestroy(p->actor_joined);
    if (p->comm_stream) (void)hipStreamDestroy(p->comm_stream);
    if (p->bwd_done) (void)hipEventDestroy(p->bwd_done);
    if (p->ar_done) (void)hipEventDestroy(p->ar_done);
    if (p->mark_ev) (void)hipEventDestroy(p->mark_ev);
    if (p->fresh_ev) (void)hipEventDestroy(p->fresh_ev);
    for (hipEvent_t e : p->rec_ev)
        if (e) (void)hipEventDestroy(e);
    delete[] p->last_actor_slot;
    for (int i = 0; i < p->n; ++i) {
        hipEvent_t* evs[3] = {&p->snap_done[i], &p->grads_done[i], &p->actor_done[i]};
        for (hipEvent_t* e : evs)
            if (*e) (void)hipEventDestroy(*e);
    }
    delete p;
}

}  // extern "C"
