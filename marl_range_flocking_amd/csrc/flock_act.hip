// Batched shared-critic acting on MI355X (gfx950): choose_action of EVERY agent for EVERY env row in one launch.
//
// Reference: learners/maddpg_shared_critic/agent_simple_shared_critic.py:92-107 (Agent.choose_action: mu = actor(obs)
// + noise()), the actor of ddpg_network.py:132-141 (fc1 -> LayerNorm -> ReLU -> fc2 -> LayerNorm -> ReLU -> mu ->
// tanh) and OUActionNoiseGPU.__call__ (utils.py:15-18: x = x_prev + theta (mu - x_prev) dt + sigma sqrt(dt) N(0,1),
// mu = 0, one process per (env, agent) here). The reference calls choose_action once per agent per env step on one
// env; the training loop at the bench's size (4096 envs x 256 agents) needs 1M actor evaluations per step.
//
// One block = one agent x 64 env rows (4 waves). The work is fc2: [64 x fc1] x [fc1 x fc2] per block, on
// v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate: no reduced precision anywhere). Nothing but the 16-B observation
// rows and the 8-B actions touches HBM per (row, agent):
//   * the A operand (the fc1 -> LayerNorm -> ReLU activations) is never stored: each lane recomputes its 4 values of
//     a k-step from the row's observation (in registers), fc1's 4-float weight rows and LayerNorm affine (LDS
//     broadcast reads) and the row's LayerNorm statistics (a prologue over all fc1 outputs of the block's rows);
//   * the B operand (fc2.weight, [fc2][fc1] row-major = contiguous along k) is read straight from global memory as
//     one float4 per lane per tile per k-step, one k-step ahead of the MFMAs; the lanes' k assignment (lane half h
//     takes k0 + 4h .. k0 + 4h + 3, MFMA s of the step pairs k0 + s with k0 + 4 + s) makes both operands contiguous;
//   * the fc2 outputs stay in the accumulators: LayerNorm (row sums by a 32-lane xor butterfly and one LDS
//     exchange between the two waves covering a row), ReLU, the 2-wide mu head and tanh run in the epilogue;
//   * XCD-aware work order: the blocks of one agent run on one XCD (block b -> work (b % 8) * W/8 + b / 8), so its
//     fc2.weight (480 KB at 400 x 300) is fetched into that XCD's L2 once and read by its 64 row tiles from there.
// The OU step and the noisy action are computed in the epilogue in the torch op order of choose_action
// (learners/shared_critic.py), bit for bit: the noise z is drawn by the caller (torch.randn on its generator).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "flock_learn.h"
#include "learn_internal.h"

using flock_learn_internal::fail;
using flock_learn_internal::launched;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// env rows per block: TM = 64 (two 32-row bands, 4 waves); 128-row blocks (four bands, every staged fc2.weight chunk read
// by twice the rows) measured 8 % slower in round 4 (2.755 vs 2.553 ms) and are not instantiated
// k depth of an LDS-staged fc2.weight chunk (STG; a multiple of 8) and the waves per SIMD the register allocation must
// allow (launch bounds). Round 4: 16-deep chunks (a 25.6-KB chunk buffer, 8 float4 of prefetch per thread) fit the block
// in 168 VGPRs and ~41 KB of LDS, so THREE blocks share a CU (was 40-deep chunks, 245 VGPRs, two blocks): 2.49-2.51
// against 2.55-2.56 ms per call (profiles/r04/act); 24-deep chunks at three waves spill (2.85 ms)
#ifndef FLOCK_ACT_KC
#define FLOCK_ACT_KC 16
#endif
constexpr int kKC = FLOCK_ACT_KC;
#ifndef FLOCK_ACT_WAVES
#define FLOCK_ACT_WAVES 3
#endif
// the same two knobs for the 16 x 16 kernel (sc_act16_kernel): 8-deep chunks (one k-step per staged chunk, a 14.6-KB
// chunk buffer, ~35 KB of LDS per block) let FOUR blocks share a CU: 2.33-2.35 against 2.41-2.44 ms per call for 16-deep
// chunks at three (0.69-0.70 of the f32 MFMA peak; profiles/r04/act16_kc/); 24-deep chunks at two: 2.70-2.72 ms
#ifndef FLOCK_ACT16_KC
#define FLOCK_ACT16_KC 8
#endif
constexpr int kKC16 = FLOCK_ACT16_KC;
// column pitch of the staged chunk, 2 mod 4 floats: the compiler pairs two tiles' 8-B B reads into ds_read2_b64, whose
// 16-lane groups bank on 32 dwords; rl * pitch then puts the 16 rows' pairs on 32 distinct banks (a pitch of KC + 4
// put rows rl and rl + 8 on one bank pair: 2-way conflicts on every B read)
#ifndef FLOCK_ACT16_PITCH
#define FLOCK_ACT16_PITCH (FLOCK_ACT16_KC + 2)
#endif
constexpr int kBP16 = FLOCK_ACT16_PITCH;
#ifndef FLOCK_ACT16_WAVES
#define FLOCK_ACT16_WAVES 4
#endif

struct ActArgs {
    const float* obs;     // [rows][A][in]
    const float* actors;  // agent-major flat buffer, agent a at actors + a * stride
    float* actions;       // [rows][A][2]
    float* ou;            // [rows][A][2] or NULL (no noise)
    const float* noise;   // [rows][A][2] N(0, 1) draws (with ou)
    int64_t rows, stride;
    int A, in, H1, H2, tiles;
    float theta, dt, c;  // OU: theta, dt, sigma * sqrt(dt)
};

__device__ __forceinline__ float xor32(float v, int m) {  // lane l <- lane l ^ m within each 32-lane half
    switch (m) {
        case 1: return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (1 << 10) | 0x1F));
        case 2: return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (2 << 10) | 0x1F));
        case 4: return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (4 << 10) | 0x1F));
        case 8: return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (8 << 10) | 0x1F));
        default: return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (16 << 10) | 0x1F));
    }
}
// one step of a transposed reduction across the 32-lane half: v[0, 2H) -> v[0, H), lane l keeping the upper half
// when (l & m) != 0 and adding its xor-m partner's copy of the half it keeps (H swizzles for 2H values)
template <int H>
__device__ __forceinline__ void tstep(float* v, int l, int m) {
    const bool hi = (l & m) != 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const float keep = hi ? v[i + H] : v[i];
        const float send = hi ? v[i] : v[i + H];
        v[i] = keep + xor32(send, m);
    }
}
// the 32-lane sums of 16 values in 16 swizzles (16 separate butterflies take 80): afterwards v[0] of lane l holds the
// sum of value (l >> 1) & 15 (lanes 2j and 2j + 1 alike)
__device__ __forceinline__ void tsum32_16(float (&v)[16], int l) {
    tstep<8>(v, l, 16);
    tstep<4>(v, l, 8);
    tstep<2>(v, l, 4);
    tstep<1>(v, l, 2);
    v[0] += xor32(v[0], 1);
}
// the same for 32 values in 31 swizzles: v[0] of lane l holds the sum of value l & 31
__device__ __forceinline__ void tsum32_32(float (&v)[32], int l) {
    tstep<16>(v, l, 16);
    tstep<8>(v, l, 8);
    tstep<4>(v, l, 4);
    tstep<2>(v, l, 2);
    tstep<1>(v, l, 1);
}
__device__ __forceinline__ float sum32(float v) {
    v += xor32(v, 16);
    v += xor32(v, 8);
    v += xor32(v, 4);
    v += xor32(v, 2);
    v += xor32(v, 1);
    return v;
}

// NT: 32-column tiles per wave (each wave covers half of the padded fc2 width: fc2 <= 64 NT); INC: compile-time
// observation width (0: runtime, <= 16)
template <int NT, int INC, bool STG, int TM>
__global__ __launch_bounds__(4 * TM, FLOCK_ACT_WAVES) void sc_act_kernel(ActArgs p) {
    constexpr int NTH = 4 * TM;  // threads: 2 waves per 32-row band (the two column halves)
    extern __shared__ float4 smem4[];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const int IN = INC ? INC : p.in, INP = (IN + 3) & ~3, H1 = p.H1, H2 = p.H2;
    const int W = p.A * p.tiles, b = blockIdx.x;
    const int work = (W & 7) == 0 ? (b & 7) * (W >> 3) + (b >> 3) : b;
    const int agent = work / p.tiles, tile = work - agent * p.tiles;
    const int64_t r0 = (int64_t)tile * TM;
    const float* P = p.actors + (int64_t)agent * p.stride;
    const float* W1 = P;
    const float* B1 = W1 + (int64_t)H1 * IN;
    const float* G1 = B1 + H1;
    const float* BE1 = G1 + H1;
    const float* W2 = BE1 + H1;
    const float* B2 = W2 + (int64_t)H2 * H1;
    const float* G2 = B2 + H2;
    const float* BE2 = G2 + H2;
    const float* WMU = BE2 + H2;
    const float* BMU = WMU + 2 * H2;

    // LDS: fc1 rows [H1][INP], (b1, g1, be1, 0) [H1], observation rows [64][INP], row statistics, reductions
    float* sW1 = reinterpret_cast<float*>(smem4);
    float4* sQ = reinterpret_cast<float4*>(sW1 + H1 * INP);
    float* sX = reinterpret_cast<float*>(sQ + H1);
    float* sMean = sX + TM * INP;
    float* sRstd = sMean + TM;
    float* sRed = sRstd + TM;      // [64][2]
    float* sMu = sRed + 2 * TM;    // [64][2 halves][2]

    for (int e = tid; e < H1 * INP; e += NTH) {
        const int k = e / INP, i = e - k * INP;
        sW1[e] = i < IN ? W1[k * IN + i] : 0.0f;
    }
    for (int k = tid; k < H1; k += NTH) sQ[k] = make_float4(B1[k], G1[k], BE1[k], 0.0f);
    for (int e = tid; e < TM * INP; e += NTH) {
        const int r = e / INP, i = e - r * INP;
        const int64_t gr = r0 + r;
        sX[e] = (i < IN && gr < p.rows) ? p.obs[(gr * p.A + agent) * IN + i] : 0.0f;
    }
    __syncthreads();

    // fc1 output of a row at k: the bias plus the dot product with the row's observation (an fma chain)
    auto fc1 = [&](const float* x, int k) {
        const float* wk = sW1 + k * INP;
        float d = sQ[k].x;
        if (INC == 4) {
            const float4 w4 = *reinterpret_cast<const float4*>(wk);
            d = fmaf(x[0], w4.x, d);
            d = fmaf(x[1], w4.y, d);
            d = fmaf(x[2], w4.z, d);
            d = fmaf(x[3], w4.w, d);
        } else {
            for (int i = 0; i < IN; ++i) d = fmaf(x[i], wk[i], d);
        }
        return d;
    };
#ifndef FLOCK_ACT_DIAG
#define FLOCK_ACT_DIAG 0  // timing-only builds (results wrong): 1 no LN1 statistics, 2 no epilogue, 4 no B fetch
#endif
    if (FLOCK_ACT_DIAG & 1) {
        if (tid < TM) {
            sMean[tid] = 0.0f;
            sRstd[tid] = 1.0f;
        }
    } else {  // LayerNorm-1 statistics: 4 threads per row (k = q mod 4), one pass over z - c with c = z(k = 0) of the row
       // (a shift inside the row's spread: mean = c + S1 / n, var = S2 / n - (S1 / n)^2 without cancellation)
        const int r = tid >> 2, q = tid & 3;
        float x[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = i < IN ? sX[r * INP + i] : 0.0f;
        const float c = fc1(x, 0);
        float s1 = 0.0f, s2 = 0.0f;
#pragma unroll 8
        for (int k = q; k < H1; k += 4) {
            const float d = fc1(x, k) - c;
            s1 += d;
            s2 = fmaf(d, d, s2);
        }
        s1 += __shfl_xor(s1, 1);
        s1 += __shfl_xor(s1, 2);
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        if (q == 0) {
            const float dm = s1 / (float)H1;
            sMean[r] = c + dm;
            sRstd[r] = 1.0f / sqrtf(fmaxf(s2 / (float)H1 - dm * dm, 0.0f) + 1e-5f);
        }
    }
    __syncthreads();

    // main loop: wave w covers rows 32 (w >> 1) .. +31 and the column half w & 1 (NT tiles of 32)
    const int band = w >> 1, half = w & 1, kh = 4 * (l >> 5);
    const int ra = 32 * band + (l & 31);  // the row of this lane's A values
    float xr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) xr[i] = i < IN ? sX[ra * INP + i] : 0.0f;
    const float sr = sRstd[ra], nmr = -sMean[ra] * sr;  // (z - mean) rstd = fma(z, rstd, -mean rstd)
    const float* bp[NT];
    bool bv[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int col = 32 * (NT * half + t) + (l & 31);
        bv[t] = col < H2;
        bp[t] = W2 + (int64_t)(bv[t] ? col : 0) * H1 + kh;
    }
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[t][v] = 0.0f;
    // A values of the k-step at k0: rows' fc1 -> LayerNorm -> ReLU at k0 + kh .. k0 + kh + 3
    auto a_vals = [&](int k0, float (&a)[4]) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int k = k0 + kh + s;
            const float4 q = sQ[k];
            const float y = fmaf(fc1(xr, k), sr, nmr);
            a[s] = fmaxf(fmaf(y, q.y, q.z), 0.0f);
        }
    };
    auto mfma_step = [&](const float (&a)[4], const float4 (&bq)[NT]) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0], bq[t].x, acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1], bq[t].y, acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[2], bq[t].z, acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[3], bq[t].w, acc[t], 0, 0, 0);
    };
    if constexpr (!STG) {  // B fragments straight from global memory, one k-step ahead
        float4 bq[NT], bn[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
            bq[t] = bv[t] ? *reinterpret_cast<const float4*>(bp[t]) : make_float4(0, 0, 0, 0);
        for (int k0 = 0; k0 < H1; k0 += 8) {
            if (k0 + 8 < H1) {
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    bn[t] = bv[t] ? *reinterpret_cast<const float4*>(bp[t] + k0 + 8) : make_float4(0, 0, 0, 0);
            }
            float a[4];
            a_vals(k0, a);
            mfma_step(a, bq);
#pragma unroll
            for (int t = 0; t < NT; ++t) bq[t] = bn[t];
        }
    } else {  // B staged through LDS: kKC-deep chunks of every column, coalesced 128-B row segments, next chunk in
              // registers during this chunk's MFMAs
        float* sB = sMu + 4 * TM;  // [64 NT][kKC + 4]
        constexpr int kPer = (64 * NT * kKC / 4 + NTH - 1) / NTH;  // float4 per thread per chunk
        const int ncol = 64 * NT;
        float4 pf[kPer];
        auto fetch = [&](int k0) {
            if (FLOCK_ACT_DIAG & 4) return;
#pragma unroll
            for (int i = 0; i < kPer; ++i) {
                const int f = tid + NTH * i, col = f / (kKC / 4), kq = 4 * (f % (kKC / 4));
                pf[i] = (col < H2 && k0 + kq < H1)
                            ? *reinterpret_cast<const float4*>(W2 + (int64_t)col * H1 + k0 + kq)
                            : make_float4(0, 0, 0, 0);
            }
        };
        fetch(0);
        // software-pipelined: the A values of the NEXT k-step are computed between this step's B-fragment reads and
        // its MFMAs (independent work the scheduler interleaves with the matrix instructions)
        float a[4];
        a_vals(0, a);
        for (int k0 = 0; k0 < H1; k0 += kKC) {
            __syncthreads();  // the previous chunk's fragments have been read
#pragma unroll
            for (int i = 0; i < kPer; ++i) {
                const int f = tid + NTH * i, col = f / (kKC / 4), kq = 4 * (f % (kKC / 4));
                if (col < ncol) *reinterpret_cast<float4*>(sB + col * (kKC + 4) + kq) = pf[i];
            }
            __syncthreads();
            if (k0 + kKC < H1) fetch(k0 + kKC);
            const int kc = H1 - k0 < kKC ? H1 - k0 : kKC;
            for (int ks = 0; ks < kc; ks += 8) {
                float4 bq[NT];
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    bq[t] = *reinterpret_cast<const float4*>(sB + (32 * (NT * half + t) + (l & 31)) * (kKC + 4) + ks + kh);
                float an[4];
                const int kn = k0 + ks + 8;
                a_vals(kn < H1 ? kn : 0, an);
                mfma_step(a, bq);
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = an[q];
            }
        }
    }

    if (FLOCK_ACT_DIAG & 2) {  // every accumulator stays live (one sum), no LayerNorm / head
        float sum = 0.0f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int v = 0; v < 16; ++v) sum += acc[t][v];
        if (tid < 2 * TM && r0 + (tid >> 1) < p.rows) p.actions[((r0 + (tid >> 1)) * p.A + agent) * 2 + (tid & 1)] = sum;
        return;
    }
    // epilogue. acc[t][v] of lane l: row 8 (v >> 2) + 4 (l >> 5) + (v & 3) of the band, column 32 (NT half + t) +
    // (l & 31). z = acc + fc2.bias, LayerNorm over the fc2 valid columns, ReLU, mu head, tanh.
    float b2[NT], g2[NT], be2[NT], wm0[NT], wm1[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int col = 32 * (NT * half + t) + (l & 31);
        b2[t] = bv[t] ? B2[col] : 0.0f;
        g2[t] = bv[t] ? G2[col] : 0.0f;
        be2[t] = bv[t] ? BE2[col] : 0.0f;
        wm0[t] = bv[t] ? WMU[col] : 0.0f;
        wm1[t] = bv[t] ? WMU[H2 + col] : 0.0f;
    }
    auto row_of = [&](int v) { return 32 * band + 8 * (v >> 2) + 4 * (l >> 5) + (v & 3); };
    // row sums over the lanes' 32 columns by transposed reductions (tsum32_*): lane l ends with the sum of one row
    const int jr = (l >> 1) & 15;  // the accumulator row (v index) whose sum lane l holds after tsum32_16
    float red[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        float s = 0.0f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            acc[t][v] = acc[t][v] + b2[t];
            s += bv[t] ? acc[t][v] : 0.0f;
        }
        red[v] = s;
    }
    tsum32_16(red, l);
    if ((l & 1) == 0) sRed[row_of(jr) * 2 + half] = red[0];
    __syncthreads();
    // the LayerNorm-2 statistics once per row (64 threads), not per lane and accumulator row
    float* sStat = sMean;  // [64] mean, then [64] rstd in sRstd (LayerNorm-1's are no longer read)
    if (tid < TM) sStat[tid] = (sRed[tid * 2] + sRed[tid * 2 + 1]) / (float)H2;
    __syncthreads();
    float mean[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) mean[v] = sStat[row_of(v)];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        float s = 0.0f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float d = acc[t][v] - mean[v];
            s += bv[t] ? d * d : 0.0f;
        }
        red[v] = s;
    }
    tsum32_16(red, l);
    if ((l & 1) == 0) sRed[row_of(jr) * 2 + half] = red[0];
    __syncthreads();
    if (tid < TM) sRstd[tid] = 1.0f / sqrtf((sRed[tid * 2] + sRed[tid * 2 + 1]) / (float)H2 + 1e-5f);
    __syncthreads();
    float mm[32];  // [0, 16) the mu head's output 0 per accumulator row, [16, 32) output 1
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const float rstd = sRstd[row_of(v)];
        float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float h = fmaxf((acc[t][v] - mean[v]) * rstd * g2[t] + be2[t], 0.0f);
            s0 += h * wm0[t];
            s1 += h * wm1[t];
        }
        mm[v] = s0;
        mm[16 + v] = s1;
    }
    tsum32_32(mm, l);
    {  // lane l holds value l & 31: output (l & 31) >> 4 of accumulator row l & 15
        const int jv = l & 15, jo = (l >> 4) & 1;
        sMu[(row_of(jv) * 2 + half) * 2 + jo] = mm[0];
    }
    __syncthreads();
    if (tid < 2 * TM) {
        const int r = tid >> 1, j = tid & 1;
        const int64_t gr = r0 + r;
        if (gr < p.rows) {
            const float mu = tanhf((sMu[(r * 2) * 2 + j] + sMu[(r * 2 + 1) * 2 + j]) + BMU[j]);
            const int64_t e = (gr * p.A + agent) * 2 + j;
            if (p.ou) {  // shared_critic.py choose_action: ou + theta * (0 - ou) * dt + (sigma sqrt(dt)) * z
                const float o = p.ou[e];
                const float drift = __fmul_rn(__fmul_rn(p.theta, __fsub_rn(0.0f, o)), p.dt);
                const float on = __fadd_rn(__fadd_rn(o, drift), __fmul_rn(p.c, p.noise[e]));
                p.ou[e] = on;
                p.actions[e] = __fadd_rn(mu, on);
            } else {
                p.actions[e] = mu;
            }
        }
    }
}

// The 16 x 16 variant (FLOCK_ACT_MFMA=16): one wave = 16 env rows x EVERY fc2 column, on v_mfma_f32_16x16x4_f32 (the
// same f32 rate as 32x32x2). NT 16-column tiles cover fc2 <= 16 NT: 304 columns computed for the reference's 300
// (1.3 % padding, against 6.7 % for the 32-column tiles). Lane l = (group g = l >> 4, row rl = l & 15) supplies the A
// values of its row at k = k0 + 2g + s (s = 0, 1: the two MFMAs of an 8-deep k-step; 2 fc1 values per lane per step,
// half the 32 x 32 kernel's) and reads each tile's B pair (k0 + 2g, k0 + 2g + 1) as one 8-B LDS read (column pitch
// kBP16 floats, 2 mod 4: conflict-free when two tiles' reads pair into ds_read2_b64). The accumulators hold rows 4g + i (i < 4) of column 16t + rl, so a row's LayerNorm-2 sums
// and its mu head stay inside one 16-lane group: xor butterflies / a transposed reduction, no LDS exchange and no
// barrier in the epilogue. fc2's bias, LayerNorm-2 affine and mu rows are staged in LDS with the fc1 rows.
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int NT, int INC>
__global__ __launch_bounds__(256, FLOCK_ACT16_WAVES) void sc_act16_kernel(ActArgs p) {
    constexpr int TM = 64, NTH = 256, NC = 16 * NT;
    extern __shared__ float4 smem4[];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const int IN = INC ? INC : p.in, INP = (IN + 3) & ~3, H1 = p.H1, H2 = p.H2;
    const int W = p.A * p.tiles, b = blockIdx.x;
    const int work = (W & 7) == 0 ? (b & 7) * (W >> 3) + (b >> 3) : b;
    const int agent = work / p.tiles, tile = work - agent * p.tiles;
    const int64_t r0 = (int64_t)tile * TM;
    const float* P = p.actors + (int64_t)agent * p.stride;
    const float* W1 = P;
    const float* B1 = W1 + (int64_t)H1 * IN;
    const float* G1 = B1 + H1;
    const float* BE1 = G1 + H1;
    const float* W2 = BE1 + H1;
    const float* B2 = W2 + (int64_t)H2 * H1;
    const float* G2 = B2 + H2;
    const float* BE2 = G2 + H2;
    const float* WMU = BE2 + H2;
    const float* BMU = WMU + 2 * H2;

    // LDS: fc1 rows [H1][INP], (b1, g1, be1, 0) [H1], observation rows [64][INP], LayerNorm-1 statistics [64] x 2,
    // fc2 bias / LayerNorm-2 gamma, beta / mu rows 0, 1 [5][NC], the staged fc2.weight chunk [NC][kBP16]
    float* sW1 = reinterpret_cast<float*>(smem4);
    float4* sQ = reinterpret_cast<float4*>(sW1 + H1 * INP);
    float* sX = reinterpret_cast<float*>(sQ + H1);
    float* sMean = sX + TM * INP;
    float* sRstd = sMean + TM;
    float* sP2 = sRstd + TM;
    float* sB = sP2 + 5 * NC;
    auto p2 = [&](int j, int col) { return sP2[j * NC + col]; };  // bias, LN-2 gamma / beta, mu rows 0 / 1

    for (int e = tid; e < H1 * INP; e += NTH) {
        const int k = e / INP, i = e - k * INP;
        sW1[e] = i < IN ? W1[k * IN + i] : 0.0f;
    }
    for (int k = tid; k < H1; k += NTH) sQ[k] = make_float4(B1[k], G1[k], BE1[k], 0.0f);
    for (int e = tid; e < TM * INP; e += NTH) {
        const int r = e / INP, i = e - r * INP;
        const int64_t gr = r0 + r;
        sX[e] = (i < IN && gr < p.rows) ? p.obs[(gr * p.A + agent) * IN + i] : 0.0f;
    }
    for (int c = tid; c < NC; c += NTH) {  // zero past fc2: padded columns add nothing anywhere
        const bool v = c < H2;
        sP2[c] = v ? B2[c] : 0.0f;
        sP2[NC + c] = v ? G2[c] : 0.0f;
        sP2[2 * NC + c] = v ? BE2[c] : 0.0f;
        sP2[3 * NC + c] = v ? WMU[c] : 0.0f;
        sP2[4 * NC + c] = v ? WMU[H2 + c] : 0.0f;
    }
    __syncthreads();
    auto fc1 = [&](const float* x, int k) {
        const float* wk = sW1 + k * INP;
        float d = sQ[k].x;
        if (INC == 4) {
            const float4 w4 = *reinterpret_cast<const float4*>(wk);
            d = fmaf(x[0], w4.x, d);
            d = fmaf(x[1], w4.y, d);
            d = fmaf(x[2], w4.z, d);
            d = fmaf(x[3], w4.w, d);
        } else {
            for (int i = 0; i < IN; ++i) d = fmaf(x[i], wk[i], d);
        }
        return d;
    };
    const int g = l >> 4, rl = l & 15, ra = 16 * w + rl;
    {  // LayerNorm-1 statistics: 4 threads per row, one shifted pass (as sc_act_kernel; computing fc1 on the MFMA
       // here instead, two passes over the 16-column tiles, measured slower: 2.53-2.54 against 2.42-2.44 ms)
        const int r = tid >> 2, q = tid & 3;
        float x[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = i < IN ? sX[r * INP + i] : 0.0f;
        const float c = fc1(x, 0);
        float s1 = 0.0f, s2 = 0.0f;
#pragma unroll 8
        for (int k = q; k < H1; k += 4) {
            const float d = fc1(x, k) - c;
            s1 += d;
            s2 = fmaf(d, d, s2);
        }
        s1 += __shfl_xor(s1, 1);
        s1 += __shfl_xor(s1, 2);
        s2 += __shfl_xor(s2, 1);
        s2 += __shfl_xor(s2, 2);
        if (q == 0) {
            const float dm = s1 / (float)H1;
            sMean[r] = c + dm;
            sRstd[r] = 1.0f / sqrtf(fmaxf(s2 / (float)H1 - dm * dm, 0.0f) + 1e-5f);
        }
    }
    __syncthreads();

    float xr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) xr[i] = i < IN ? sX[ra * INP + i] : 0.0f;
    const float sr = sRstd[ra], nmr = -sMean[ra] * sr;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[t][i] = 0.0f;
    auto a_vals = [&](int k0, float (&a)[2]) {  // this lane's row at k0 + 2g + s
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int k = k0 + 2 * g + s;
            const float4 q = sQ[k];
            const float y = fmaf(fc1(xr, k), sr, nmr);
            a[s] = fmaxf(fmaf(y, q.y, q.z), 0.0f);
        }
    };
    constexpr int kPer = (NC * kKC16 / 4 + NTH - 1) / NTH;  // float4 per thread per chunk
    float4 pf[kPer];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int f = tid + NTH * i, col = f / (kKC16 / 4), kq = 4 * (f % (kKC16 / 4));
            pf[i] = (col < H2 && k0 + kq < H1) ? *reinterpret_cast<const float4*>(W2 + (int64_t)col * H1 + k0 + kq)
                                               : make_float4(0, 0, 0, 0);
        }
    };
    auto stage = [&](float* buf) {
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int f = tid + NTH * i, col = f / (kKC16 / 4), kq = 4 * (f % (kKC16 / 4));
            if (col < NC) {  // two 8-B stores (the pitch keeps rows 8-B, not 16-B, aligned)
                float2* dst = reinterpret_cast<float2*>(buf + col * kBP16 + kq);
                dst[0] = make_float2(pf[i].x, pf[i].y);
                dst[1] = make_float2(pf[i].z, pf[i].w);
            }
        }
    };
    fetch(0);
    float a[2];
    a_vals(0, a);
    // (two chunk buffers with one barrier per chunk, fc2's row parameters then read from global memory to keep four
    // blocks per CU, measured slower: 2.36-2.38 against 2.30-2.31 ms, profiles/r04/act16_kc/db_ab.txt)
    for (int k0 = 0; k0 < H1; k0 += kKC16) {
        __syncthreads();  // the previous chunk's pairs have been read
        stage(sB);
        __syncthreads();
        if (k0 + kKC16 < H1) fetch(k0 + kKC16);
        const int kc = H1 - k0 < kKC16 ? H1 - k0 : kKC16;
        for (int ks = 0; ks < kc; ks += 8) {
            float an[2];
            const int kn = k0 + ks + 8;
            a_vals(kn < H1 ? kn : 0, an);
            const float* bcol = sB + rl * kBP16 + ks + 2 * g;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float2 bb = *reinterpret_cast<const float2*>(bcol + 16 * t * kBP16);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], bb.x, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], bb.y, acc[t], 0, 0, 0);
            }
            a[0] = an[0];
            a[1] = an[1];
        }
    }

    // epilogue: acc[t][i] = fc2 output of row 16 w + 4 g + i, column 16 t + rl (before the bias)
    float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int col = 16 * t + rl;
        const bool v = col < H2;
        const float b2 = p2(0, col);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            acc[t][i] = acc[t][i] + b2;
            s[i] += v ? acc[t][i] : 0.0f;
        }
    }
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) s[i] += xor32(s[i], m);  // the 16-lane sums, in every lane of the group
    float mean[4], var[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < 4; ++i) mean[i] = s[i] / (float)H2;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const bool v = 16 * t + rl < H2;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float d = acc[t][i] - mean[i];
            var[i] += v ? d * d : 0.0f;
        }
    }
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) var[i] += xor32(var[i], m);
    float rstd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) rstd[i] = 1.0f / sqrtf(var[i] / (float)H2 + 1e-5f);
    float mm[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};  // [i] mu output 0 of row i, [4 + i] output 1
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int col = 16 * t + rl;
        const float g2 = p2(1, col), be2 = p2(2, col), w0 = p2(3, col), w1 = p2(4, col);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float h = fmaxf((acc[t][i] - mean[i]) * rstd[i] * g2 + be2, 0.0f);
            mm[i] += h * w0;
            mm[4 + i] += h * w1;
        }
    }
    // transposed reduction over the 16-lane group: lanes 2j, 2j + 1 end with value j = ((rl >> 3) & 1) 4 +
    // ((rl >> 2) & 1) 2 + ((rl >> 1) & 1)
    tstep<4>(mm, l, 8);
    tstep<2>(mm, l, 4);
    tstep<1>(mm, l, 2);
    mm[0] += xor32(mm[0], 1);
    if ((l & 1) == 0) {
        const int jv = (((rl >> 3) & 1) << 2) | (((rl >> 2) & 1) << 1) | ((rl >> 1) & 1);
        const int j = jv >> 2, row = 16 * w + 4 * g + (jv & 3);
        const int64_t gr = r0 + row;
        if (gr < p.rows) {
            const float mu = tanhf(mm[0] + BMU[j]);
            const int64_t e = (gr * p.A + agent) * 2 + j;
            if (p.ou) {  // shared_critic.py choose_action: ou + theta * (0 - ou) * dt + (sigma sqrt(dt)) * z
                const float o = p.ou[e];
                const float drift = __fmul_rn(__fmul_rn(p.theta, __fsub_rn(0.0f, o)), p.dt);
                const float on = __fadd_rn(__fadd_rn(o, drift), __fmul_rn(p.c, p.noise[e]));
                p.ou[e] = on;
                p.actions[e] = __fadd_rn(mu, on);
            } else {
                p.actions[e] = mu;
            }
        }
    }
}

template <int NT, int INC, int TM>
int launch_act(hipStream_t st, const ActArgs& a, size_t lds, bool stage) {
    if (stage && lds + sizeof(float) * 64 * NT * (kKC + 4) <= 64 * 1024) {
        lds += sizeof(float) * 64 * NT * (kKC + 4);
        hipLaunchKernelGGL((sc_act_kernel<NT, INC, true, TM>), dim3(a.A * a.tiles), dim3(4 * TM), lds, st, a);
    } else {
        hipLaunchKernelGGL((sc_act_kernel<NT, INC, false, TM>), dim3(a.A * a.tiles), dim3(4 * TM), lds, st, a);
    }
    return launched();
}

// the 16 x 16 kernel (NT 16-column tiles; in_dim 4, the LDS staging path, 64-row blocks)
template <int NT>
int launch_act16(hipStream_t st, ActArgs a) {
    a.tiles = (int)((a.rows + 63) / 64);
    const size_t lds = sizeof(float) * ((size_t)a.H1 * 4 + 4 * (size_t)a.H1 + 64 * 4 + 2 * 64 +
                                        5 * 16 * NT + (size_t)16 * NT * kBP16);
    if (lds > 64 * 1024) return fail(-5, "flock_sc_act: fc1 too wide for the LDS staging");
    hipLaunchKernelGGL((sc_act16_kernel<NT, 4>), dim3(a.A * a.tiles), dim3(256), lds, st, a);
    return launched();
}

template <int NT, int INC>
int launch_act_tm(hipStream_t st, ActArgs a, int inp, bool stage, int tm) {
    a.tiles = (int)((a.rows + tm - 1) / tm);
    const size_t lds = sizeof(float) * ((size_t)a.H1 * inp + 4 * (size_t)a.H1 + (size_t)tm * inp + 8 * (size_t)tm);
    if (lds > 64 * 1024) return fail(-5, "flock_sc_act: fc1 too wide for the LDS staging");
    return launch_act<NT, INC, 64>(st, a, lds, stage);
}

}  // namespace

extern "C" int flock_sc_act(void* stream, int64_t rows, int n_agents, int in_dim, int fc1, int fc2, const float* obs,
                            const float* actors, int64_t actor_stride, float* actions, float* ou_state,
                            const float* noise, float theta, float dt, float sigma_sqrt_dt) {
    if (!obs || !actors || !actions || (ou_state && !noise))
        return fail(-3, "flock_sc_act: NULL argument");
    if (rows < 0 || n_agents < 1 || in_dim < 1 || in_dim > 16 || fc1 < 8 || (fc1 & 7) || fc2 < 1 || fc2 > 320)
        return fail(-5, "flock_sc_act: needs 1 <= in_dim <= 16, fc1 a multiple of 8, 1 <= fc2 <= 320");
    if (((uintptr_t)actors & 15) || (actor_stride & 3))
        return fail(-5, "flock_sc_act: actors must be 16-B aligned with a stride that is a multiple of 4");
    const int64_t per = (int64_t)fc1 * (in_dim + 3) + (int64_t)fc2 * (fc1 + 5) + 2;
    if (actor_stride < per) return fail(-5, "flock_sc_act: actor_stride smaller than one actor");
    if (rows == 0) return 0;
    constexpr int tm = 64;  // env rows per block (128-row blocks measured 8 % slower, round 4)
    if ((rows + 63) / 64 * n_agents > 0x7fffffff) return fail(-5, "flock_sc_act: too many rows x agents");
    ActArgs a;
    a.obs = obs;
    a.actors = actors;
    a.actions = actions;
    a.ou = ou_state;
    a.noise = noise;
    a.rows = rows;
    a.stride = actor_stride;
    a.A = n_agents;
    a.in = in_dim;
    a.H1 = fc1;
    a.H2 = fc2;
    a.tiles = 0;
    a.theta = theta;
    a.dt = dt;
    a.c = sigma_sqrt_dt;
    const int inp = (in_dim + 3) & ~3;
    hipStream_t st = (hipStream_t)stream;
    const int nt = (fc2 + 63) / 64;
    constexpr bool stage = true;  // fc2.weight through LDS (launch_act falls back to global reads past 64 KB of LDS)
    if (in_dim == 4) {  // the 16 x 16 kernel at the widths it is instantiated for
        switch ((fc2 + 15) / 16) {  // the widths with an instantiation; others take the 32 x 32 kernel
            case 7: return launch_act16<7>(st, a);
            case 19: return launch_act16<19>(st, a);
            case 20: return launch_act16<20>(st, a);
            default: break;
        }
    }
    if (in_dim == 4) {
        switch (nt) {
            case 1: return launch_act_tm<1, 4>(st, a, inp, stage, tm);
            case 2: return launch_act_tm<2, 4>(st, a, inp, stage, tm);
            case 3: return launch_act_tm<3, 4>(st, a, inp, stage, tm);
            case 4: return launch_act_tm<4, 4>(st, a, inp, stage, tm);
            default: return launch_act_tm<5, 4>(st, a, inp, stage, tm);
        }
    }
    switch (nt) {
        case 1: return launch_act_tm<1, 0>(st, a, inp, stage, tm);
        case 2: return launch_act_tm<2, 0>(st, a, inp, stage, tm);
        case 3: return launch_act_tm<3, 0>(st, a, inp, stage, tm);
        case 4: return launch_act_tm<4, 0>(st, a, inp, stage, tm);
        default: return launch_act_tm<5, 0>(st, a, inp, stage, tm);
    }
}
