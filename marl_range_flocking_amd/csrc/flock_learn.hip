// flock_learn.hip — learner-side HIP kernels (gfx950): fused Adam + soft target update over flat parameter
// buffers, global grad L2 norm (clip_grad_norm_ without a host sync), fused GRU-cell forward/backward (the
// elementwise part of nn.GRUCell; the gate GEMMs run as batched rocBLAS/hipBLASLt GEMMs), and row gather/scatter
// for the device-resident replay rings. C ABI: include/flock_learn.h.
//
// Every learner keeps its parameters, gradients and Adam moments of ALL agents in one flat f32 buffer each, so one
// launch updates every parameter of every agent (the reference runs one torch.optim.Adam per agent network).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "flock_learn.h"
#include "learn_internal.h"

#pragma clang fp contract(off)

namespace flock_learn_internal {
thread_local char g_err[256] = "";
int fail(int code, const char* msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return code;
}
int launched() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(-4, hipGetErrorString(e));
}
}  // namespace flock_learn_internal

namespace {
using flock_learn_internal::fail;
using flock_learn_internal::launched;

constexpr int kBlock = 256;

int grid_for(int64_t n, int per_thread = 4) {
    int64_t g = (n + (int64_t)kBlock * per_thread - 1) / ((int64_t)kBlock * per_thread);
    if (g < 1) g = 1;
    if (g > 2048) g = 2048;  // grid-stride beyond (memory-bound: 256 CUs x 8 blocks)
    return (int)g;
}

__device__ __forceinline__ float sqrt_rn(float x) { return __builtin_sqrtf(x); }

// torch.optim.Adam, single-tensor path (torch/optim/adam.py _single_tensor_adam), per element:
//   m = m.lerp(g, 1 - b1)                 lerp: w < 0.5 ? m + w * (g - m) : g - (g - m) * (1 - w)
//   v = v * b2 + (1 - b2) * g * g         mul_(b2).addcmul_(g, g, value=1 - b2)
//   p = p + (-lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)     addcdiv_
// then optionally the target network soft update (mode 0: t*(1-tau) + p*tau, maddpg nets net.py:305-309;
// mode 1: tau*p + (1-tau)*t, shared critic agent_simple_shared_critic.py:172-185).
struct AdamArgs {
    int64_t n;
    float *p, *m, *v, *target;
    const float *g, *grad_scale;
    const int64_t* step;  // device step count (graph-capturable path) or null: neg_step / bc2s given
    float lr, beta1, beta2, w1, one_minus_b2, neg_step, bc2s, eps, tau, one_minus_tau;
    int target_mode;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float* t, const AdamArgs& a,
                                          float gs, float neg_step, float bc2s) {
    if (a.grad_scale) g = g * gs;
    m = (a.w1 < 0.5f) ? m + a.w1 * (g - m) : g - (g - m) * (1.0f - a.w1);
    v = v * a.beta2;
    v = v + (a.one_minus_b2 * g) * g;
    const float denom = sqrt_rn(v) / bc2s + a.eps;
    p = p + (neg_step * m) / denom;
    if (t) *t = a.target_mode == 0 ? *t * a.one_minus_tau + p * a.tau : a.tau * p + a.one_minus_tau * *t;
}

// VEC: every pointer 16-B aligned -> float4 loads and stores of each stream (the update is HBM-bound:
// 16 or 20 B read + 12 or 16 B written per parameter), the n % 4 tail by block 0. Same per-element arithmetic as
// the scalar path, so both give identical bits.
template <bool VEC>
__global__ __launch_bounds__(kBlock) void adam_kernel(AdamArgs a) {
    __shared__ float sh[2];
    float neg_step = a.neg_step, bc2s = a.bc2s;
    if (a.step) {
        if (threadIdx.x == 0) {
            const double st = (double)*a.step;
            const double bc1 = 1.0 - pow((double)a.beta1, st);
            const double bc2 = 1.0 - pow((double)a.beta2, st);
            sh[0] = (float)(-(double)a.lr / bc1);
            sh[1] = (float)sqrt(bc2);
        }
        __syncthreads();
        neg_step = sh[0];
        bc2s = sh[1];
    }
    const float gs = a.grad_scale ? *a.grad_scale : 1.0f;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t i0 = blockIdx.x * (int64_t)kBlock + threadIdx.x;
    if (VEC) {
        const int64_t nq = a.n >> 2;
        // two float4 of every stream per thread and iteration, all loads issued before the arithmetic: 906M
        // parameters with the target (config 5's critics), 6.68 -> 5.80-5.86 ms per call (4.9 -> 5.6 TB/s; another box
        // 7.21 -> 6.81-6.83); four: as two; non-temporal loads and stores: flat (tools/adam_bw.py, profiles/r05/adam/)
        constexpr int U = 2;
        auto ld4 = [](const float* b, int64_t q) { return reinterpret_cast<const float4*>(b)[q]; };
        auto st4 = [](float* b, int64_t q, float4 x) { reinterpret_cast<float4*>(b)[q] = x; };
        for (int64_t q0 = i0; q0 < nq; q0 += U * stride) {
            float4 p[U], g[U], m[U], v[U], t[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t q = q0 + u * stride;
                if (q < nq) {
                    p[u] = ld4(a.p, q);
                    g[u] = ld4(a.g, q);
                    m[u] = ld4(a.m, q);
                    v[u] = ld4(a.v, q);
                    t[u] = a.target ? ld4(a.target, q) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t q = q0 + u * stride;
                if (q < nq) {
                    float* tp = a.target ? &t[u].x : nullptr;
                    adam_elem(p[u].x, g[u].x, m[u].x, v[u].x, tp, a, gs, neg_step, bc2s);
                    adam_elem(p[u].y, g[u].y, m[u].y, v[u].y, tp ? tp + 1 : nullptr, a, gs, neg_step, bc2s);
                    adam_elem(p[u].z, g[u].z, m[u].z, v[u].z, tp ? tp + 2 : nullptr, a, gs, neg_step, bc2s);
                    adam_elem(p[u].w, g[u].w, m[u].w, v[u].w, tp ? tp + 3 : nullptr, a, gs, neg_step, bc2s);
                    st4(a.p, q, p[u]);
                    st4(a.m, q, m[u]);
                    st4(a.v, q, v[u]);
                    if (a.target) st4(a.target, q, t[u]);
                }
            }
        }
        if (blockIdx.x != 0) return;
        i0 = (nq << 2) + threadIdx.x;  // tail
    }
    for (int64_t i = i0; i < a.n; i += VEC ? a.n : stride) {
        float p = a.p[i], m = a.m[i], v = a.v[i];
        adam_elem(p, a.g[i], m, v, a.target ? a.target + i : nullptr, a, gs, neg_step, bc2s);
        a.p[i] = p;
        a.m[i] = m;
        a.v[i] = v;
    }
}

template <bool VEC>
__global__ __launch_bounds__(kBlock) void soft_update_kernel(int64_t n, float* __restrict__ target,
                                                             const float* __restrict__ src, float tau,
                                                             float one_minus_tau, int mode) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t i0 = blockIdx.x * (int64_t)kBlock + threadIdx.x;
    auto f = [&](float t, float s) { return mode == 0 ? t * one_minus_tau + s * tau : tau * s + one_minus_tau * t; };
    if (VEC) {
        const int64_t nq = n >> 2;
        for (int64_t q = i0; q < nq; q += stride) {
            float4 t = reinterpret_cast<const float4*>(target)[q];
            const float4 s = reinterpret_cast<const float4*>(src)[q];
            t.x = f(t.x, s.x);
            t.y = f(t.y, s.y);
            t.z = f(t.z, s.z);
            t.w = f(t.w, s.w);
            reinterpret_cast<float4*>(target)[q] = t;
        }
        if (blockIdx.x != 0) return;
        i0 = (nq << 2) + threadIdx.x;
    }
    for (int64_t i = i0; i < n; i += VEC ? n : stride) target[i] = f(target[i], src[i]);
}

bool aligned16(const void* p) { return p == nullptr || ((uintptr_t)p & 15u) == 0; }

int launch_adam(void* stream, const AdamArgs& a) {
    const bool vec = aligned16(a.p) && aligned16(a.g) && aligned16(a.m) && aligned16(a.v) && aligned16(a.target);
    if (vec)
        hipLaunchKernelGGL(adam_kernel<true>, dim3(grid_for(a.n, 4)), dim3(kBlock), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(adam_kernel<false>, dim3(grid_for(a.n, 4)), dim3(kBlock), 0, (hipStream_t)stream, a);
    return launched();
}

// sum of squares: pass 1 per-block partials (f64 accumulation), pass 2 one block folds them and writes
// out[0] = ||g||_2 and out[1] = min(max_norm / (||g|| + 1e-6), 1) (torch.nn.utils.clip_grad_norm_).
__global__ __launch_bounds__(kBlock) void sq_partial_kernel(int64_t n, const float* __restrict__ g,
                                                            double* __restrict__ partial) {
    __shared__ double red[kBlock];
    double acc = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const double x = g[i];
        acc += x * x;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(kBlock) void sq_final_kernel(int nparts, const double* __restrict__ partial,
                                                          float max_norm, float* __restrict__ out) {
    __shared__ double red[kBlock];
    double acc = 0.0;
    for (int i = threadIdx.x; i < nparts; i += kBlock) acc += partial[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float norm = (float)sqrt(red[0]);
        out[0] = norm;
        const float coef = max_norm / (norm + 1e-6f);
        out[1] = coef < 1.0f ? coef : 1.0f;
    }
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// nn.GRUCell elementwise part (ATen gru_cell, RNN.cpp): rows of gi = x W_ih^T + b_ih and gh = h W_hh^T + b_hh
// (gate order r, z, n), h' = (h - n) * z + n. ws keeps (r, z, n, gh_n) for the backward.
__global__ __launch_bounds__(kBlock) void gru_fwd_kernel(int64_t rows, int H, const float* __restrict__ gi,
                                                         const float* __restrict__ gh, const float* __restrict__ h,
                                                         float* __restrict__ hout, float* __restrict__ ws) {
    const int64_t n = rows * H;
    for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < n; e += (int64_t)gridDim.x * kBlock) {
        const int64_t row = e / H;
        const int c = (int)(e - row * H);
        const float* a = gi + row * 3 * H;
        const float* b = gh + row * 3 * H;
        const float r = sigmoidf_(b[c] + a[c]);
        const float z = sigmoidf_(b[H + c] + a[H + c]);
        const float ghn = b[2 * H + c];
        const float nn = tanhf(a[2 * H + c] + ghn * r);
        const float hv = h[e];
        hout[e] = (hv - nn) * z + nn;
        if (ws) {
            float* w = ws + row * 4 * H;
            w[c] = r;
            w[H + c] = z;
            w[2 * H + c] = nn;
            w[3 * H + c] = ghn;
        }
    }
}

__global__ __launch_bounds__(kBlock) void gru_bwd_kernel(int64_t rows, int H, const float* __restrict__ dhout,
                                                         const float* __restrict__ h, const float* __restrict__ ws,
                                                         float* __restrict__ dgi, float* __restrict__ dgh,
                                                         float* __restrict__ dh) {
    const int64_t n = rows * H;
    for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < n; e += (int64_t)gridDim.x * kBlock) {
        const int64_t row = e / H;
        const int c = (int)(e - row * H);
        const float* w = ws + row * 4 * H;
        const float r = w[c], z = w[H + c], nn = w[2 * H + c], ghn = w[3 * H + c];
        const float go = dhout[e];
        const float hv = h[e];
        const float dn = go * (1.0f - z);
        const float dz = go * (hv - nn);
        const float dan = dn * (1.0f - nn * nn);
        const float dr = dan * ghn;
        const float dar = dr * (r * (1.0f - r));
        const float daz = dz * (z * (1.0f - z));
        float* gi_ = dgi + row * 3 * H;
        float* gh_ = dgh + row * 3 * H;
        gi_[c] = dar;
        gi_[H + c] = daz;
        gi_[2 * H + c] = dan;
        gh_[c] = dar;
        gh_[H + c] = daz;
        gh_[2 * H + c] = dan * r;
        dh[e] = go * z;
    }
}

// VDN QNet feature chain of A agents over R rows each, ONE launch (learners/vdn/net.py:19-33 agent_feature_i =
// Linear(n_obs, 64)-ReLU-Linear(64, 32)-ReLU, then the GRUCell input side x W_ih^T + b_ih of every chunk step):
//   y1 = relu(x W1^T + b1) [64], y2 = relu(y1 W2^T + b2) [32], gi = y2 Wih^T + bih [96]
// replaces three batched GEMMs (K = n_obs, 64, 32) and two ReLU passes whose [A][R][64] / [A][R][32] intermediates
// made the round trip through HBM. One block per agent walks its rows 64 at a time; wave w owns rows [16 w, 16 w + 16)
// of each group and runs each layer as f32 MFMA tiles (v_mfma_f32_16x16x4_f32: exact f32, a k-ordered fmaf chain per
// output) over all of the layer's 16-column tiles: A operand = the wave's activation rows, B operand = the weight rows
// ([o][k] layout), both read per lane from LDS rows padded to 2 mod 32 floats (16 rows x 2 k per half-wave on
// distinct banks). y1 / y2 stay in LDS for the next layer; gi (and y1 / y2 when the backward needs them) are written
// from the accumulators, 16 lanes to 64 contiguous bytes of a row. x element (a, c, b, f) at
// x[a*xa + c*xc + b*xb + f], row r = c*B + b (the replay gather's [B][C][A][n] layout is read in place).
// Config 4 (512 agents x 320 rows), per launch: lane-per-row FMA with broadcast weight reads 77 us, MFMA tiles over
// 64-row blocks 72 us (each block's serial load -> compute chain at two blocks per CU), this per-agent walk with
// the next rows' x in flight 41 us.
constexpr int kF1 = 64, kF2 = 32, kFG = 96, kFRows = 64, kFMaxIn = 16;
constexpr int kSW1 = kFMaxIn + 2, kSY1 = kF1 + 2, kSY2 = kF2 + 2;  // LDS row strides (floats)
using f32x4_t = float __attribute__((ext_vector_type(4)));

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations (lgkmcnt), not for its global loads
// (__syncthreads() waits for vmcnt(0) too, which would drain the next rows' prefetch at every barrier). The global
// loads' own waits stay where their registers are first used.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// NT column tiles of 16: acc[t] += A[16 rows][K] * W[16 t .. 16 t + 16][K]^T, k in steps of 4 (one MFMA each)
template <int NT>
__device__ __forceinline__ void mfma_rows(f32x4_t (&acc)[NT], const float* a, int sa, const float* w, int sw,
                                          int K, int lane) {
    const int i = lane & 15, kk = lane >> 4;
    for (int k = 0; k < K; k += 4) {
        const float av = a[i * sa + k + kk];
#pragma unroll
        for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, w[(16 * t + i) * sw + k + kk], acc[t], 0, 0, 0);
    }
}

__global__ __launch_bounds__(kBlock) void vdn_feat_fwd_kernel(int R, int B, int NI, const float* __restrict__ x,
                                                              int64_t xa, int64_t xc, int64_t xb,
                                                              const float* __restrict__ W1, const float* __restrict__ b1,
                                                              const float* __restrict__ W2, const float* __restrict__ b2,
                                                              const float* __restrict__ Wi, const float* __restrict__ bi,
                                                              float* __restrict__ y1o, float* __restrict__ y2o,
                                                              float* __restrict__ gi) {
    // one block per agent (57 KB of LDS, two blocks per CU: the 512 agents of config 4 in one round); the weights
    // are staged once and the block walks the agent's rows 64 at a time, loading the next 64 rows of x into
    // registers while the current ones run through the three layers
    __shared__ float w1[kF1 * kSW1];
    __shared__ float w2[kF2 * kSY1];
    __shared__ float wi[kFG * kSY2];
    __shared__ float bs[kF1 + kF2 + kFG];
    __shared__ float xs[kFRows * kSW1];
    __shared__ float y1s[kFRows * kSY1];
    __shared__ float y2s[kFRows * kSY2];
    const int64_t a = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int K1 = (NI + 3) & ~3;
    const int sx = K1 + 2;  // xs / w1 row stride: 2 mod 4 (and so 2 (2j+1) mod 32: distinct banks for 16 rows)
    for (int e = tid; e < kF1 * K1; e += kBlock) {
        const int o = e / K1, k = e - o * K1;
        w1[o * sx + k] = k < NI ? W1[(a * kF1 + o) * NI + k] : 0.0f;
    }
    for (int e = tid; e < kF2 * kF1; e += kBlock) w2[(e / kF1) * kSY1 + (e % kF1)] = W2[a * kF2 * kF1 + e];
    for (int e = tid; e < kFG * kF2; e += kBlock) wi[(e / kF2) * kSY2 + (e % kF2)] = Wi[a * kFG * kF2 + e];
    if (tid < kF1) bs[tid] = b1[a * kF1 + tid];
    if (tid < kF2) bs[kF1 + tid] = b2[a * kF2 + tid];
    if (tid < kFG) bs[kF1 + kF2 + tid] = bi[a * kFG + tid];
    constexpr int kXPT = kFRows * kFMaxIn / kBlock;  // x elements per thread per 64 rows (at most)
    float xr[kXPT];
    auto load_x = [&](int r0) {
#pragma unroll
        for (int q = 0; q < kXPT; ++q) {
            const int e = tid + kBlock * q, rr = e / K1, f = e - rr * K1, r = r0 + rr;
            xr[q] = 0.0f;
            if (e < kFRows * K1 && r < R && f < NI) {
                const int c = r / B, b = r - c * B;
                xr[q] = x[a * xa + c * xc + b * xb + f];
            }
        }
    };
    load_x(0);
    const int col = lane & 15, row4 = 16 * wv + 4 * (lane >> 4);  // C/D: col = lane & 15, row = 4 (lane >> 4) + v
    for (int r0 = 0; r0 < R; r0 += kFRows) {
        const int nr = min(kFRows, R - r0);
#pragma unroll
        for (int q = 0; q < kXPT; ++q) {
            const int e = tid + kBlock * q;
            if (e < kFRows * K1) xs[(e / K1) * sx + (e % K1)] = xr[q];
        }
        lds_barrier();  // xs (and, first time round, the weights) visible; the previous rows' reads are done
        if (r0 + kFRows < R) load_x(r0 + kFRows);  // in flight while these rows compute
        const int64_t base = a * R + r0;
        {  // layer 1: 4 column tiles
            f32x4_t acc[4] = {};
            mfma_rows<4>(acc, xs + 16 * wv * sx, sx, w1, sx, K1, lane);
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const float y = fmaxf(acc[t][v] + bs[16 * t + col], 0.0f);
                    y1s[(row4 + v) * kSY1 + 16 * t + col] = y;
                    if (y1o && row4 + v < nr) y1o[(base + row4 + v) * kF1 + 16 * t + col] = y;
                }
        }
        lds_barrier();
        {  // layer 2: 2 column tiles
            f32x4_t acc[2] = {};
            mfma_rows<2>(acc, y1s + 16 * wv * kSY1, kSY1, w2, kSY1, kF1, lane);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const float y = fmaxf(acc[t][v] + bs[kF1 + 16 * t + col], 0.0f);
                    y2s[(row4 + v) * kSY2 + 16 * t + col] = y;
                    if (y2o && row4 + v < nr) y2o[(base + row4 + v) * kF2 + 16 * t + col] = y;
                }
        }
        lds_barrier();
        {  // GRU input side: 6 column tiles, written from the accumulators (16 lanes = 64 contiguous bytes)
            f32x4_t acc[6] = {};
            mfma_rows<6>(acc, y2s + 16 * wv * kSY2, kSY2, wi, kSY2, kF2, lane);
#pragma unroll
            for (int t = 0; t < 6; ++t)
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    if (row4 + v < nr)
                        gi[(base + row4 + v) * kFG + 16 * t + col] = acc[t][v] + bs[kF1 + kF2 + 16 * t + col];
        }
    }
}

// Backward of the same chain, ONE launch (the five batched GEMMs, two ReLU masks and three row sums of the autograd
// backward, learners/core.py _VdnFeatFn): from dgi = dLoss/dgi [A][R][96] and the saved y1 / y2,
//   dz2 = (dgi Wih) [y2 > 0]   dz1 = (dz2 W2) [y1 > 0]
//   dWih = dgi^T y2, dbih = sum_r dgi, dW2 = dz2^T y1, db2 = sum_r dz2, dW1 = dz1^T x, db1 = sum_r dz1
// One block of 8 waves (two per SIMD, so one wave's dependent MFMA chain hides behind the other's) per agent walks
// its rows 64 at a time, the next 64 rows of dgi / y1 / y2 / x in registers while the current ones compute. Every
// row chunk is staged FEATURE-major in LDS ([feature][row], stride 64 + 2), so the same arrays serve as the A
// operand of the row GEMMs (dz2, dz1: A[row][k] read as T[k][row]) and as both operands of the weight-gradient
// GEMMs, whose K dimension is the rows: the 24 tiles of dWih (6 x 2), dW2 (2 x 4) and dW1 (4 x 1) stay in MFMA
// accumulators across all chunks (3 per wave) and are written once at the end; the bias sums run on VALU from the
// same LDS rows. f32 MFMA (v_mfma_f32_16x16x4_f32): each output is a k-ordered fmaf chain.
constexpr int kBS = kFRows + 2;  // feature-major row stride (floats): 2 mod 4
constexpr int kBB = 512;         // threads per block of the backward
__global__ __launch_bounds__(kBB) void vdn_feat_bwd_kernel(int R, int B, int NI, const float* __restrict__ x,
                                                           int64_t xa, int64_t xc, int64_t xb,
                                                           const float* __restrict__ W2, const float* __restrict__ Wi,
                                                           const float* __restrict__ y1, const float* __restrict__ y2,
                                                           const float* __restrict__ dgi,
                                                           float* __restrict__ dW1, float* __restrict__ db1,
                                                           float* __restrict__ dW2, float* __restrict__ db2,
                                                           float* __restrict__ dWi, float* __restrict__ dbi) {
    __shared__ float wiN[kFG * (kF2 + 2)];   // Wih [96][32] as stored: B[k][j] of dz2 = dgi Wih (k = 96 outputs)
    __shared__ float w2N[kF2 * (kF1 + 2)];   // W2 [32][64] as stored: B[k][j] of dz1 = dz2 W2 (k = 32 outputs)
    __shared__ float gT[kFG * kBS];          // dgi chunk, feature-major [96][64]
    __shared__ float y2T[kF2 * kBS];         // [32][64]
    __shared__ float y1T[kF1 * kBS];         // [64][64]
    __shared__ float xT[kFMaxIn * kBS];      // [16][64] (features >= n_obs are zero)
    __shared__ float z2T[kF2 * kBS];         // dz2 [32][64]
    __shared__ float z1T[kF1 * kBS];         // dz1 [64][64]
    const int64_t a = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;  // 8 waves
    const int i16 = lane & 15, kk = lane >> 4;
    for (int e = tid; e < kFG * kF2; e += kBB) wiN[(e / kF2) * (kF2 + 2) + e % kF2] = Wi[a * kFG * kF2 + e];
    for (int e = tid; e < kF2 * kF1; e += kBB) w2N[(e / kF1) * (kF1 + 2) + e % kF1] = W2[a * kF2 * kF1 + e];
    // per-thread register staging of the next chunk: dgi 64 x 96 (12 floats / thread), y1 64 x 64 (8), y2 64 x 32
    // (4), x 64 x 16 (2), each read row-major with consecutive threads on consecutive floats
    constexpr int kG = kFRows * kFG / kBB, kY1 = kFRows * kF1 / kBB, kY2 = kFRows * kF2 / kBB,
                  kX = kFRows * kFMaxIn / kBB;
    float rg[kG], r1[kY1], r2[kY2], rx[kX];
    const int64_t base_a = a * (int64_t)R;
    auto load = [&](int r0) {
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int e = tid + kBB * q, rr = e / kFG;
            rg[q] = r0 + rr < R ? dgi[(base_a + r0) * kFG + e] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < kY1; ++q) {
            const int e = tid + kBB * q, rr = e / kF1;
            r1[q] = r0 + rr < R ? y1[(base_a + r0) * kF1 + e] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < kY2; ++q) {
            const int e = tid + kBB * q, rr = e / kF2;
            r2[q] = r0 + rr < R ? y2[(base_a + r0) * kF2 + e] : 0.0f;
        }
#pragma unroll
        for (int q = 0; q < kX; ++q) {
            const int e = tid + kBB * q, rr = e / kFMaxIn, f = e - rr * kFMaxIn, r = r0 + rr;
            rx[q] = 0.0f;
            if (r < R && f < NI) {
                const int c = r / B, b = r - c * B;
                rx[q] = x[a * xa + c * xc + b * xb + f];
            }
        }
    };
    // persistent weight-gradient accumulators, three 16 x 16 tiles per wave: unit u = 3 wv + j of the 24 (dWih
    // units 0..11 -> tile (m, n) = (u >> 1, u & 1); dW2 units 12..19 -> ((u - 12) >> 2, (u - 12) & 3); dW1 units
    // 20..23 -> rows 16 (u - 20) of the 64 outputs x the 16 padded features)
    f32x4_t acc3[3] = {};
    float bsum = 0.0f;  // thread tid < 192: bias sum of feature tid (dbih 0..95, db2 96..127, db1 128..191)
    load(0);
    const int col = i16, row4 = 4 * kk;  // C/D layout: col = lane & 15, row = 4 (lane >> 4) + v
    const int rg4 = wv & 3;              // the 16-row group of the row GEMMs this wave works on
    for (int r0 = 0; r0 < R; r0 += kFRows) {
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int e = tid + kBB * q, rr = e / kFG, f = e - rr * kFG;
            gT[f * kBS + rr] = rg[q];
        }
#pragma unroll
        for (int q = 0; q < kY1; ++q) {
            const int e = tid + kBB * q, rr = e / kF1, f = e - rr * kF1;
            y1T[f * kBS + rr] = r1[q];
        }
#pragma unroll
        for (int q = 0; q < kY2; ++q) {
            const int e = tid + kBB * q, rr = e / kF2, f = e - rr * kF2;
            y2T[f * kBS + rr] = r2[q];
        }
#pragma unroll
        for (int q = 0; q < kX; ++q) {
            const int e = tid + kBB * q, rr = e / kFMaxIn, f = e - rr * kFMaxIn;
            xT[f * kBS + rr] = rx[q];
        }
        lds_barrier();  // the chunk (and, first time round, the weights) visible; last chunk's reads are done
        if (r0 + kFRows < R) load(r0 + kFRows);  // in flight while this chunk computes
        {  // dz2 = (dgi Wih) [y2 > 0]: waves w and w + 4 share rows 16 (w & 3) .., one column tile each, K = 96
            const int t = wv >> 2;
            f32x4_t acc = {};
#pragma unroll 4
            for (int k = 0; k < kFG; k += 4)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(gT[(k + kk) * kBS + 16 * rg4 + i16],
                                                           wiN[(k + kk) * (kF2 + 2) + 16 * t + i16], acc, 0, 0, 0);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int r = 16 * rg4 + row4 + v, o = 16 * t + col;
                z2T[o * kBS + r] = y2T[o * kBS + r] > 0.0f ? acc[v] : 0.0f;
            }
        }
        lds_barrier();
        {  // dz1 = (dz2 W2) [y1 > 0]: two column tiles per wave, K = 32
            f32x4_t acc[2] = {};
            const int t0 = 2 * (wv >> 2);
#pragma unroll
            for (int k = 0; k < kF2; k += 4) {
                const float av = z2T[(k + kk) * kBS + 16 * rg4 + i16];
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, w2N[(k + kk) * (kF1 + 2) + 16 * (t0 + j) + i16],
                                                                  acc[j], 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int r = 16 * rg4 + row4 + v, o = 16 * (t0 + j) + col;
                    z1T[o * kBS + r] = y1T[o * kBS + r] > 0.0f ? acc[j][v] : 0.0f;
                }
        }
        lds_barrier();
        // weight gradients, K = this chunk's 64 rows: A[m][k] = T_a[m][row k], B[n][k] = T_b[n][row k]
#pragma unroll 2
        for (int k = 0; k < kFRows; k += 4) {
            const int kr = k + kk;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int u = 3 * wv + j;
                const float* Ta;
                const float* Tb;
                int m, n;
                if (u < 12) {
                    Ta = gT, Tb = y2T, m = u >> 1, n = u & 1;
                } else if (u < 20) {
                    Ta = z2T, Tb = y1T, m = (u - 12) >> 2, n = (u - 12) & 3;
                } else {
                    Ta = z1T, Tb = xT, m = u - 20, n = 0;
                }
                acc3[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ta[(16 * m + i16) * kBS + kr],
                                                               Tb[(16 * n + i16) * kBS + kr], acc3[j], 0, 0, 0);
            }
        }
        if (tid < kFG + kF2 + kF1) {  // bias sums: one feature per thread, rows in order
            const float* src = tid < kFG ? gT + tid * kBS : tid < kFG + kF2 ? z2T + (tid - kFG) * kBS
                                                                           : z1T + (tid - kFG - kF2) * kBS;
            const int nr = min(kFRows, R - r0);
            if (nr == kFRows) {
#pragma unroll 16
                for (int r = 0; r < kFRows; ++r) bsum += src[r];
            } else {
                for (int r = 0; r < nr; ++r) bsum += src[r];
            }
        }
        lds_barrier();  // the next chunk's stores overwrite these arrays
    }
    // write the weight gradients from the accumulators (C/D: row = 4 kk + v within the tile, column = lane & 15)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int u = 3 * wv + j;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            if (u < 12) {
                const int m = u >> 1, n = u & 1;
                dWi[(a * kFG + 16 * m + row4 + v) * kF2 + 16 * n + col] = acc3[j][v];
            } else if (u < 20) {
                const int m = (u - 12) >> 2, n = (u - 12) & 3;
                dW2[(a * kF2 + 16 * m + row4 + v) * kF1 + 16 * n + col] = acc3[j][v];
            } else if (col < NI) {
                dW1[(a * kF1 + 16 * (u - 20) + row4 + v) * NI + col] = acc3[j][v];
            }
        }
    }
    if (tid < kFG)
        dbi[a * kFG + tid] = bsum;
    else if (tid < kFG + kF2)
        db2[a * kF2 + tid - kFG] = bsum;
    else if (tid < kFG + kF2 + kF1)
        db1[a * kF1 + tid - kFG - kF2] = bsum;
}

// dst[r, :] = src[idx[r], :]  (replay minibatch / chunk gather); one wave per row, 16-B vectors when aligned
// GRUCell recurrence of A independent networks over a whole chunk of C steps, ONE block per network (replaces
// C x (hidden GEMM + gate kernel + reset) launches per network: vdn/train_flock.py:23-36 and
// maddpg_official_rnn/MADDPG.py:95-132 step their GRUCells once per chunk step). Step t:
//   gh = h W_hh^T + b_hh;  r, z, n, h' as gru_fwd_kernel;  hs[t] = h';  h = keep[t] ? h' : 0 (the done reset)
// gi: [A][C][B][3H] input-side pre-activations of every step (computed for all steps by one GEMM beforehand);
// keep: uint8 at keep[t*kt + a*ka + b*kb]; the initial hidden state is zero (every reference chunk starts from
// init_hidden). Thread (j, b): hidden unit j = tid % H of rows b = tid / H + (256 / H) * q; its three W_hh rows
// live in registers, the hidden states in LDS (ping-pong). ws [A][C][B][4H] = (r, z, n, gh_n) for the backward.
// The q head fused (QH, VDN's QNet.q: q = h' W_q^T + b_q of every step's output, learners/vdn/net.py:36-37): W_q /
// b_q staged in LDS, each step's outputs h' kept in a ping-pong LDS buffer, and after the step's barrier the
// B x NA q values of the step computed from it (float4 reads, k-ordered fmaf from b_q) into q [A][C][B][NA]; hs may
// then be NULL (no backward).
struct QHead {
    const float* W;  // [A][NA][H]
    const float* b;  // [A][NA]
    float* q;        // [A][C][B][NA]
    int NA;
};
template <int H, bool QH = false>
__global__ __launch_bounds__(kBlock) void gru_seq_fwd_kernel(int C, int B, const float* __restrict__ gi,
                                                             const float* __restrict__ W, const float* __restrict__ bias,
                                                             const uint8_t* __restrict__ keep, int64_t kt, int64_t ka,
                                                             int64_t kb, float* __restrict__ hs,
                                                             float* __restrict__ ws, QHead qh = QHead{}, int Bg = 0) {
    // row chunks (the rows' recurrences are independent): block (a, y) runs rows [y B, y B + B) of the Bg rows
    // (Bg = 0: one chunk of B rows); global rows are indexed in Bg, the LDS state in the chunk
    // (the fused q head's instantiation runs one chunk: QH compiles the chunk arithmetic out)
    extern __shared__ float4 seq_smem[];
    const int64_t rb0 = (!QH && Bg) ? (int64_t)blockIdx.y * B : 0;
    const int64_t BG = (!QH && Bg) ? Bg : B;
    if constexpr (!QH) {
        if (Bg) B = (int)min((int64_t)B, BG - rb0);
        gi += rb0 * 3 * H;
        keep += rb0 * kb;
        if (hs) hs += rb0 * H;
        if (ws) ws += rb0 * 4 * H;
    }
    float* hcur = reinterpret_cast<float*>(seq_smem);
    float* hnxt = hcur + B * H;
    float* hq = hnxt + B * H;      // QH: [2][B][H] step outputs (ping-pong)
    float* wq = hq + 2 * B * H;    // QH: [NA][H] W_q, then [NA] b_q
    const int64_t a = blockIdx.x;
    if (QH) {
        for (int e = threadIdx.x; e < qh.NA * (H + 1); e += kBlock)
            wq[e] = e < qh.NA * H ? qh.W[a * qh.NA * H + e] : qh.b[a * qh.NA + e - qh.NA * H];
    }
    const int tid = threadIdx.x, j = tid % H, bstep = kBlock / H;
    const float* Wa = W + a * 3 * H * H;
    float wr[H], wz[H], wn[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
        wr[i] = Wa[j * H + i];
        wz[i] = Wa[(H + j) * H + i];
        wn[i] = Wa[(2 * H + j) * H + i];
    }
    const float br = bias[a * 3 * H + j], bz = bias[a * 3 * H + H + j], bn = bias[a * 3 * H + 2 * H + j];
    for (int e = tid; e < B * H; e += kBlock) hcur[e] = 0.0f;
    __syncthreads();
    // the global operands (gi, keep) of a thread's RB rows are loaded together, one memory latency per RB rows
    // (config 4: 63.5 -> 60.7 us per launch, 0.1899-0.1905 -> 0.1885-0.1891 ms per step, profiles/r05/grufwd/; the
    // same in gru_seq_bwd_kernel spilled at its two-wave register budget)
    constexpr int RB = 4;
    for (int t = 0; t < C; ++t) {
        for (int b0 = tid / H; b0 < B; b0 += RB * bstep) {
            float gr[RB], gz[RB], gn[RB];
            bool kp[RB];
#pragma unroll
            for (int u = 0; u < RB; ++u) {
                const int b = b0 + u * bstep;
                if (b < B) {
                    const float* g = gi + ((a * C + t) * BG + b) * 3 * H;
                    gr[u] = g[j];
                    gz[u] = g[H + j];
                    gn[u] = g[2 * H + j];
                    kp[u] = keep[t * kt + a * ka + b * kb] != 0;
                }
            }
#pragma unroll
            for (int u = 0; u < RB; ++u) {
                const int b = b0 + u * bstep;
                if (b >= B) break;
                const float4* hp = reinterpret_cast<const float4*>(hcur + b * H);
                float sr = 0.0f, sz = 0.0f, sn = 0.0f;
#pragma unroll
                for (int i4 = 0; i4 < H / 4; ++i4) {
                    const float4 v = hp[i4];
                    sr = fmaf(wr[4 * i4], v.x, sr); sz = fmaf(wz[4 * i4], v.x, sz); sn = fmaf(wn[4 * i4], v.x, sn);
                    sr = fmaf(wr[4 * i4 + 1], v.y, sr); sz = fmaf(wz[4 * i4 + 1], v.y, sz); sn = fmaf(wn[4 * i4 + 1], v.y, sn);
                    sr = fmaf(wr[4 * i4 + 2], v.z, sr); sz = fmaf(wz[4 * i4 + 2], v.z, sz); sn = fmaf(wn[4 * i4 + 2], v.z, sn);
                    sr = fmaf(wr[4 * i4 + 3], v.w, sr); sz = fmaf(wz[4 * i4 + 3], v.w, sz); sn = fmaf(wn[4 * i4 + 3], v.w, sn);
                }
                const int64_t row = (a * C + t) * BG + b;
                const float r = sigmoidf_((sr + br) + gr[u]);
                const float z = sigmoidf_((sz + bz) + gz[u]);
                const float ghn = sn + bn;
                const float nn = tanhf(gn[u] + ghn * r);
                const float hv = hcur[b * H + j];
                const float ho = (hv - nn) * z + nn;
                if (!QH || hs) hs[row * H + j] = ho;
                if (QH) hq[(t & 1) * B * H + b * H + j] = ho;
                if (ws) {
                    float* w = ws + row * 4 * H;
                    w[j] = r;
                    w[H + j] = z;
                    w[2 * H + j] = nn;
                    w[3 * H + j] = ghn;
                }
                hnxt[b * H + j] = kp[u] ? ho : 0.0f;
            }
        }
        __syncthreads();
        if (QH) {  // q of step t (its h' stay in hq[t & 1] until after the next step's barrier)
            const float* hb = hq + (t & 1) * B * H;
            for (int e = threadIdx.x; e < B * qh.NA; e += kBlock) {
                const int b = e / qh.NA, o = e - b * qh.NA;
                const float4* w4 = reinterpret_cast<const float4*>(wq + o * H);
                const float4* h4 = reinterpret_cast<const float4*>(hb + b * H);
                float acc = wq[qh.NA * H + o];
#pragma unroll
                for (int k4 = 0; k4 < H / 4; ++k4) {
                    const float4 w = w4[k4], h = h4[k4];
                    acc = fmaf(w.x, h.x, acc);
                    acc = fmaf(w.y, h.y, acc);
                    acc = fmaf(w.z, h.z, acc);
                    acc = fmaf(w.w, h.w, acc);
                }
                qh.q[((a * C + t) * BG + rb0 + b) * qh.NA + o] = acc;
            }
        }
        float* tmp = hcur;
        hcur = hnxt;
        hnxt = tmp;
    }
}

// Backpropagation through gru_seq_fwd_kernel's chunk, one block per network, t = C-1 .. 0:
//   go = dhs[t] + carry;  gate gradients as gru_bwd_kernel -> dgi[t] (= dgh for the r, z gates; dgh_n = dan r)
//   dh_prev = go z + dgh W_hh;  carry = keep[t-1] ? dh_prev : 0
//   dW_hh += dgh^T h_prev, db_hh += sum_b dgh   (h_prev = keep[t-1] ? hs[t-1] : 0, zero at t = 0)
// dW / db are written (this recurrence is their only use inside the chunk). LDS: dgh [B][3H], h_prev and carry
// [B][H]. Thread (i, b) for dh_prev keeps column i of W_hh in registers; thread tid owns the dW entries (g, tid % H)
// of the gate quads tid / H + (256 / H) u.
// QH (the fused q head's backward): dhs is dq [A][C][B][NA] (the gradient of the q values); the step's dL/dh' is
// dq W_q (column i of W_q in registers), and dW_q = sum_(t,b) dq^T h', db_q = sum_(t,b) dq accumulate per thread over
// its rows and steps, then over the kBlock / H row groups in a fixed order (LDS) -> dWq [A][NA][H], dbq [A][NA].
struct QHeadBwd {
    const float* W;  // [A][NA][H]
    float* dW;       // [A][NA][H]
    float* db;       // [A][NA]
    int NA;
};
constexpr int kMaxQ = 16;
template <int H, int NQ = 0>  // NQ > 0: the q head fused, at most NQ actions (registers sized for NQ)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2))) void gru_seq_bwd_kernel(int C, int B, const float* __restrict__ dhs,
                                                             const float* __restrict__ hs, const float* __restrict__ ws,
                                                             const float* __restrict__ W,
                                                             const uint8_t* __restrict__ keep, int64_t kt, int64_t ka,
                                                             int64_t kb, float* __restrict__ dgi,
                                                             float* __restrict__ dW, float* __restrict__ db,
                                                             QHeadBwd qh = QHeadBwd{}, int Bg = 0, int64_t rb0 = 0,
                                                             int acc = 0) {
    // row chunk (non-QH): rows [rb0, rb0 + B) of Bg (Bg = 0: all B rows); acc: dW / db += this chunk's sums (chunks
    // launched in order on one stream, so the sums run over the chunks in row order)
    constexpr bool QH = NQ > 0;
    const int64_t BG = (!QH && Bg) ? Bg : B;
    if constexpr (!QH) {
        dhs += rb0 * H;
        hs += rb0 * H;
        ws += rb0 * 4 * H;
        keep += rb0 * kb;
        dgi += rb0 * 3 * H;
    } else {
        acc = 0;
    }
    constexpr int NQA = QH ? NQ : 1;
    constexpr int G = 3 * H, NW = G * H / kBlock;  // dW entries per thread
    extern __shared__ float4 seq_smem[];
    float* dgh = reinterpret_cast<float*>(seq_smem);  // [B][G]
    float* hprev = dgh + B * G;                        // [B][H]
    float* carry = hprev + B * H;                      // [B][H]
    const int64_t a = blockIdx.x;
    const int tid = threadIdx.x, i = tid % H, bstep = kBlock / H;
    // QH: W_q in LDS behind carry ([NA][H]); dW_q[:, i] partials in registers; lanes i < NA also sum db_q[i]
    float* wq = carry + B * H;
    float* dqs = wq + (QH ? qh.NA * H : 0);  // QH: [B][NA] dq of the step
    float aqb = 0.0f;
    // dW_q partials: thread-private LDS slots [kBlock / H][NA][H] (no sharing: no barrier; keeps the 256-VGPR
    // budget of two waves per SIMD without spills)
    float* aqs = dqs + (QH ? B * qh.NA : 0);
    const int grp0 = tid / H;
    if (QH)
        for (int o = 0; o < qh.NA; ++o) aqs[(grp0 * qh.NA + o) * H + i] = 0.0f;
    if (QH)
        for (int e = tid; e < qh.NA * H; e += kBlock) wq[e] = qh.W[a * qh.NA * H + e];
    const float* Wa = W + a * G * H;
    float wc[G];  // column i of W_hh
#pragma unroll
    for (int g = 0; g < G; ++g) wc[g] = Wa[g * H + i];
    float accw[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) accw[q] = 0.0f;
    float accb = 0.0f;
    for (int e = tid; e < B * H; e += kBlock) carry[e] = 0.0f;
    for (int t = C - 1; t >= 0; --t) {
        // h_prev of step t (the reset previous output), and the gate gradients
        for (int e = tid; e < B * H; e += kBlock) {
            const int b = e / H;
            float v = 0.0f;
            if (t > 0 && keep[(t - 1) * kt + a * ka + b * kb]) v = hs[((a * C + t - 1) * BG + b) * H + (e - b * H)];
            hprev[e] = v;
        }
        if (QH)  // this step's dq rows (contiguous [B][NA]) into LDS: one coalesced round trip, broadcast reads below
            for (int e = tid; e < B * qh.NA; e += kBlock) dqs[e] = dhs[(a * C + t) * B * qh.NA + e];
        __syncthreads();  // carry (previous iteration), hprev and dq visible
        for (int b = tid / H; b < B; b += bstep) {
            const int64_t row = (a * C + t) * BG + b;
            const float* w = ws + row * 4 * H;
            const float r = w[i], z = w[H + i], nn = w[2 * H + i], ghn = w[3 * H + i];
            float dho;
            if (QH) {  // dL/dh' of the q head: dq W_q, k-ordered; and its dW_q / db_q partials
                const float* dq = dqs + b * qh.NA;
                const float ho = hs[row * H + i];
                dho = 0.0f;
#pragma unroll 2
                for (int o = 0; o < NQA; ++o)
                    if (o < qh.NA) {
                        const float d = dq[o];
                        dho = fmaf(d, wq[o * H + i], dho);
                        float* slot = aqs + (grp0 * qh.NA + o) * H + i;
                        *slot = fmaf(d, ho, *slot);
                    }
                if (i < qh.NA) aqb += dq[i];
            } else {
                dho = dhs[row * H + i];
            }
            const float go = dho + carry[b * H + i];
            const float hv = hprev[b * H + i];
            const float dn = go * (1.0f - z);
            const float dz = go * (hv - nn);
            const float dan = dn * (1.0f - nn * nn);
            const float dr = dan * ghn;
            const float dar = dr * (r * (1.0f - r));
            const float daz = dz * (z * (1.0f - z));
            float* gi_ = dgi + row * G;
            gi_[i] = dar;
            gi_[H + i] = daz;
            gi_[2 * H + i] = dan;
            dgh[b * G + i] = dar;
            dgh[b * G + H + i] = daz;
            dgh[b * G + 2 * H + i] = dan * r;
            carry[b * H + i] = go * z;  // the direct term of dh_prev; the W_hh term is added below
        }
        __syncthreads();
        // dW_hh / db_hh partial sums of this step. Thread (ii = tid % H, m0 = tid / H) owns the NW entries
        // (g, ii) with g in the gate quads m0 + (kBlock / H) u: per row b ONE hprev read and NW / 4 float4 reads of
        // dgh (broadcast within the wave) instead of 2 NW scalar reads; each entry's sum runs over b in the same
        // order as before (same bits)
        {
            constexpr int NGQ = NW / 4, QS = kBlock / H;  // gate quads per thread, quad stride
            static_assert(NW % 4 == 0 && G % 4 == 0 && (G / 4) == NGQ * QS, "gru_seq_bwd: dW tiling");
            const int ii = tid % H, m0 = tid / H;
            float s[NW];
#pragma unroll
            for (int q = 0; q < NW; ++q) s[q] = 0.0f;
            for (int b = 0; b < B; ++b) {
                const float hv = hprev[b * H + ii];
                const float4* d4 = reinterpret_cast<const float4*>(dgh + b * G);
#pragma unroll
                for (int u = 0; u < NGQ; ++u) {
                    const float4 v = d4[m0 + QS * u];
                    s[4 * u + 0] = fmaf(v.x, hv, s[4 * u + 0]);
                    s[4 * u + 1] = fmaf(v.y, hv, s[4 * u + 1]);
                    s[4 * u + 2] = fmaf(v.z, hv, s[4 * u + 2]);
                    s[4 * u + 3] = fmaf(v.w, hv, s[4 * u + 3]);
                }
            }
#pragma unroll
            for (int q = 0; q < NW; ++q) accw[q] += s[q];
        }
        if (tid < G) {
            float s = 0.0f;
            for (int b = 0; b < B; ++b) s += dgh[b * G + tid];
            accb += s;
        }
        // dh_prev = go z + dgh W_hh, masked by the reset that produced h_prev
        for (int b = tid / H; b < B; b += bstep) {
            const float4* d4 = reinterpret_cast<const float4*>(dgh + b * G);
            float s = 0.0f;
#pragma unroll
            for (int g4 = 0; g4 < G / 4; ++g4) {
                const float4 v = d4[g4];
                s = fmaf(v.x, wc[4 * g4], s);
                s = fmaf(v.y, wc[4 * g4 + 1], s);
                s = fmaf(v.z, wc[4 * g4 + 2], s);
                s = fmaf(v.w, wc[4 * g4 + 3], s);
            }
            const bool kept = t > 0 && keep[(t - 1) * kt + a * ka + b * kb];
            carry[b * H + i] = kept ? carry[b * H + i] + s : 0.0f;
        }
        __syncthreads();  // dgh / hprev reads done before the next step overwrites them
    }
#pragma unroll
    for (int q = 0; q < NW; ++q) {  // entry (g, ii) of thread tid: g = 4 (m0 + (kBlock / H) (q / 4)) + q % 4
        const int g = 4 * (tid / H + (kBlock / H) * (q >> 2)) + (q & 3);
        float* d = dW + a * G * H + g * H + tid % H;
        *d = acc ? *d + accw[q] : accw[q];
    }
    if (tid < G) db[a * G + tid] = acc ? db[a * G + tid] + accb : accb;
    if (QH) {  // the q head's gradients: the bstep row groups' partials summed in group order
        float* redb = dgh;  // [bstep][NA] db_q partials (the loop is done with dgh: its last barrier)
        const int grp = tid / H;
        if (i < qh.NA) redb[grp * qh.NA + i] = aqb;
        __syncthreads();
        for (int e = tid; e < qh.NA * H; e += kBlock) {
            float s = 0.0f;
            for (int q = 0; q < bstep; ++q) s += aqs[q * qh.NA * H + e];
            qh.dW[a * qh.NA * H + e] = s;
        }
        if (tid < qh.NA) {
            float s = 0.0f;
            for (int q = 0; q < bstep; ++q) s += redb[q * qh.NA + tid];
            qh.db[a * qh.NA + tid] = s;
        }
    }
}

__global__ __launch_bounds__(kBlock) void gather_rows_kernel(int64_t rows, int64_t width, const float* __restrict__ src,
                                                             const int64_t* __restrict__ idx, float* __restrict__ dst,
                                                             int scatter) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
    const bool vec = (width & 3) == 0;
    for (int64_t r = wave; r < rows; r += nwaves) {
        const int64_t ir = idx[r];
        const float* s = scatter ? src + r * width : src + ir * width;
        float* d = scatter ? dst + ir * width : dst + r * width;
        if (vec) {
            const float4* s4 = reinterpret_cast<const float4*>(s);
            float4* d4 = reinterpret_cast<float4*>(d);
            for (int64_t c = lane; c < width / 4; c += 64) d4[c] = s4[c];
        } else {
            for (int64_t c = lane; c < width; c += 64) d[c] = s[c];
        }
    }
}

// replay-ring insert: every field of n rows at ring rows start .. start + n - 1 (mod cap), one launch for all fields
// (grid.y = field). kind 0: f32 copy; 1: u8 (bool) -> 1 - x (the reference's stored "terminal", utils.py:52);
// 2: u8 -> x. float4 / uchar4 vectors when the field's flat offsets are multiples of 4 (never straddling the wrap).
struct RingStore {
    FlockRingField f[8];
    int nf;
    int64_t n, cap, start;
};

__global__ __launch_bounds__(kBlock) void ring_store_kernel(RingStore rs) {
    const FlockRingField F = rs.f[blockIdx.y];
    const int64_t total = rs.n * F.width, wrap = rs.cap * F.width, d0 = rs.start * F.width;
    const bool i64 = F.kind == 3;  // int64 -> f32 (torch .float(): round to nearest)
    const bool u8 = F.kind == 1 || F.kind == 2;
    const bool vec = !i64 && ((total | wrap | d0) & 3) == 0 && ((uintptr_t)F.dst & 15) == 0 &&
                     ((uintptr_t)F.src & (u8 ? 3 : 15)) == 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    if (vec) {
        for (int64_t q = blockIdx.x * (int64_t)kBlock + threadIdx.x; q < total / 4; q += stride) {
            float4 v;
            if (!u8) {
                v = reinterpret_cast<const float4*>(F.src)[q];
            } else {
                const uchar4 b = reinterpret_cast<const uchar4*>(F.src)[q];
                v = make_float4(b.x, b.y, b.z, b.w);
                if (F.kind == 1) v = make_float4(1.0f - v.x, 1.0f - v.y, 1.0f - v.z, 1.0f - v.w);
            }
            int64_t d = d0 + 4 * q;
            if (d >= wrap) d -= wrap;
            *reinterpret_cast<float4*>(F.dst + d) = v;
        }
    } else {
        for (int64_t q = blockIdx.x * (int64_t)kBlock + threadIdx.x; q < total; q += stride) {
            float v;
            if (i64) {
                v = (float)reinterpret_cast<const int64_t*>(F.src)[q];
            } else if (!u8) {
                v = reinterpret_cast<const float*>(F.src)[q];
            } else {
                v = (float)reinterpret_cast<const uint8_t*>(F.src)[q];
                if (F.kind == 1) v = 1.0f - v;
            }
            int64_t d = d0 + q;
            if (d >= wrap) d -= wrap;
            F.dst[d] = v;
        }
    }
}

}  // namespace

extern "C" {

int flock_ring_store(void* stream, int64_t n, int64_t capacity, int64_t start, int nfields,
                     const FlockRingField* fields) {
    if (n <= 0) return 0;
    if (!fields || nfields < 1 || nfields > 8) return fail(-5, "flock_ring_store: 1..8 fields");
    if (n > capacity || start < 0 || start >= capacity)
        return fail(-5, "flock_ring_store: need n <= capacity and 0 <= start < capacity");
    RingStore rs;
    int64_t widest = 0;
    for (int i = 0; i < nfields; ++i) {
        if (!fields[i].src || !fields[i].dst) return fail(-3, "flock_ring_store: NULL pointer");
        if (fields[i].width < 1 || fields[i].kind < 0 || fields[i].kind > 3)
            return fail(-5, "flock_ring_store: bad field");
        rs.f[i] = fields[i];
        if (fields[i].width > widest) widest = fields[i].width;
    }
    rs.nf = nfields;
    rs.n = n;
    rs.cap = capacity;
    rs.start = start;
    int64_t blocks = (n * widest / 4 + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(ring_store_kernel, dim3((unsigned)blocks, nfields), dim3(kBlock), 0, (hipStream_t)stream, rs);
    return launched();
}

const char* flock_learn_last_error(void) { return flock_learn_internal::g_err; }

int flock_adam_step(void* stream, int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                    const float* grad_scale, float lr, float beta1, float beta2, float eps, int64_t step,
                    float* target, float tau, int target_mode) {
    if (n <= 0) return 0;
    if (!param || !grad || !exp_avg || !exp_avg_sq) return fail(-3, "flock_adam_step: NULL pointer");
    if (step < 1) return fail(-5, "flock_adam_step: step must be >= 1");
    // bias corrections in double then rounded, like the python-float math of _single_tensor_adam
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    AdamArgs a{n, param, exp_avg, exp_avg_sq, target, grad, grad_scale, nullptr, lr, beta1, beta2,
               (float)(1.0 - (double)beta1), (float)(1.0 - (double)beta2), (float)(-(double)lr / bc1),
               (float)sqrt(bc2), eps, tau, (float)(1.0 - (double)tau), target_mode};
    return launch_adam(stream, a);
}

int flock_adam_step_dev(void* stream, int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        const float* grad_scale, float lr, float beta1, float beta2, float eps, const int64_t* step,
                        float* target, float tau, int target_mode) {
    if (n <= 0) return 0;
    if (!param || !grad || !exp_avg || !exp_avg_sq || !step) return fail(-3, "flock_adam_step_dev: NULL pointer");
    AdamArgs a{n, param, exp_avg, exp_avg_sq, target, grad, grad_scale, step, lr, beta1, beta2,
               (float)(1.0 - (double)beta1), (float)(1.0 - (double)beta2), 0.0f, 1.0f, eps, tau,
               (float)(1.0 - (double)tau), target_mode};
    return launch_adam(stream, a);
}

int flock_soft_update(void* stream, int64_t n, float* target, const float* src, float tau, int mode) {
    if (n <= 0) return 0;
    if (!target || !src) return fail(-3, "flock_soft_update: NULL pointer");
    if (aligned16(target) && aligned16(src))
        hipLaunchKernelGGL(soft_update_kernel<true>, dim3(grid_for(n, 4)), dim3(kBlock), 0, (hipStream_t)stream, n,
                           target, src, tau, (float)(1.0 - (double)tau), mode);
    else
        hipLaunchKernelGGL(soft_update_kernel<false>, dim3(grid_for(n, 4)), dim3(kBlock), 0, (hipStream_t)stream, n,
                           target, src, tau, (float)(1.0 - (double)tau), mode);
    return launched();
}

int flock_grad_norm(void* stream, int64_t n, const float* grad, double* partial, int max_parts, float max_norm,
                    float* out) {
    if (!grad || !partial || !out) return fail(-3, "flock_grad_norm: NULL pointer");
    int parts = grid_for(n);
    if (parts > max_parts) parts = max_parts;
    hipLaunchKernelGGL(sq_partial_kernel, dim3(parts), dim3(kBlock), 0, (hipStream_t)stream, n, grad, partial);
    hipLaunchKernelGGL(sq_final_kernel, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, parts, partial, max_norm, out);
    return launched();
}

int flock_gru_fwd(void* stream, int64_t rows, int H, const float* gi, const float* gh, const float* h, float* hout,
                  float* ws) {
    if (rows <= 0) return 0;
    if (!gi || !gh || !h || !hout) return fail(-3, "flock_gru_fwd: NULL pointer");
    hipLaunchKernelGGL(gru_fwd_kernel, dim3(grid_for(rows * H)), dim3(kBlock), 0, (hipStream_t)stream, rows, H, gi,
                       gh, h, hout, ws);
    return launched();
}

int flock_gru_bwd(void* stream, int64_t rows, int H, const float* dhout, const float* h, const float* ws, float* dgi,
                  float* dgh, float* dh) {
    if (rows <= 0) return 0;
    if (!dhout || !h || !ws || !dgi || !dgh || !dh) return fail(-3, "flock_gru_bwd: NULL pointer");
    hipLaunchKernelGGL(gru_bwd_kernel, dim3(grid_for(rows * H)), dim3(kBlock), 0, (hipStream_t)stream, rows, H, dhout,
                       h, ws, dgi, dgh, dh);
    return launched();
}

// rows per block of the whole-chunk GRU recurrences: LDS [2][rows][32] floats forward (<= 160 KB: 640 rows), [5][rows]
// [32] backward (256 rows)
constexpr int kSeqRows = 640, kSeqBwdRows = 256;

int flock_gru_seq_fwd(void* stream, int A, int C, int B, int H, const float* gi, const float* w_hh, const float* b_hh,
                      const uint8_t* keep, int64_t keep_st, int64_t keep_sa, int64_t keep_sb, float* hs, float* ws) {
    if (A <= 0 || C <= 0 || B <= 0) return 0;
    if (!gi || !w_hh || !b_hh || !keep || !hs) return fail(-3, "flock_gru_seq_fwd: NULL pointer");
    if (H != 32) return fail(-2, "flock_gru_seq_fwd: hidden size must be 32");
    // more rows than one block's LDS holds (e.g. the union batch of agent-sharded critics at 8 ranks): row chunks of
    // kSeqRows in grid y (the rows' recurrences are independent)
    const int Bc = B <= kSeqRows ? B : kSeqRows, nch = (B + Bc - 1) / Bc;
    const size_t lds = (size_t)2 * Bc * H * sizeof(float);
    if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(gru_seq_fwd_kernel<32>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(-4, "flock_gru_seq_fwd: cannot raise the LDS limit");
    hipLaunchKernelGGL(gru_seq_fwd_kernel<32>, dim3(A, nch), dim3(kBlock), lds, (hipStream_t)stream, C, Bc, gi, w_hh,
                       b_hh, keep, keep_st, keep_sa, keep_sb, hs, ws, QHead{}, nch > 1 ? B : 0);
    return launched();
}

int flock_gru_seq_q_fwd(void* stream, int A, int C, int B, int H, int NA, const float* gi, const float* w_hh,
                        const float* b_hh, const float* w_q, const float* b_q, const uint8_t* keep, int64_t keep_st,
                        int64_t keep_sa, int64_t keep_sb, float* hs, float* ws, float* q) {
    if (A <= 0 || C <= 0 || B <= 0) return 0;
    if (!gi || !w_hh || !b_hh || !w_q || !b_q || !keep || !q) return fail(-3, "flock_gru_seq_q_fwd: NULL pointer");
    if (H != 32) return fail(-2, "flock_gru_seq_q_fwd: hidden size must be 32");
    if (NA < 1 || NA > kMaxQ) return fail(-2, "flock_gru_seq_q_fwd: 1 <= n_actions <= 16");
    if (ws && !hs) return fail(-3, "flock_gru_seq_q_fwd: ws needs hs (the backward reads both)");
    const size_t lds = ((size_t)4 * B * H + (size_t)NA * (H + 1)) * sizeof(float);
    if (lds > 160 * 1024) return fail(-2, "flock_gru_seq_q_fwd: B too large for LDS");
    if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(gru_seq_fwd_kernel<32, true>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(-4, "flock_gru_seq_q_fwd: cannot raise the LDS limit");
    hipLaunchKernelGGL((gru_seq_fwd_kernel<32, true>), dim3(A), dim3(kBlock), lds, (hipStream_t)stream, C, B, gi, w_hh,
                       b_hh, keep, keep_st, keep_sa, keep_sb, hs, ws, QHead{w_q, b_q, q, NA}, 0);
    return launched();
}

int flock_gru_seq_q_bwd(void* stream, int A, int C, int B, int H, int NA, const float* dq, const float* hs,
                        const float* ws, const float* w_hh, const float* w_q, const uint8_t* keep, int64_t keep_st,
                        int64_t keep_sa, int64_t keep_sb, float* dgi, float* dw_hh, float* db_hh, float* dw_q,
                        float* db_q) {
    if (A <= 0 || C <= 0 || B <= 0) return 0;
    if (!dq || !hs || !ws || !w_hh || !w_q || !keep || !dgi || !dw_hh || !db_hh || !dw_q || !db_q)
        return fail(-3, "flock_gru_seq_q_bwd: NULL pointer");
    if (H != 32) return fail(-2, "flock_gru_seq_q_bwd: hidden size must be 32");
    if (NA < 1 || NA > kMaxQ) return fail(-2, "flock_gru_seq_q_bwd: 1 <= n_actions <= 16");
    // dgh, h_prev, carry, W_q; the q head's final reduction ((kBlock / H) (NA H + NA) floats) reuses the same space
    // from its start once the recurrence is done
    const size_t body = (size_t)B * (3 * H + 2 * H + NA) + (size_t)NA * H + (size_t)(kBlock / H) * NA * H;
    const size_t red = (size_t)(kBlock / H) * NA;  // the db_q partials over dgh at the end
    const size_t lds = (body > red ? body : red) * sizeof(float);
    if (lds > 160 * 1024) return fail(-2, "flock_gru_seq_q_bwd: B too large for LDS");
    const QHeadBwd qh{w_q, dw_q, db_q, NA};
    auto go = [&](auto kern) {
        if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return fail(-4, "flock_gru_seq_q_bwd: cannot raise the LDS limit");
        hipLaunchKernelGGL(kern, dim3(A), dim3(kBlock), lds, (hipStream_t)stream, C, B, dq, hs, ws, w_hh, keep,
                           keep_st, keep_sa, keep_sb, dgi, dw_hh, db_hh, qh, 0, (int64_t)0, 0);
        return launched();
    };
    // registers sized for the head: the smallest instantiation that holds NA
    if (NA <= 4) return go(gru_seq_bwd_kernel<32, 4>);
    if (NA <= 6) return go(gru_seq_bwd_kernel<32, 6>);
    if (NA <= 8) return go(gru_seq_bwd_kernel<32, 8>);
    if (NA <= 10) return go(gru_seq_bwd_kernel<32, 10>);
    return go(gru_seq_bwd_kernel<32, 16>);
}

int flock_gru_seq_bwd(void* stream, int A, int C, int B, int H, const float* dhs, const float* hs, const float* ws,
                      const float* w_hh, const uint8_t* keep, int64_t keep_st, int64_t keep_sa, int64_t keep_sb,
                      float* dgi, float* dw_hh, float* db_hh) {
    if (A <= 0 || C <= 0 || B <= 0) return 0;
    if (!dhs || !hs || !ws || !w_hh || !keep || !dgi || !dw_hh || !db_hh)
        return fail(-3, "flock_gru_seq_bwd: NULL pointer");
    if (H != 32) return fail(-2, "flock_gru_seq_bwd: hidden size must be 32");
    // more rows than one block's LDS holds: row chunks of kSeqBwdRows launched in order, each adding its dW / db sums
    const int Bc = B <= kSeqBwdRows ? B : kSeqBwdRows;
    const size_t lds = (size_t)Bc * (3 * H + 2 * H) * sizeof(float);
    if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(gru_seq_bwd_kernel<32>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return fail(-4, "flock_gru_seq_bwd: cannot raise the LDS limit");
    for (int b0 = 0; b0 < B; b0 += Bc) {
        const int n = B - b0 < Bc ? B - b0 : Bc;
        hipLaunchKernelGGL(gru_seq_bwd_kernel<32>, dim3(A), dim3(kBlock), lds, (hipStream_t)stream, C, n, dhs, hs, ws,
                           w_hh, keep, keep_st, keep_sa, keep_sb, dgi, dw_hh, db_hh, QHeadBwd{}, Bc < B ? B : 0,
                           (int64_t)b0, b0 > 0 ? 1 : 0);
        if (int rc = launched()) return rc;
    }
    return 0;
}

int flock_vdn_feat_fwd(void* stream, int A, int R, int B, int n_in, const float* x, int64_t x_sa, int64_t x_sc,
                       int64_t x_sb, const float* w1, const float* b1, const float* w2, const float* b2,
                       const float* w_ih, const float* b_ih, float* y1, float* y2, float* gi) {
    if (A <= 0 || R <= 0) return 0;
    if (!x || !w1 || !b1 || !w2 || !b2 || !w_ih || !b_ih || !gi) return fail(-3, "flock_vdn_feat_fwd: NULL pointer");
    if (n_in < 1 || n_in > kFMaxIn) return fail(-2, "flock_vdn_feat_fwd: n_in must be in [1, 16]");
    if (B < 1 || R % B != 0) return fail(-5, "flock_vdn_feat_fwd: R must be a multiple of B");
    hipLaunchKernelGGL(vdn_feat_fwd_kernel, dim3(A), dim3(kBlock), 0, (hipStream_t)stream,
                       R, B, n_in, x, x_sa, x_sc, x_sb, w1, b1, w2, b2, w_ih, b_ih, y1, y2, gi);
    return launched();
}

int flock_vdn_feat_bwd(void* stream, int A, int R, int B, int n_in, const float* x, int64_t x_sa, int64_t x_sc,
                       int64_t x_sb, const float* w2, const float* w_ih, const float* y1, const float* y2,
                       const float* dgi, float* dw1, float* db1, float* dw2, float* db2, float* dw_ih,
                       float* db_ih) {
    if (A <= 0) return 0;
    if (!x || !w2 || !w_ih || !y1 || !y2 || !dgi || !dw1 || !db1 || !dw2 || !db2 || !dw_ih || !db_ih)
        return fail(-3, "flock_vdn_feat_bwd: NULL pointer");
    if (n_in < 1 || n_in > kFMaxIn) return fail(-2, "flock_vdn_feat_bwd: n_in must be in [1, 16]");
    if (R < 1 || B < 1 || R % B != 0) return fail(-5, "flock_vdn_feat_bwd: R must be a positive multiple of B");
    hipLaunchKernelGGL(vdn_feat_bwd_kernel, dim3(A), dim3(kBB), 0, (hipStream_t)stream, R, B, n_in, x, x_sa, x_sc,
                       x_sb, w2, w_ih, y1, y2, dgi, dw1, db1, dw2, db2, dw_ih, db_ih);
    return launched();
}

int flock_gather_rows(void* stream, int64_t rows, int64_t width, const float* src, const int64_t* idx, float* dst) {
    if (rows <= 0) return 0;
    if (!src || !idx || !dst) return fail(-3, "flock_gather_rows: NULL pointer");
    int blocks = (int)((rows * 64 + kBlock - 1) / kBlock);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, rows, width, src, idx,
                       dst, 0);
    return launched();
}

int flock_scatter_rows(void* stream, int64_t rows, int64_t width, const float* src, const int64_t* idx, float* dst) {
    if (rows <= 0) return 0;
    if (!src || !idx || !dst) return fail(-3, "flock_scatter_rows: NULL pointer");
    int blocks = (int)((rows * 64 + kBlock - 1) / kBlock);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, rows, width, src, idx,
                       dst, 1);
    return launched();
}

}  // extern "C"
