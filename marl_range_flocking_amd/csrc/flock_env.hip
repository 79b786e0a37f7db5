// flock_env.hip — MI355X (gfx950) batched flocking-environment stepper. C ABI: include/flock_amd.h.
//
// One launch per vectorized step. A workgroup owns G whole envs (G = 256 / N for N <= 256, else 1; one agent per
// lane), so every agent-agent pair of an env is visible in the workgroup's LDS and nothing crosses workgroups.
//
//   phase 1  kinematics + check_boundary for the lane's agent (reference _updateState / check_boundary), the new
//            position is stored to HBM and to LDS [env][agent] (float2, env stride padded to even)
//   phase 2  per-env float sums in a fixed power-of-two LDS tree (uw: centre of mass; uw_discrete: mean heading)
//   phase 3  all-pairs scan: the lane streams its env's N positions from LDS (broadcast ds_read_b128, two
//            candidates per read), computes d2 with the reference's op order, packs
//            key = (bits(d2) with the low IB mantissa bits cleared) | j  (IB = ceil(log2 N)),
//            and keeps the L = k+2 smallest keys in registers with a branch-free insertion network
//            (1 v_min_u32 + (L-1) v_med3_u32 per candidate; no divergence, no sort)
//            Step variants with N >= 128 scan a CELL LIST instead of all N (phase 3c below).
//   phase 3c agents are binned into a Gx x Gy grid (about one agent per cell, rows about twice the typical
//            (k+1)-th neighbour distance tall) by an LDS counting sort (block-wide DPP prefix scan) into an extended
//            cell-sorted array of (x, y, j, sx) in which every cell row also carries ghost copies of its last and first
//            kRg columns when the box is periodic, so any run of up to 2 kRg + 1 columns of a row is one contiguous
//            range. SEEDED scan (the usual case): nn_idx holds the previous step's neighbours on entry; the lane's
//            own agent and those k seeds are k+1 distinct agents, so their largest current distance bounds the
//            (k+1)-th nearest, and every agent inside the disk of that radius (widened by >= 16 truncated-d2
//            buckets) is scanned: the cells under the disk, at most kRows rows, each row's chord one range, all
//            rows streamed as ONE sequence per lane (the wave loops max-over-lanes(total) slots, not a per-row
//            maximum per row). Every agent outside the disk has a larger key than the (k+1)-th smallest, so the
//            top k+1 keys and the ambiguity test of phase 4 are exactly the full scan's. Lanes without usable
//            seeds (first step, stale or invalid indices, too large a radius) take a SQUARE scan (rows cy +- 1,
//            columns cx +- kRg) kept only if PROVABLY the full scan's: every unscanned agent lies at least m = the
//            distance to the block's edge away (no agents beyond a box edge without wrap), so if the truncated-d2
//            bucket of m^2 (shrunk by a 1e-5 safety factor) exceeds the L-th key, no unscanned key can enter the top
//            L; only then the full scan. An ambiguous bucket (phase 4) is rescanned exactly over the square, which
//            contains every candidate of that bucket in both cases. Keys carry j, so the order of agents within a
//            cell (LDS atomics) never matters.
//   phase 4  exactness: the k+1 winners are re-sorted by their exact (d2, j); if the (k+2)-th key shares the
//            truncated-d2 bucket of the (k+1)-th, the lane falls back to an exact (d2, j) rescan (rare). The
//            result is the ascending (d2, j) order — a valid tie resolution of the reference's
//            topk(-sqrt(d2), k+1) — identical to oracle/flock_oracle.c.
//   phase 5  distances (correctly-rounded sqrt of the k winners only), clamp, collisions, done, per-env any_done
//            (LDS atomic OR), reward, observation memory roll.
//
// Float arithmetic: every op is rounded separately (__fmul_rn / __fadd_rn / __fdiv_rn / sqrt_rn, and the file
// is built with -ffp-contract=off), in the reference's op order; cosf/sinf are ocml's (sincosf: the same bits).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flock_amd.h"
#include "flock_mem.h"

#pragma clang fp contract(off)

namespace {

constexpr int kMem = 4;  // observation memory depth (gym_flock_uw.py:59, gym_flock.py:42)
constexpr int kSense = 4;  // internal variant: kNN only (flock_knn)
constexpr float kHalfPi = 1.57079637f;  // float(pi/2): torch.clamp casts the bound to float (gym_flock_v2.py:327)
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

thread_local char g_err[256] = "";

int fail(int code, const char* msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return code;
}

struct Params {
    int E, N, k, G, S, P, ib;
    int env0;  // first env of this launch (a step split into several launches; 0 otherwise)
    int pf_ahead;  // > 0: each block pulls the inputs of block blockIdx.x + pf_ahead into L2 (step_kernel's PFM)
    int launches;  // FlockStepExt.launches: the step as this many launches over env ranges (0: the diagnostics knob)
    int variant, periodic, rigid, clamp;
    float box, sensor_range, cd, dt, v_min, v_max, noise_std, com_r;
    uint64_t seed, rng_offset;
    int n_actions;
    float* pos;
    float* heading;
    float* prev_heading;
    float* vel;
    const float* action;
    const int64_t* action_id;
    const float* noise;
    const float* table;
    const float* mem_in;
    float* mem_out;
    float* dnn;
    int64_t* idx;
    float* reward;
    uint8_t* done;
    uint8_t* any_done;
    int* status;
    // fused replay insert (flock_step_v2_store)
    float *r_state, *r_action, *r_reward, *r_new, *r_term, *r_astate, *r_anew;
    const float* r_prev;
    int64_t r_cap, r_start, r_skip;
    int r_group, r_done;  // agents per ring row (1 or N); stored flag: 0 -> 1 - done, 1 -> done
    int r_ids, r_env_done;  // action stored as the f32 action id; terminal one flag per env row (any_done)
    uint16_t* seeds;      // [E][N][k] compact kNN search seeds (rw), or NULL: nn_idx on entry is the hint
    // cell list (step variants, N >= 128)
    int cells, gx, gy, ecap;  // cells != 0: cell list on a gx x gy grid; extended-array capacity per env (2N + 2)
    float cwx, cwy, inv_cwx, inv_cwy, cell_eps, r_lim;
    // reset
    float range_lo, range_hi, head_hi, check_distance;
    int max_attempts, repair;
    const uint8_t* env_mask;
    uint8_t* valid;
    int normalize;  // normalize_distance: Euclidean kNN of positions / max_e |p| (full-scan path only, see dispatch)
};

// ---------------------------------------------------------------------------------------------------------------
// phase timing (diagnostics build only: tools/phase_prof.py compiles this file with -DFLOCK_PHASE_PROF into a
// separate library; the product build has no counters)
#ifdef FLOCK_PHASE_PROF
// 64 slots x 32 counters (slot = blockIdx mod 64) so the end-of-kernel atomics do not pile onto one address
__device__ unsigned long long g_phase[64 * 32];
__device__ unsigned long long g_blk[4096][2];  // per block: start (thread 0) and end (max over waves), s_memrealtime
__device__ unsigned long long g_blkph[4096][8];  // per block: thread 0's s_memrealtime at each phase mark
#define PHASE(n)                                                             \
    do {                                                                     \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
        ph_acc[n] += t_ - t_prev;                                            \
        t_prev = t_;                                                         \
        if (threadIdx.x == 0 && blockIdx.x < 4096)                           \
            g_blkph[blockIdx.x][n] = __builtin_amdgcn_s_memrealtime();       \
    } while (0)
#define PHASE_COUNT(n, v) \
    do {                  \
        ph_acc[n] += (v); \
    } while (0)
#define PHASE_FLUSH()                                                                               \
    do {                                                                                            \
        ph_acc[19] += __builtin_amdgcn_s_memtime() - st0_;                                          \
        ph_acc[23] += __builtin_amdgcn_s_memrealtime() - rt0_;                                      \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) {                                         \
            if (threadIdx.x == 0) g_blk[blockIdx.x][0] = rt0_;                                      \
            atomicMax(&g_blk[blockIdx.x][1], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
        }                                                                                           \
        if ((threadIdx.x & 63) == 0)                                                                \
            _Pragma("unroll") for (int q_ = 0; q_ < 24; ++q_)                                       \
                if (ph_acc[q_]) atomicAdd(&g_phase[(blockIdx.x & 63) * 32 + q_], ph_acc[q_]);       \
    } while (0)
#else
#define PHASE_FLUSH() \
    do {              \
    } while (0)
#define PHASE(n) \
    do {         \
    } while (0)
#define PHASE_COUNT(n, v) \
    do {                  \
    } while (0)
#endif

// ---------------------------------------------------------------------------------------------------------------
// small helpers

// Correctly-rounded sqrt. NOTE: HIP's __fsqrt_rn is ocml's *native* (1-ulp) sqrt unless OCML_BASIC_ROUNDED_OPERATIONS
// is defined; __builtin_sqrtf lowers to v_sqrt_f32 + the two-FMA correction (IEEE round-to-nearest), like torch.sqrt.
__device__ __forceinline__ float sqrt_rn(float x) { return __builtin_sqrtf(x); }

__device__ __forceinline__ float clamp_t(float x, float lo, float hi) {  // torch.clamp: NaN propagates
    x = (x < lo) ? lo : x;
    return (x > hi) ? hi : x;
}

__device__ __forceinline__ float nan_to_num(float x) {  // torch.nan_to_num defaults
    if (__builtin_isnan(x)) return 0.0f;
    if (__builtin_isinf(x)) return x > 0.0f ? 3.402823466e+38f : -3.402823466e+38f;
    return x;
}

// check_boundary, gym_flock_v2.py:271-304 (non-rigid: teleport to 0.001 / box, not a modulo)
__device__ __forceinline__ float boundary(float v, float box, int rigid) {
    if (rigid) {
        v = (v < box) ? v : box;
        return (v > 0.0f) ? v : 0.0f;
    }
    v = (v < box) ? v : 0.001f;
    return (v > 0.0f) ? v : box;
}

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// d2 with the reference op order: periodic gym_flock_v2.py:140-144 (|d|, B-|d| if |d| > B/2, mul, mul, add).
// min(|d|, B-|d|) == where(|d| > B/2, B-|d|, |d|) bit for bit: B-|d| is exact for |d| >= B/2 (Sterbenz) and
// rounds to >= B/2 otherwise.
template <bool PERIODIC>
__device__ __forceinline__ float pair_d2(float xi, float yi, float xj, float yj, float box) {
    float dx = __fsub_rn(xi, xj);
    float dy = __fsub_rn(yi, yj);
    if (PERIODIC) {
        const float ax = fabsf(dx), ay = fabsf(dy);
        dx = fminf(ax, __fsub_rn(box, ax));
        dy = fminf(ay, __fsub_rn(box, ay));
    }
    return __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
}

// max over the 64 lanes (every lane active), as a wave-uniform scalar: DPP max within each row of 16 (quad_perm
// [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then the four row results by readlane. No LDS round trips.
template <int CTRL>
__device__ __forceinline__ int dpp_max(int v) {
    return max(v, __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ int wave_max(int v) {
    v = dpp_max<0xB1>(v);
    v = dpp_max<0x4E>(v);
    v = dpp_max<0x141>(v);
    v = dpp_max<0x140>(v);
    return __builtin_amdgcn_readfirstlane(max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
                                              max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48))));
}

// unsigned min over the 64 lanes (every lane active), wave-uniform: the same DPP pattern as wave_max
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_minu(uint32_t v) {
    return min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = dpp_minu<0xB1>(v);
    v = dpp_minu<0x4E>(v);
    v = dpp_minu<0x141>(v);
    v = dpp_minu<0x140>(v);
    const uint32_t a = min((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16));
    const uint32_t b = min((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48));
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)min(a, b));
}

// inclusive prefix sum over the 64 lanes (every lane active): DPP row_shr 1/2/4/8 within rows of 16, then
// row_bcast 15 / 31 across rows (lanes without a source read the 0 of `old`)
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}

// replay-ring stores of the fused insert: non-temporal (the rows are read back only by the learner's minibatch
// gathers, long after the XCD's L2 has turned over). Same-box A/B at config 3 (`profiles/r03/ntring/`): env kernel
// alone 42.5-43.8 -> 39.2-42.1 us against plain stores; write-through stores and non-temporal stores for the other
// output streams too were slower (44.9-45.2 us)
template <typename T>
__device__ __forceinline__ void st_ring(T* p, T v) {
    __builtin_nontemporal_store(v, p);
}

// pair_d2 of two candidates at once: the squares and sums as packed f32 ops (v_pk_mul / v_pk_add, one candidate
// per half; each half rounds exactly like the scalar mul, mul, add), so both packed issue slots do useful work.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Accessors of the step kernel's per-agent streams (state in, state / observation / replay record out): plain
// accesses. Measured and dropped (round 1-3 A/B builds): non-temporal loads and stores of every stream (env kernel
// 51.4 -> 52.2 us, the co-running update slower), non-temporal input loads only (43.9-45.2 against 38.2-39.5 us),
// non-temporal or write-through output stores (44.9-45.2 us): these streams are the next step's inputs.
template <typename T>
__device__ __forceinline__ T ldnt(const T* p) {
    return *p;
}
template <typename T>
__device__ __forceinline__ void stnt(T* p, T v) {
    *p = v;
}
// inputs read once and never written back by the step (the action, the previous observation row of the fused insert)
template <typename T>
__device__ __forceinline__ T ld_once(const T* p) {
    return *p;
}
// The same streams with a compile-time cache policy: non-temporal in the instantiation whose launches have more env
// blocks than are resident and whose state does not fit the MALL (config 5, PFM 3: 1.5 GB of state per step), so
// that the lines the L2 pull-ahead brings in for the next block generation are not evicted by this generation's
// streams (step_kernel's kNtIn / kNtOut)
template <bool NT, typename T>
__device__ __forceinline__ void st_o(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}
template <bool NT, typename T>
__device__ __forceinline__ T ld_i(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}

template <bool PERIODIC>
__device__ __forceinline__ f32x2 pair_d2x2(float xi, float yi, float x0, float y0, float x1, float y1, float box) {
    float dx0 = __fsub_rn(xi, x0), dx1 = __fsub_rn(xi, x1);
    float dy0 = __fsub_rn(yi, y0), dy1 = __fsub_rn(yi, y1);
    if (PERIODIC) {
        const float ax0 = fabsf(dx0), ax1 = fabsf(dx1), ay0 = fabsf(dy0), ay1 = fabsf(dy1);
        dx0 = fminf(ax0, __fsub_rn(box, ax0));
        dx1 = fminf(ax1, __fsub_rn(box, ax1));
        dy0 = fminf(ay0, __fsub_rn(box, ay0));
        dy1 = fminf(ay1, __fsub_rn(box, ay1));
    }
    const f32x2 dx = {dx0, dx1}, dy = {dy0, dy1};
    return dx * dx + dy * dy;
}

// Philox4x32-10 (Salmon et al. 2011), counter-based: (key = seed, counter = (c0, c1, c2, c3)).
struct U4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ U4 philox(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
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
    return {c0, c1, c2, c3};
}
__device__ __forceinline__ float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }  // [0,1)

// ---------------------------------------------------------------------------------------------------------------
// phase 3/4: kNN of one agent against its env's LDS-resident positions.
// Output: bd[0..W) / bj[0..W) = the W = L-1 smallest (d2, j) in ascending order (slots beyond N: +inf / INT_MAX).

template <int L>
__device__ __forceinline__ void key_insert(uint32_t (&key)[L], uint32_t kx) {
    uint32_t nk[L];
    nk[0] = min(key[0], kx);
#pragma unroll
    for (int s = 1; s < L; ++s) nk[s] = med3u(key[s - 1], kx, key[s]);
#pragma unroll
    for (int s = 0; s < L; ++s) key[s] = nk[s];
}

// phase 3: all N candidates (broadcast ds_read_b128, two per read)
template <int L, bool PERIODIC>
__device__ __forceinline__ void scan_all(uint32_t (&key)[L], const float2* __restrict__ cand, int N, int ib, float xi,
                                         float yi, float box) {
    const uint32_t hi_mask = ~((1u << ib) - 1u);
#pragma unroll
    for (int s = 0; s < L; ++s) key[s] = kEmpty;
    const float4* cand4 = reinterpret_cast<const float4*>(cand);
    int j = 0;
    // 8 candidates per trip, their 4 LDS reads issued together: small-N steps run one wave per SIMD, where a
    // read per candidate pair leaves the LDS latency exposed on every pair
#pragma unroll 1
    for (; j + 7 < N; j += 8) {
        float4 c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = cand4[(j >> 1) + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const f32x2 d = pair_d2x2<PERIODIC>(xi, yi, c[u].x, c[u].y, c[u].z, c[u].w, box);
            key_insert<L>(key, (__float_as_uint(d.x) & hi_mask) | (uint32_t)(j + 2 * u));
            key_insert<L>(key, (__float_as_uint(d.y) & hi_mask) | (uint32_t)(j + 2 * u + 1));
        }
    }
#pragma unroll 1
    for (; j + 1 < N; j += 2) {
        const float4 c = cand4[j >> 1];  // broadcast: every lane of the env reads the same 16 B
        const f32x2 d = pair_d2x2<PERIODIC>(xi, yi, c.x, c.y, c.z, c.w, box);
        key_insert<L>(key, (__float_as_uint(d.x) & hi_mask) | (uint32_t)j);
        key_insert<L>(key, (__float_as_uint(d.y) & hi_mask) | (uint32_t)(j + 1));
    }
    if (j < N) {
        const float2 c = cand[j];
        key_insert<L>(key, (__float_as_uint(pair_d2<PERIODIC>(xi, yi, c.x, c.y, box)) & hi_mask) | (uint32_t)j);
    }
}

// phase 3 over candidates [j0, j1) only (j0 even): one quarter of a split scan (step_kernel SPL > 1)
template <int L, bool PERIODIC>
__device__ __forceinline__ void scan_range(uint32_t (&key)[L], const float2* __restrict__ cand, int j0, int j1, int ib,
                                           float xi, float yi, float box) {
    const uint32_t hi_mask = ~((1u << ib) - 1u);
#pragma unroll
    for (int s = 0; s < L; ++s) key[s] = kEmpty;
    const float4* cand4 = reinterpret_cast<const float4*>(cand);
    int j = j0;
#pragma unroll 1
    for (; j + 7 < j1; j += 8) {
        float4 c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = cand4[(j >> 1) + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const f32x2 d = pair_d2x2<PERIODIC>(xi, yi, c[u].x, c[u].y, c[u].z, c[u].w, box);
            key_insert<L>(key, (__float_as_uint(d.x) & hi_mask) | (uint32_t)(j + 2 * u));
            key_insert<L>(key, (__float_as_uint(d.y) & hi_mask) | (uint32_t)(j + 2 * u + 1));
        }
    }
#pragma unroll 1
    for (; j < j1; ++j) {
        const float2 c = cand[j];
        key_insert<L>(key, (__float_as_uint(pair_d2<PERIODIC>(xi, yi, c.x, c.y, box)) & hi_mask) | (uint32_t)j);
    }
}

// Cell-list scans (step variants, N >= 128). The env's agents are binned into a Gx x Gy grid of cells about as
// tall as twice the typical (k+1)-th neighbour distance and about one agent per cell (Gy = max(kRows, 0.38 sqrt N),
// Gx = max(2 kRg + 4, N / Gy)), and stored cell-sorted, row by row, in an extended array ext of (x, y, j, sx): every
// cell row also carries ghost copies of its last kRg columns (in front) and its first kRg columns (behind) when the
// box is periodic, so any run of up to 2 kRg + 1 columns of a row is ONE contiguous range. sx = box for a ghost
// copy, else 0.
constexpr int kRg = 8;    // ghost columns per side of a row
constexpr int kRows = 3;  // rows of a seeded scan (its radius is at most one row height)
// EVR (step_kernel's even-row layout, per instantiation): every virtual row of ext ends with a one-entry sentinel
// cell (+inf position), so that the seeded scan may read one entry past any row range without reaching the next row,
// and pads every row range to an even length: a slot pair then never straddles two rows (scan_seeded)
// virtual cells per row of the prefix: front ghosts, the gx columns, back ghosts (and the row sentinel)
__host__ __device__ constexpr int row_stride(int gx, bool evr) { return gx + 2 * kRg + (evr ? 1 : 0); }
// ext capacity per env: N entries, at most N ghost copies, two trailing sentinels (and the row sentinels)
__host__ __device__ constexpr int ext_cap(int n, int gy, bool evr) { return 2 * n + 2 + (evr ? gy : 0); }

// d2 of two candidates, bit-identical to the reference's periodic / Euclidean d2 in op order (gym_flock_v2.py:140-144,
// :160-165). x: with Gx >= 2 kRg + 4 and every scanned cell at most kRg(+1) columns from the lane's cell, a regular
// entry has |dx| < B/2 (the reference keeps |dx|, and (0 - |dx|)^2 == dx^2 bit for bit) and a ghost entry (sx = B)
// has |dx| > B/2 (the reference takes B - |dx|), so min(|dx|, B - |dx|) is one subtraction with an |.| modifier.
// y: the reference formula (rows wrap by index).
template <bool PERIODIC>
__device__ __forceinline__ f32x2 cand_d2x2(float xi, float yi, float box, const float4& q0, const float4& q1) {
    const float dx0 = __fsub_rn(q0.w, fabsf(__fsub_rn(xi, q0.x))), dx1 = __fsub_rn(q1.w, fabsf(__fsub_rn(xi, q1.x)));
    float dy0 = __fsub_rn(yi, q0.y), dy1 = __fsub_rn(yi, q1.y);
    if (PERIODIC) {
        const float a0 = fabsf(dy0), a1 = fabsf(dy1);
        dy0 = fminf(a0, __fsub_rn(box, a0));
        dy1 = fminf(a1, __fsub_rn(box, a1));
    }
    const f32x2 dx = {dx0, dx1}, dy = {dy0, dy1};
    return dx * dx + dy * dy;
}

__device__ __forceinline__ int wrap_row(int yy, int G) { return yy < 0 ? yy + G : (yy >= G ? yy - G : yy); }

// Seeded scan, flattened. The caller guarantees that the disk of radius r around the lane's agent holds k+1
// distinct agents (the lane itself and its previous neighbours) and that r exceeds their largest distance by a factor
// that moves it >= 16 truncated-d2 buckets up, so every agent outside the disk has a larger key than the (k+1)-th
// smallest and every agent sharing that key's bucket is inside: the top k+1 keys (and the ambiguity test of
// knn_finalize) are exactly the full scan's. The lane's candidates are the cells under the disk, row by row (at most
// kRows rows, r <= one row height; per row the columns under the disk's chord, one contiguous range of ext), taken
// as ONE sequence: candidate t of the lane is ext[t + b_q] for the row q with P_q <= t < P_{q+1} (P = running row
// totals). The wave runs max-over-lanes(total) slots, two per iteration, with the slot index t wave-uniform.
// Call with every lane of the wave active; lanes with use = false scan nothing.
template <int L, bool PERIODIC, bool EVR>
__device__ __forceinline__ void scan_seeded(uint32_t (&key)[L], const float4* __restrict__ ext,
                                            const int* __restrict__ pre, int gx, int gy, int cy, bool use, float r,
                                            int ib, float xi, float yi, float box, float cwy, float inv_cwx,
                                            float inv_cwy, int cmax) {
    const uint32_t hi_mask = ~((1u << ib) - 1u);
    const int W2 = row_stride(gx, EVR);
#pragma unroll
    for (int s = 0; s < L; ++s) key[s] = kEmpty;
    int b[kRows], P[kRows];  // P[u]: candidates before row slot u; b[u]: ext index of candidate t in slot u minus t
    int tot = 0;
    int qlo = 1, qhi = 0;
    if (use) {
        qlo = (int)floorf((yi - r) * inv_cwy) - cy;
        qhi = (int)floorf((yi + r) * inv_cwy) - cy;
        if (!PERIODIC) {
            qlo = max(qlo, -cy);
            qhi = min(qhi, gy - 1 - cy);
        }
    }
    const float r2 = r * r;
#pragma unroll
    for (int u = 0; u < kRows; ++u) {
        const int q = qlo + u;
        P[u] = tot;
        b[u] = cmax;  // an unused (trailing) row: its slots land on the sentinel, never on entries scanned before
        if (q <= qhi) {
            const int yy = cy + q;
            const float ylo = (float)yy * cwy;
            const float dy = fmaxf(fmaxf(ylo - yi, yi - (ylo + cwy)), 0.0f);
            if (dy <= r) {
                // chord half-width, rounded up (raw v_sqrt_f32 is within 1 ulp; the r * 2^-10 term covers the
                // rounding of r2 - dy^2 near a grazing row and of the cell assignment)
                const float hw = __builtin_amdgcn_sqrtf(fmaxf(r2 - dy * dy, 0.0f)) * 1.000001f + r * 0.0009765625f;
                const int xa = max((int)floorf((xi - hw) * inv_cwx), -kRg);
                const int xb = min((int)floorf((xi + hw) * inv_cwx), gx + kRg - 1);
                const int* pr = pre + (PERIODIC ? wrap_row(yy, gy) : yy) * W2;
                const int s0 = pr[xa + kRg], e0 = pr[xb + kRg + 1];
                b[u] = s0 - tot;
                tot += EVR ? (e0 - s0 + 1) & ~1 : e0 - s0;  // EVR: the padded slot reads the entry after the range
            }
        }
    }
    const int slots = wave_max(tot);
    const int b0 = b[0], b1 = b[1], b2 = b[2], P1 = P[1], P2 = P[2];  // (EVR)
#ifdef FLOCK_PHASE_PROF
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&g_phase[(blockIdx.x & 63) * 32 + 21], (unsigned long long)((slots + 1) / 2));
        atomicAdd(&g_phase[(blockIdx.x & 63) * 32 + 22], 1ull);
    }
#endif
    // Slots past the lane's total are not masked. With a trailing unused row they land on the +inf sentinel at cmax
    // (the entry count); after a lane's third row they read the entries that follow its last range (agents of the
    // env outside its disk and never scanned before, whose computed d2 is at least their true periodic d2, so their
    // keys lie above the (k+1)-th and its bucket: the top k+1 and the ambiguity test are unchanged).
    auto cand_index = [&](int tt, int& c0, int& c1) {
        c0 = tt + b[0];
        c1 = tt + 1 + b[0];
#pragma unroll
        for (int u = 1; u < kRows; ++u) {
            c0 = (tt >= P[u]) ? tt + b[u] : c0;
            c1 = (tt + 1 >= P[u]) ? tt + 1 + b[u] : c1;
        }
        c0 = min(c0, cmax);
        c1 = min(c1, cmax);
    };
#pragma unroll 1
    for (int t = 0; t < slots; t += 2) {
        int c0, c1;
        float4 q0, q1;
        if constexpr (EVR) {
            static_assert(kRows == 3, "the even-row slot map is written for three rows");
            c0 = min(t + (t >= P2 ? b2 : (t >= P1 ? b1 : b0)), cmax);
            c1 = c0 + 1;  // same row (even row totals), or the second sentinel at cmax + 1
            q0 = ext[c0];
            q1 = ext[c0 + 1];
        } else {
            cand_index(t, c0, c1);
            q0 = ext[c0];
            q1 = ext[c1];
        }
        const f32x2 d = cand_d2x2<PERIODIC>(xi, yi, box, q0, q1);
        key_insert<L>(key, (__float_as_uint(d.x) & hi_mask) | (uint32_t)__float_as_int(q0.z));
        key_insert<L>(key, (__float_as_uint(d.y) & hi_mask) | (uint32_t)__float_as_int(q1.z));
    }
}

// Square scan with proof (lanes without usable seeds): rows cy-Ry..cy+Ry, columns cx-kRg..cx+kRg, one row range at
// a time (tmax = the wave-wide maximum of the row's range lengths); returns true when the top-L keys are provably
// those of the full scan: every agent outside the block lies at least m = the distance to the block's edge away, so
// if the truncated-d2 bucket of m^2 (shrunk by a 1e-5 safety factor) exceeds the L-th key, no unscanned key can enter
// the top L. Call with every lane of the wave active (lanes with live = false scan nothing and return true).
template <int L, bool PERIODIC, bool EVR>
__device__ __forceinline__ bool scan_square(uint32_t (&key)[L], const float4* __restrict__ ext,
                                            const int* __restrict__ pre, int gx, int gy, int cx, int cy, int Ry,
                                            int ib, float xi, float yi, float box, float cwx, float cwy, float eps,
                                            int cmax, bool live) {
    const uint32_t hi_mask = ~((1u << ib) - 1u);
    const int W2 = row_stride(gx, EVR);
#pragma unroll
    for (int s = 0; s < L; ++s) key[s] = kEmpty;
#pragma unroll 1
    for (int rr = -Ry; rr <= Ry; ++rr) {
        int yr = cy + rr;
        bool row = live;
        if (PERIODIC)
            yr = wrap_row(yr, gy);
        else
            row = row && yr >= 0 && yr < gy;
        const int* pr = pre + (row ? yr : 0) * W2;
        const int s0 = row ? pr[cx] : 0, e0 = row ? pr[cx + 2 * kRg + 1] : 0;
        const int tmax = wave_max(e0 - s0);
#pragma unroll 1
        for (int t = 0; t < tmax; t += 2) {
            const int c = s0 + t;
            const float4 q0 = ext[min(c, cmax)], q1 = ext[min(c + 1, cmax)];
            const f32x2 d = cand_d2x2<PERIODIC>(xi, yi, box, q0, q1);
            const uint32_t k0 = (__float_as_uint(d.x) & hi_mask) | (uint32_t)__float_as_int(q0.z);
            const uint32_t k1 = (__float_as_uint(d.y) & hi_mask) | (uint32_t)__float_as_int(q1.z);
            key_insert<L>(key, c < e0 ? k0 : kEmpty);
            key_insert<L>(key, c + 1 < e0 ? k1 : kEmpty);
        }
    }
    // every agent outside the scanned block is at least m away; without wrap, a side of the block that reaches the
    // box edge has no agents beyond it
    const float inf = __builtin_inff();
    const float lx = (float)(cx - kRg) * cwx, rx = (float)(cx + kRg + 1) * cwx;
    const float ly = (float)(cy - Ry) * cwy, ry = (float)(cy + Ry + 1) * cwy;
    const float ml = (!PERIODIC && cx - kRg <= 0) ? inf : xi - lx, mr = (!PERIODIC && cx + kRg >= gx - 1) ? inf : rx - xi;
    const float mb = (!PERIODIC && cy - Ry <= 0) ? inf : yi - ly, mt = (!PERIODIC && cy + Ry >= gy - 1) ? inf : ry - yi;
    const float m = fminf(fminf(ml, mr), fminf(mb, mt)) - eps;
    const float bound = m > 0.0f ? fminf((m * m) * 0.99998f, 3.0e38f) : 0.0f;
    return !live || (__float_as_uint(bound) & hi_mask) > key[L - 1];
}

// exact ordered insertion of (d2, j) into the W best, lexicographic (any visiting order)
template <int W>
__device__ __forceinline__ void insert_exact(float (&bd)[W], int (&bj)[W], float d, int j) {
    if (d < bd[W - 1] || (d == bd[W - 1] && j < bj[W - 1])) {
        bool lt[W];
#pragma unroll
        for (int s = 0; s < W; ++s) lt[s] = d < bd[s] || (d == bd[s] && j < bj[s]);
#pragma unroll
        for (int s = W - 1; s >= 1; --s) {
            bd[s] = lt[s - 1] ? bd[s - 1] : (lt[s] ? d : bd[s]);
            bj[s] = lt[s - 1] ? bj[s - 1] : (lt[s] ? j : bj[s]);
        }
        bd[0] = lt[0] ? d : bd[0];
        bj[0] = lt[0] ? j : bj[0];
    }
}

// exact rescan of an ambiguous bucket over the scanned neighbourhood only (rows cy-Ry..cy+Ry, columns cx-kRg..cx+kRg,
// which contains a seeded lane's disk and a square lane's proved block): every unscanned d2 exceeds every d2 of the
// ambiguous bucket, so the exact top k+1 by (d2, j) lies in the scanned ranges (per-lane loops: no wave-wide ops)
template <int L, bool PERIODIC, bool EVR>
__device__ __forceinline__ void exact_rescan_cells(float (&bd)[L - 1], int (&bj)[L - 1],
                                                   const float4* __restrict__ ext, const int* __restrict__ pre,
                                                   int gx, int gy, int cx, int cy, int Ry, float xi, float yi,
                                                   float box) {
    constexpr int W = L - 1;
    const int W2 = row_stride(gx, EVR);
#pragma unroll
    for (int s = 0; s < W; ++s) {
        bd[s] = __builtin_inff();
        bj[s] = 0x7fffffff;
    }
    for (int r = -Ry; r <= Ry; ++r) {
        int yr = cy + r;
        if (PERIODIC)
            yr = wrap_row(yr, gy);
        else if (yr < 0 || yr >= gy)
            continue;
        const int* pr = pre + yr * W2;
        for (int c = pr[cx]; c < pr[cx + 2 * kRg + 1]; ++c) {
            const float4 q = ext[c];
            insert_exact<W>(bd, bj, pair_d2<PERIODIC>(xi, yi, q.x, q.y, box), __float_as_int(q.z));
        }
    }
}

// The same exact rescan with the whole wave (call with every lane of the wave active; `amb` marks the lanes that need
// it). An ambiguous lane is rare (~5e-5 of the lanes at config 3), but its serial rescan (~50 dependent LDS reads and
// branchy insertions over rows cy-1..cy+1, columns cx-kRg..cx+kRg) held its block ~2x as long and set the launch's
// tail (timing build without rescans: 49 -> 43 us). Here the 64 lanes take one candidate each of the ambiguous
// lane's neighbourhood per pass and the exact (d2, j) order comes from W rounds of wave-wide minima (d2 bits, then
// j among the lanes holding that d2): the same (d2, j) set, hence the same result, as exact_rescan_cells.
// R = 0 lanes (no cell list, or a cell lane that fell back to the full scan) rescan all N agents of their env from
// lpos the same way (knn_finalize's serial full rescan: the config-2 kernel's straggler blocks).
template <int L, bool PERIODIC, bool CELL, bool EVR>
__device__ __forceinline__ void exact_rescan_wave(float (&bd)[L - 1], int (&bj)[L - 1], bool amb, int R,
                                                  const float2* __restrict__ lpos, int S, int N,
                                                  const float4* __restrict__ ext_all, const int* __restrict__ pre_all,
                                                  int ecap, int npre, int g, int gx, int gy, int cx, int cy, float xi,
                                                  float yi, float box) {
    constexpr int W = L - 1;
    const int W2 = row_stride(gx, EVR);
    const int lane = __lane_id();
    uint64_t todo = __ballot(amb);
    while (todo) {
        const int src = __ffsll((long long)todo) - 1;
        todo &= todo - 1;
        const float sx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xi), src));
        const float sy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yi), src));
        const int sg = __builtin_amdgcn_readlane(g, src);  // lanes past the env (G = 1, N < 256) carry g = 1
        const bool cells = CELL && __builtin_amdgcn_readlane(R, src) == 1;
        const float2* cand = lpos + sg * S;
        const float4* ext = ext_all + sg * ecap;
        int rs[3] = {0, 0, 0}, rn[3] = {N, 0, 0};  // ext row ranges (cell lanes), else all N of lpos
        if (cells) {
            const int scx = __builtin_amdgcn_readlane(cx, src), scy = __builtin_amdgcn_readlane(cy, src);
            const int* pre = pre_all + sg * npre;
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                int yr = scy + u - 1;
                bool row = true;
                if (PERIODIC)
                    yr = wrap_row(yr, gy);
                else
                    row = yr >= 0 && yr < gy;
                const int* pr = pre + (row ? yr : 0) * W2;
                rs[u] = row ? pr[scx] : 0;
                rn[u] = row ? pr[scx + 2 * kRg + 1] - rs[u] : 0;
            }
        }
        const int n01 = rn[0] + rn[1], total = n01 + rn[2];
        float ud[W];
        int uj[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            ud[w] = __builtin_inff();
            uj[w] = 0x7fffffff;
        }
        for (int base = 0; base < total; base += 64) {
            const int tt = base + lane;
            uint32_t kd = 0xFFFFFFFFu, kj = 0xFFFFFFFFu;  // d2 >= 0: its bits order like the floats (inf < ~0u)
            if (tt < total) {
                if (cells) {
                    const int c = tt < rn[0] ? rs[0] + tt : (tt < n01 ? rs[1] + tt - rn[0] : rs[2] + tt - n01);
                    const float4 q = ext[c];
                    kd = __float_as_uint(pair_d2<PERIODIC>(sx, sy, q.x, q.y, box));
                    kj = (uint32_t)__float_as_int(q.z);
                } else {
                    const float2 q = cand[tt];
                    kd = __float_as_uint(pair_d2<PERIODIC>(sx, sy, q.x, q.y, box));
                    kj = (uint32_t)tt;
                }
            }
#pragma unroll 1
            for (int w = 0; w < W; ++w) {
                const uint32_t md = wave_min_u32(kd);
                if (md == 0xFFFFFFFFu) break;
                const uint32_t mj = wave_min_u32(kd == md ? kj : 0xFFFFFFFFu);
                const float d = __uint_as_float(md);
                if (!(d < ud[W - 1] || (d == ud[W - 1] && (int)mj < uj[W - 1]))) break;  // the rest cannot enter
                insert_exact<W>(ud, uj, d, (int)mj);
                if (kd == md && kj == mj) kd = kj = 0xFFFFFFFFu;  // taken (one lane: (d2, j) pairs are distinct)
            }
        }
        if (lane == src) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                bd[w] = ud[w];
                bj[w] = uj[w];
            }
        }
    }
}

// phase 4: exact (d2, j) order of the W best keys, or (ambiguous (k+1)/(k+2) bucket) an exact rescan of all N
// candidates when full_rescan, else return true and let the caller rescan its neighbourhood
template <int L, bool PERIODIC>
__device__ __forceinline__ bool knn_finalize(const uint32_t (&key)[L], const float2* __restrict__ cand, int N, int k,
                                             int ib, float xi, float yi, float box, float (&bd)[L - 1],
                                             int (&bj)[L - 1], bool full_rescan = true) {
    constexpr int W = L - 1;
    const uint32_t lo_mask = (1u << ib) - 1u, hi_mask = ~lo_mask;
    // (k+1)-th and (k+2)-th smallest keys (k is a runtime value <= L-2; static-index select, no scratch)
    uint32_t kk = kEmpty, kr = kEmpty;
#pragma unroll
    for (int s = 0; s < L; ++s) {
        if (s == k) kk = key[s];
        if (s == k + 1) kr = key[s];
    }
    const bool ambiguous = (kr != kEmpty) && ((kr & hi_mask) == (kk & hi_mask));

    if (!ambiguous) {
        // exact (d2, j) for the W best keys; keys of different truncated buckets are already in exact d2 order, so
        // the odd-even transposition sort (only same-bucket keys move) runs only when two adjacent keys share one
        bool same = false;
#pragma unroll
        for (int s = 0; s + 1 < W; ++s) same |= (key[s] & hi_mask) == (key[s + 1] & hi_mask);
#pragma unroll
        for (int s = 0; s < W; ++s) {
            if (key[s] == kEmpty) {
                bd[s] = __builtin_inff();
                bj[s] = 0x7fffffff;
            } else {
                const int jj = (int)(key[s] & lo_mask);
                const float2 c = cand[jj];
                bd[s] = pair_d2<PERIODIC>(xi, yi, c.x, c.y, box);
                bj[s] = jj;
            }
        }
        if (same) {
#pragma unroll
        for (int pass = 0; pass < W; ++pass) {
#pragma unroll
            for (int s = (pass & 1); s + 1 < W; s += 2) {
                const bool sw = (bd[s + 1] < bd[s]) || (bd[s + 1] == bd[s] && bj[s + 1] < bj[s]);
                const float td = sw ? bd[s + 1] : bd[s];
                const int tj = sw ? bj[s + 1] : bj[s];
                bd[s + 1] = sw ? bd[s] : bd[s + 1];
                bj[s + 1] = sw ? bj[s] : bj[s + 1];
                bd[s] = td;
                bj[s] = tj;
            }
        }
        }
    } else if (full_rescan) {
        // exact rescan: branch-free ordered insertion of (d2, j); ascending j + strict '<' keeps lower j first
#pragma unroll
        for (int s = 0; s < W; ++s) {
            bd[s] = __builtin_inff();
            bj[s] = 0x7fffffff;
        }
        for (int jj = 0; jj < N; ++jj) {
            const float2 c = cand[jj];
            const float d = pair_d2<PERIODIC>(xi, yi, c.x, c.y, box);
            if (d < bd[W - 1]) {
                bool lt[W];
#pragma unroll
                for (int s = 0; s < W; ++s) lt[s] = d < bd[s];
#pragma unroll
                for (int s = W - 1; s >= 1; --s) {
                    bd[s] = lt[s - 1] ? bd[s - 1] : (lt[s] ? d : bd[s]);
                    bj[s] = lt[s - 1] ? bj[s - 1] : (lt[s] ? jj : bj[s]);
                }
                bd[0] = lt[0] ? d : bd[0];
                bj[0] = lt[0] ? jj : bj[0];
            }
        }
    } else {
        return true;
    }
    return false;
}

template <int L, bool PERIODIC>
__device__ __forceinline__ void knn_scan(const float2* __restrict__ cand, int N, int k, int ib, float xi, float yi,
                                         float box, float (&bd)[L - 1], int (&bj)[L - 1]) {
    uint32_t key[L];
    scan_all<L, PERIODIC>(key, cand, N, ib, xi, yi, box);
    knn_finalize<L, PERIODIC>(key, cand, N, k, ib, xi, yi, box, bd, bj);
}

// fused replay insert with one terminal flag per env row (FlockRing.env_done): the env's any_done at its ring row
__device__ __forceinline__ void env_done_row(const Params& p, int env, int flag) {
    if (p.r_state && p.r_env_done && env >= p.r_skip) {
        int64_t row = p.r_start + env - p.r_skip;
        if (row >= p.r_cap) row -= p.r_cap;
        p.r_term[row] = (flag != 0) == (p.r_done != 0) ? 1.0f : 0.0f;
    }
}

// ---------------------------------------------------------------------------------------------------------------
// the fused step kernel

constexpr int clog2c(int n) {
    int b = 0;
    while ((1 << b) < n) ++b;
    return b;
}

// VAR >= 0, NC > 0: an instantiation specialised on the variant, N (k = L - 2) and the cell grid (GXC x GYC) of one
// hot configuration. The launch's Params copy gets those fields as compile-time constants, so the variant branches,
// the env/lane split (t / N), the LDS carve-up and every trip count that depends on them fold away (fewer SGPRs
// live across the kernel). Same code, same results as the generic instantiation.
// SPL > 1 (small N without cells, SPL * N threads per block): one env per block, SPL waves-worth of lanes per env.
// The first N lanes are the env's agents for every phase; the candidate scan alone is split: lane group q scans
// candidates [q N / SPL, (q + 1) N / SPL) for agent (t mod N), and the agents' lanes merge the SPL partial top-L
// key lists through LDS (the same key set, hence the same result, as the one-lane scan). At N = 64 this gives 4x the
// waves of one lane per agent, where one wave per SIMD left every latency exposed.
template <int L, bool PERIODIC, bool CELL, int VAR = -1, int NC = 0, int GXC = 0, int GYC = 0, int SPL = 1, int PFM = 0,
          bool EVR = false>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void step_kernel(const Params pin) {
    static_assert(SPL == 1 || (NC > 0 && !CELL && (NC % (2 * SPL)) == 0), "split scans: specialised N, no cells");
    Params p = pin;
    if (VAR >= 0) p.variant = VAR;
    // config 5 (PFM 3): non-temporal state streams and the pull-ahead issued after the binning (kPullAt 1), so that
    // the pulled lines spend less time in an L2 this generation's streams are turning over. Same-box A/B
    // (profiles/r05/c5pull/): env launch 0.639 -> 0.590 ms, PMC reads 88.7 -> 58.6 B per agent-step; the pull after
    // the kinematics (0, kept for PFM 1), before the binning, after the scans or before the outputs, and either policy
    // alone, measured between the two
    constexpr bool kNtOut = PFM == 3;
    constexpr bool kNtIn = PFM == 3;
    constexpr int kPullAt = PFM == 3 ? 1 : 0;
    if (NC > 0) {  // make_cfg / dispatch values for N = NC
        p.N = NC;
        p.k = L - 2;
        p.G = SPL > 1 ? 1 : (NC <= 256 ? 256 / NC : 1);
        p.S = (NC + 1) & ~1;
        p.P = 1 << clog2c(NC);
        p.ib = clog2c(NC) < 1 ? 1 : clog2c(NC);
        if (CELL) {
            p.gx = GXC;
            p.gy = GYC;
            p.ecap = ext_cap(NC, GYC, EVR);
        }
    }
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float2* lpos = reinterpret_cast<float2*>(smem);               // [G][S]
    float* red = reinterpret_cast<float*>(lpos + p.G * p.S);      // [G][2][P]
    int* flags = reinterpret_cast<int*>(red + 2 * p.G * p.P);     // [G] collision flags, [G] arrivals (G = 1)
    // cell list (CELL): ext [G][ecap] float4 (16-B aligned), cnt [G][gx*gy], pre [G][npre]: exclusive prefix over
    // the "virtual cells" of every row [ghosts of columns gx-kRg..gx-1, columns 0..gx-1, ghosts of columns 0..kRg-1]
    const int gx = p.gx, gy = p.gy, ncell = gx * gy, W2 = row_stride(gx, EVR), npre = gy * W2 + 1;
    float4* ext_all =
        reinterpret_cast<float4*>(smem + ((((size_t)(flags + 2 * p.G) - (size_t)smem) + 15) & ~(size_t)15));
    int* cnt_all = reinterpret_cast<int*>(ext_all + (CELL ? p.G * p.ecap : 0));
    int* pre_all = cnt_all + (CELL ? p.G * ncell : 0);
    int* wtot_all = pre_all + (CELL ? p.G * npre : 0);  // [G][16] per-wave totals of the binning scan

    const int variant = p.variant;
#ifdef FLOCK_PHASE_PROF
    unsigned long long ph_acc[24];
#pragma unroll
    for (int q_ = 0; q_ < 24; ++q_) ph_acc[q_] = 0;
    unsigned long long t_prev = __builtin_amdgcn_s_memtime();
    const unsigned long long st0_ = t_prev, rt0_ = __builtin_amdgcn_s_memrealtime();  // in-kernel clock
#endif
    const int t = threadIdx.x;
    const int g = t / p.N;
    const int i = t - g * p.N;
    const bool in_group = g < p.G;
    PHASE_COUNT(20, 1);
    const int env = p.env0 + blockIdx.x * p.G + g;
    const bool active = in_group && env < p.E;
    const size_t a = (size_t)env * p.N + i;
    if (in_group && i == 0) flags[g] = 0;
    if (t == 0) flags[p.G] = 0;  // arrival counter of the G = 1 any_done (published by the phase-2 barrier)
    if (CELL && in_group)  // published by the phase-2 barrier
        for (int c = i; c < ncell; c += p.N) cnt_all[g * ncell + c] = 0;

    // ---- phase 1: kinematics + boundary ------------------------------------------------------------------
    float x = 0.0f, y = 0.0f, h = 0.0f;
    float2 act_in = make_float2(0.0f, 0.0f);  // fused replay insert: the raw action (v2) or the f32 action id
    float prev_obs[L - 2];  // fused replay insert: the previous observation row, loaded early (latency hidden)
#pragma unroll
    for (int s = 0; s < L - 2; ++s) prev_obs[s] = 0.0f;
    // fused replay insert: ring unit (row) of this agent and its slot within the row (one row per agent, or one
    // row per env holding every agent's fields, group = N)
    const int64_t r_unit = p.r_group == 1 ? (int64_t)a : (int64_t)env;
    const int r_slot = p.r_group == 1 ? 0 : i;
    // cell path: previous neighbour indices (nn_idx on entry, a search hint only), loaded early and checked at use
    int64_t hint[L - 2];
    const bool has_hint = CELL && active && (p.seeds != nullptr || p.idx != nullptr);
#pragma unroll
    for (int s = 0; s < L - 2; ++s) hint[s] = -1;
    // k = 4 seeds: one 8-B load (a * k u16 is 8-B aligned), unpacked only at the seeded scan
    const bool seed_packed = has_hint && p.seeds && L - 2 == 4 && p.k == 4;
    uint2 seed_raw = make_uint2(0u, 0u);
    // the inputs needed only after phase 1 (seeds, the previous observation of the fused insert) are loaded after
    // the kinematics inputs, so that at kernel start, when every resident block loads at once, the loads the
    // kinematics waits on are not queued behind them
    auto load_late = [&]() {
        if (seed_packed) {
            const u32x2 sv = ld_i<kNtIn>(reinterpret_cast<const u32x2*>(p.seeds + a * p.k));
            seed_raw = make_uint2(sv.x, sv.y);
        } else if (has_hint && p.seeds) {
            const uint16_t* hp = p.seeds + a * p.k;
#pragma unroll
            for (int s = 0; s < L - 2; ++s)
                if (s < p.k) hint[s] = hp[s];
        } else if (has_hint) {
            const int64_t* hp = p.idx + a * p.k;
#pragma unroll
            for (int s = 0; s < L - 2; ++s)
                if (s < p.k) hint[s] = hp[s];
        }
        if (active && p.r_state && r_unit >= p.r_skip) {
            const float* po = p.r_prev + a * p.k;
            if (L - 2 == 4 && p.k == 4) {  // one 16-B load (rows of 4 floats are 16-B aligned)
                const f32x4 v = ld_i<kNtIn>(reinterpret_cast<const f32x4*>(po));
                prev_obs[0] = v.x;
                prev_obs[1 % (L - 2)] = v.y;
                prev_obs[2 % (L - 2)] = v.z;
                prev_obs[3 % (L - 2)] = v.w;
            } else {
#pragma unroll
                for (int s = 0; s < L - 2; ++s)
                    if (s < p.k) prev_obs[s] = po[s];
            }
        }
    };
    constexpr bool kLateAfter = true;  // the seeds / previous-obs loads after the kinematics loads (round 1)
    // small-N Euclidean kernels (uw / flock observation memory): the three frames the roll keeps, loaded now so
    // their latency hides behind the step (only in the !CELL, !PERIODIC instantiation: no register cost elsewhere)
    constexpr bool kMemEarly = !CELL && !PERIODIC;
    constexpr int kMemKeep = kMemEarly ? (kMem - 1) * (L - 2) : 1;
    float mrow[kMemKeep];
#pragma unroll
    for (int s = 0; s < kMemKeep; ++s) mrow[s] = 0.0f;
    float prev_h = 0.0f;  // uw reward: the previous heading (:202-204), loaded early
    if (active && variant == FLOCK_VARIANT_UW) prev_h = p.prev_heading[a];
    if constexpr (SPL > 1 && kMemEarly) {  // split instantiation: lane groups 1..SPL-1 roll memory frames 0..2 (k = 4)
        const int q = t / NC, ia = t - q * NC;
        const int envb = p.env0 + (int)blockIdx.x;
        if (q >= 1 && envb < p.E && (variant == FLOCK_VARIANT_UW || variant == FLOCK_VARIANT_FLOCK)) {
            const size_t ab = (size_t)envb * NC + ia;
#pragma unroll
            for (int f = q - 1; f < kMem - 1; f += SPL - 1)
                reinterpret_cast<float4*>(p.mem_out + ab * kMem * 4)[f + 1] =
                    reinterpret_cast<const float4*>(p.mem_in + ab * kMem * 4)[f];
        }
    }
    if (kMemEarly && SPL == 1 && active && (variant == FLOCK_VARIANT_UW || variant == FLOCK_VARIANT_FLOCK)) {
        const float* mi = p.mem_in + a * kMem * p.k;
        if (L - 2 == 4 && p.k == 4) {  // 3 x float4 (rows are 64-B aligned)
#pragma unroll
            for (int f = 0; f < kMem - 1; ++f) {
                const float4 v = reinterpret_cast<const float4*>(mi)[f];
                mrow[(f * (L - 2) + 0) % kMemKeep] = v.x;
                mrow[(f * (L - 2) + 1) % kMemKeep] = v.y;
                mrow[(f * (L - 2) + 2) % kMemKeep] = v.z;
                mrow[(f * (L - 2) + 3) % kMemKeep] = v.w;
            }
        } else {
#pragma unroll
            for (int f = 0; f < kMem - 1; ++f)
#pragma unroll
                for (int c = 0; c < L - 2; ++c)
                    if (c < p.k) mrow[(f * (L - 2) + c) % kMemKeep] = mi[f * p.k + c];
        }
    }
    if (active) {
        const f32x2 pp = ld_i<kNtIn>(reinterpret_cast<const f32x2*>(p.pos) + a);
        x = pp.x;
        y = pp.y;
        if (variant == FLOCK_VARIANT_V2) {  // gym_flock_v2.py:317-350 (heading=True)
            const f32x2 ac = ld_i<kNtIn>(reinterpret_cast<const f32x2*>(p.action) + a);
            act_in = make_float2(ac.x, ac.y);
            const float ang = clamp_t(ac.y, -kHalfPi, kHalfPi);             // :327
            h = __fadd_rn(ld_i<kNtIn>(p.heading + a), __fmul_rn(ang, p.dt));        // :329
#ifdef FLOCK_PHASE_PROF  // diagnostics: the kinematics inputs' arrival (phase 9) apart from the rest of phase 0
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(h), "v"(x) : "memory");
            PHASE(9);
#endif
            const float lin = clamp_t(ac.x, p.v_min, p.v_max);               // :331
            float sn, cs;
            sincosf(h, &sn, &cs);                                            // ocml: the sinf / cosf bits
            float vx = __fmul_rn(lin, cs);                                   // :335
            float vy = __fmul_rn(lin, sn);                                   // :336
            vx = __fmul_rn(nan_to_num(vx), p.dt);                            // :346, :349
            vy = __fmul_rn(nan_to_num(vy), p.dt);
            x = __fadd_rn(x, vx);                                            // :350
            y = __fadd_rn(y, vy);
            st_o<kNtOut>(p.heading + a, h);
            st_o<kNtOut>(reinterpret_cast<f32x2*>(p.vel) + a, f32x2{vx, vy});
        } else if (variant == FLOCK_VARIANT_UW) {  // gym_flock_uw.py:269-302 (heading=False)
            const float2 ac = reinterpret_cast<const float2*>(p.action)[a];
            const float n = sqrt_rn(__fadd_rn(__fmul_rn(ac.x, ac.x), __fmul_rn(ac.y, ac.y)));  // :294
            float vx = __fmul_rn(nan_to_num(__fdiv_rn(ac.x, n)), p.dt);     // :294-301
            float vy = __fmul_rn(nan_to_num(__fdiv_rn(ac.y, n)), p.dt);
            x = __fadd_rn(x, vx);                                            // :302
            y = __fadd_rn(y, vy);
            h = p.heading[a];
            reinterpret_cast<float2*>(p.vel)[a] = make_float2(vx, vy);
        } else if (variant == FLOCK_VARIANT_UW_DISCRETE) {  // gym_flock_uw_discrete.py:324-366
            int64_t id = p.action_id[a];
            act_in.x = (float)id;  // memory.put stores the action ids as floats (vdn/train_flock.py:99-102)
            if (id < 0 || id >= p.n_actions) {  // the reference raises KeyError (:329)
                if (p.status) atomicOr(p.status, 1);
                id = 0;
            }
            const float2 mean = reinterpret_cast<const float2*>(p.table)[id];
            float nl, na;
            if (p.noise) {
                const float2 nz = reinterpret_cast<const float2*>(p.noise)[a];
                nl = nz.x;
                na = nz.y;
            } else {  // torch.normal(mean, 0.1) (:333-334): Box-Muller on Philox uniforms
                const U4 r = philox(p.seed, (uint32_t)a, (uint32_t)(a >> 32), (uint32_t)p.rng_offset,
                                    (uint32_t)(p.rng_offset >> 32) ^ 0x5EEDu);
                const float u1 = fmaxf(u01(r.x), 1.0f / 16777216.0f), u2 = u01(r.y);
                // hardware transcendentals (v_log_f32 is log2; v_sin / v_cos_f32 take revolutions, u2 already is
                // one): the draws must be N(0, std), not the bits of a particular libm (torch.normal's CPU stream
                // cannot be reproduced on the device anyway); the ocml logf / sinf / cosf cost ~100 VALU per agent
                const float rad = __builtin_sqrtf(-2.0f * 0.693147180560f * __builtin_amdgcn_logf(u1));
                nl = rad * __builtin_amdgcn_cosf(u2) * p.noise_std;
                na = rad * __builtin_amdgcn_sinf(u2) * p.noise_std;
            }
            float lin = __fadd_rn(mean.x, nl);
            const float ang = clamp_t(__fadd_rn(mean.y, na), -0.025f, 0.025f);  // :343
            h = __fadd_rn(p.heading[a], __fmul_rn(ang, p.dt));                   // :345
            lin = clamp_t(lin, 5e-6f, p.v_max);                                   // :347
            float sn, cs;
            sincosf(h, &sn, &cs);
            float vx = __fmul_rn(lin, cs);                                        // :351
            float vy = __fmul_rn(lin, sn);                                        // :352
            const float n = sqrt_rn(__fadd_rn(__fmul_rn(vx, vx), __fmul_rn(vy, vy)));  // :358
            vx = __fmul_rn(nan_to_num(__fdiv_rn(vx, n)), p.dt);                  // :358-365
            vy = __fmul_rn(nan_to_num(__fdiv_rn(vy, n)), p.dt);
            x = __fadd_rn(x, vx);                                                 // :366
            y = __fadd_rn(y, vy);
            p.heading[a] = h;
            reinterpret_cast<float2*>(p.vel)[a] = make_float2(vx, vy);
        } else if (variant == FLOCK_VARIANT_FLOCK) {  // gym_flock.py:194-200
            const float2 ac = reinterpret_cast<const float2*>(p.action)[a];
            const float2 v0 = reinterpret_cast<const float2*>(p.vel)[a];
            float vx = __fadd_rn(v0.x, __fmul_rn(ac.x, p.dt));                   // :196
            float vy = __fadd_rn(v0.y, __fmul_rn(ac.y, p.dt));
            const float n = sqrt_rn(__fadd_rn(__fmul_rn(vx, vx), __fmul_rn(vy, vy)));  // :198
            vx = __fdiv_rn(vx, n);
            vy = __fdiv_rn(vy, n);
            x = __fadd_rn(x, __fmul_rn(vx, p.dt));                               // :200
            y = __fadd_rn(y, __fmul_rn(vy, p.dt));
            reinterpret_cast<float2*>(p.vel)[a] = make_float2(vx, vy);
        }
        if (variant != kSense) {
            x = boundary(x, p.box, p.rigid);  // check_boundary :271-304
            y = boundary(y, p.box, p.rigid);
            st_o<kNtOut>(reinterpret_cast<f32x2*>(p.pos) + a, f32x2{x, y});
        }
        lpos[g * p.S + i] = make_float2(x, y);
    }
#ifdef FLOCK_PHASE_PROF
    PHASE(10);  // kinematics arithmetic and stores issued
#endif
    if (kLateAfter) load_late();
#ifdef FLOCK_PHASE_PROF
    PHASE(11);  // late loads issued
#endif
    // L2 pull-ahead (pf_ahead > 0: more env blocks than are resident, launch_spec): the block that will take this
    // one's place on the CU is pf_ahead blocks later; one lane per 128 B pulls its positions, headings and actions
    // into the caches (one dword each, kept in a register that is only consumed at the end), issued after this
    // block's own loads so that no wait for them waits for the pull. Config 5: 0.807 -> 0.760 ms per launch, 0.687 with
    // the late inputs too (PFM 3); config 3 as one launch (4096 blocks, 2048 resident): 39.0-39.2 -> 37.2-37.8 µs
    // (the late inputs there: 38.7-39.7 µs, not pulled) (profiles/r04/pf/)
    int pf_sink = 0;
    const bool pf_on = PFM != 0 && p.pf_ahead > 0;  // PFM: 1 the kinematics inputs, 3 also the late inputs
    auto do_pull = [&]() {
        const int eb = p.env0 + (int)(blockIdx.x + p.pf_ahead) * p.G;
        const int ne = min(p.G, p.E - eb);
        if (ne > 0) {
            const int nb = ne * p.N;             // agents of that block
            const int l8 = (nb * 8 + 127) >> 7;  // lines of the 8-B fields, of the heading
            const int l4 = (nb * 4 + 127) >> 7;
            const char* base = nullptr;
            int q = t;
            if (q < l8) {
                base = reinterpret_cast<const char*>(p.pos) + (size_t)eb * p.N * 8;
            } else if ((q -= l8) < l4) {
                base = reinterpret_cast<const char*>(p.heading) + (size_t)eb * p.N * 4;
            } else if ((q -= l4) < l8) {
                base = variant == FLOCK_VARIANT_UW_DISCRETE ? reinterpret_cast<const char*>(p.action_id)
                                                             : reinterpret_cast<const char*>(p.action);
                if (base) base += (size_t)eb * p.N * 8;
            } else if ((q -= l8) < ((PFM & 2) && p.seeds && p.k == 4 ? l8 : 0)) {  // PFM & 2: the compact seeds,
                base = reinterpret_cast<const char*>(p.seeds) + (size_t)eb * p.N * 8;
            } else if ((q -= ((PFM & 2) && p.seeds && p.k == 4 ? l8 : 0)) <
                       ((PFM & 2) && p.r_state && p.k == 4 ? 2 * l8 : 0)) {  // the previous observation rows
                base = reinterpret_cast<const char*>(p.r_prev) + (size_t)eb * p.N * 16;
            }
            if (base) pf_sink = *reinterpret_cast<const int*>(base + (size_t)q * 128);
        }
    };
    if (pf_on && kPullAt == 0) do_pull();

    PHASE(0);
    // ---- phase 2: per-env sums in a fixed tree order (same order as oracle tree_sum) -------------------------
    // (the rounds s < 64 as wave shuffles, 5 block barriers instead of 10 at N = 512: bitwise the same, config 4
    // 0.1899-0.1910 vs 0.1893-0.1906 ms per step, config 2 flat; profiles/r05/wavetail/: not kept)
    float s0 = 0.0f, s1 = 0.0f;
    if (variant == FLOCK_VARIANT_UW || variant == FLOCK_VARIANT_UW_DISCRETE) {
        float* r0 = red + (size_t)g * 2 * p.P;
        float* r1 = r0 + p.P;
        if (in_group) {
            r0[i] = active ? (variant == FLOCK_VARIANT_UW ? x : h) : 0.0f;
            r1[i] = active ? y : 0.0f;
            if (i < p.P - p.N) {
                r0[p.N + i] = 0.0f;
                r1[p.N + i] = 0.0f;
            }
        }
        __syncthreads();
        for (int s = p.P >> 1; s >= 1; s >>= 1) {
            if (in_group && i < s) {
                r0[i] = __fadd_rn(r0[i], r0[i + s]);
                r1[i] = __fadd_rn(r1[i], r1[i + s]);
            }
            __syncthreads();
        }
        if (in_group) {
            s0 = __fdiv_rn(r0[0], (float)p.N);
            s1 = __fdiv_rn(r1[0], (float)p.N);
        }
    } else {
        __syncthreads();
    }
    // normalize_distance (gym_flock_uw.py:127-133, gym_flock_uw_discrete.py:175-181, gym_flock.py:94-98, the RNN
    // fork's gym_flock_v2.py:136-141): the kNN runs on positions / max_i torch.norm(p_i) of the env; the state, the
    // centre-of-mass and alignment terms keep the raw positions. Runtime flag of the full-scan (!CELL, SPL = 1)
    // Euclidean instantiations only: dispatch() routes normalize there.
    float kx = x, ky = y;  // the kNN's coordinates of this agent
    if (!CELL && !PERIODIC && SPL == 1 && p.normalize) {
        float* r0 = red + (size_t)g * 2 * p.P;
        __syncthreads();  // phase 2's sums have been read
        if (in_group) {
            r0[i] = active ? sqrt_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y))) : 0.0f;  // norms >= 0: 0 pads
            if (i < p.P - p.N) r0[p.N + i] = 0.0f;
        }
        __syncthreads();
        for (int s = p.P >> 1; s >= 1; s >>= 1) {  // the max is exact in any order
            if (in_group && i < s) r0[i] = fmaxf(r0[i], r0[i + s]);
            __syncthreads();
        }
        if (active) {
            const float m = r0[0];
            kx = __fdiv_rn(x, m);
            ky = __fdiv_rn(y, m);
            lpos[g * p.S + i] = make_float2(kx, ky);
        }
        __syncthreads();
    }

    PHASE(1);
    // ---- phase 3c: cell binning (counting sort into the extended cell-sorted array) --------------------------
    int cx = 0, cy = 0;
#ifdef FLOCK_DIAG_BINREP  // diagnostics: the binning phase run FLOCK_DIAG_BINREP times (its marginal cost; same results)
    for (int rep_ = 0; rep_ < FLOCK_DIAG_BINREP; ++rep_)
#endif
    if (CELL) {
        int* cnt = cnt_all + g * ncell;
        int* pre = pre_all + g * npre;
        float4* ext = ext_all + g * p.ecap;
#ifdef FLOCK_DIAG_BINREP
        if (rep_ > 0) {
            if (in_group)
                for (int c = i; c < ncell; c += p.N) cnt[c] = 0;
            __syncthreads();
        }
#endif
        int rank = 0;
        if (active) {
            cx = min((int)(x * p.inv_cwx), gx - 1);  // x, y in [0, box] after check_boundary
            cy = min((int)(y * p.inv_cwy), gy - 1);
            rank = atomicAdd(&cnt[cy * gx + cx], 1);
        }
        __syncthreads();
        // exclusive prefix over the env's virtual cells by all of its lanes (envs are wave-aligned whenever CELL):
        // `per` consecutive virtual cells per lane, a DPP wave scan, the wave totals through LDS
        {
            const int nv = npre - 1, per = (npre + p.N - 1) / p.N;
            const int f0 = in_group ? i * per : npre;
            const int y0 = f0 / W2, e0 = f0 - y0 * W2;
            auto vcount = [&](int yy, int e) {
                if (EVR && e == W2 - 1) return 1;                                        // the row sentinel
                if (e < kRg) return PERIODIC ? cnt[yy * gx + gx - kRg + e] : 0;          // ghosts of the last columns
                if (e >= gx + kRg) return PERIODIC ? cnt[yy * gx + e - gx - kRg] : 0;    // ghosts of the first columns
                return cnt[yy * gx + e - kRg];
            };
            int local = 0;
            for (int q = 0, yy = y0, e = e0; q < per && f0 + q < nv; ++q) {
                local += vcount(yy, e);
                if (++e == W2) {
                    e = 0;
                    ++yy;
                }
            }
            const int inc = wave_incl_scan(local);
            const int wv = i >> 6;
            int* wtot = wtot_all + g * 16;
            const int wsum = __builtin_amdgcn_readlane(inc, 63);
            if (in_group && (i & 63) == 0) wtot[wv] = wsum;
            __syncthreads();
            int run = inc - local;
            if (in_group)
                for (int w = 0; w < wv; ++w) run += wtot[w];
            for (int q = 0, yy = y0, e = e0; q < per && f0 + q < npre; ++q) {
                pre[f0 + q] = run;
                if (f0 + q < nv) run += vcount(yy, e);
                if (++e == W2) {
                    e = 0;
                    ++yy;
                }
            }
        }
        __syncthreads();
        if (active) {
            const float4 ent = make_float4(x, y, __int_as_float(i), 0.0f);
            const float4 ghost = make_float4(x, y, __int_as_float(i), p.box);  // sx = B: see pair_d2_shift
            const int* pr = pre + cy * W2;
            ext[pr[cx + kRg] + rank] = ent;
            if (PERIODIC && cx >= gx - kRg) ext[pr[cx - gx + kRg] + rank] = ghost;  // in front (gx >= 2 kRg)
            if (PERIODIC && cx < kRg) ext[pr[gx + kRg + cx] + rank] = ghost;        // behind
        }
        // a sentinel behind the last entry (the seeded scan's clamp target): +inf position, d2 = +inf, a key above
        // every real one
        if (in_group && i == 0) {
            ext[pre[npre - 1]] = make_float4(__builtin_inff(), __builtin_inff(), __int_as_float(0), 0.0f);
            if (EVR)  // and a second one (ext_cap): the scan's slot pairs read c and c + 1
                ext[pre[npre - 1] + 1] = make_float4(__builtin_inff(), __builtin_inff(), __int_as_float(0), 0.0f);
        }
        if (EVR && in_group && i < gy)  // each row's sentinel cell
            ext[pre[i * W2 + W2 - 1]] = make_float4(__builtin_inff(), __builtin_inff(), __int_as_float(0), 0.0f);
        __syncthreads();
    }

    PHASE(2);
    if (pf_on && kPullAt == 1) do_pull();
    // ---- phase 3/4: kNN -------------------------------------------------------------------------------
    float bd[L - 1];
    int bj[L - 1];
    uint32_t key[L];
    bool ok = false;
    int R = 0;  // scanned neighbourhood radius (0: all N)
    if (CELL) {  // every lane of the wave (the trip counts are wave-wide maxima); lanes without an agent scan nothing
        const float4* ext = ext_all + g * p.ecap;
        const int* pre = pre_all + g * npre;
        const int cmax = p.ecap - 2;
        // seeds: the lane itself and its k previous neighbours (nn_idx on entry) are k+1 distinct agents, so their
        // largest distance bounds the (k+1)-th nearest; r adds 2^(ib-20) relative (>= 16 truncated-d2 buckets) and
        // a 1e-5 box margin. Seeds that are out of range or repeated (a stale or uninitialised buffer) fall back.
        bool use = false;
        float r = 0.0f;
        bool seeds_ok = has_hint;
        if (seed_packed) {
            hint[0] = seed_raw.x & 0xFFFFu;
            hint[1 % (L - 2)] = seed_raw.x >> 16;
            hint[2 % (L - 2)] = seed_raw.y & 0xFFFFu;
            hint[3 % (L - 2)] = seed_raw.y >> 16;
        }
        int seed[L - 2];
#pragma unroll
        for (int s = 0; s < L - 2; ++s) {
            seed[s] = (int)min((uint64_t)hint[s], (uint64_t)(p.N - 1));  // in range for the LDS read either way
            if (s < p.k) seeds_ok = seeds_ok && (uint64_t)hint[s] < (uint64_t)p.N && seed[s] != i;
        }
#pragma unroll
        for (int s = 0; s < L - 2; ++s)
#pragma unroll
            for (int u = s + 1; u < L - 2; ++u)
                if (u < p.k) seeds_ok = seeds_ok && seed[s] != seed[u];
        if (active && seeds_ok) {
            const float2* cand = lpos + g * p.S;
            float rho2 = 0.0f;
#pragma unroll
            for (int s = 0; s < L - 2; ++s)
                if (s < p.k) {
                    const float2 c = cand[seed[s]];
                    rho2 = fmaxf(rho2, pair_d2<PERIODIC>(x, y, c.x, c.y, p.box));
                }
            r = sqrtf(rho2) * (1.0f + __int_as_float((127 + p.ib - 20) << 23)) + p.cell_eps;
            // at most kRows rows; periodic: at most kRg - 1 columns either side (see cand_d2x2). Without wrap, rows
            // and columns beyond the box are empty, so only the rows inside it count
            int q0 = (int)floorf((y - r) * p.inv_cwy), q1 = (int)floorf((y + r) * p.inv_cwy);
            if (!PERIODIC) {
                q0 = max(q0, 0);
                q1 = min(q1, gy - 1);
            }
            use = (!PERIODIC || r <= p.r_lim) && q1 - q0 < kRows;
        }
#ifdef FLOCK_DIAG_NOSCAN  // diagnostics only: cost of everything but the cell scans (results are wrong)
        use = false;
#pragma unroll
        for (int s = 0; s < L; ++s) key[s] = kEmpty;
#else
        scan_seeded<L, PERIODIC, EVR>(key, ext, pre, gx, gy, cy, use, r, p.ib, x, y, p.box, p.cwy, p.inv_cwx, p.inv_cwy,
                                 pre[npre - 1]);
#endif
        ok = use;
        R = 1;  // rows of the exact rescan
        PHASE(3);
#ifdef FLOCK_DIAG_NOSCAN
        ok = true;
        if (false) {
#else
        if (__ballot(active && !use) != 0) {  // wave-uniform: lanes without a usable disk take the proved square
#endif
            PHASE_COUNT(16, 1);
            uint32_t key2[L];
            const bool ok2 = scan_square<L, PERIODIC, EVR>(key2, ext, pre, gx, gy, cx, cy, 1, p.ib, x, y, p.box, p.cwx,
                                                      p.cwy, p.cell_eps, cmax, active && !use);
            if (!use) {
#pragma unroll
                for (int s = 0; s < L; ++s) key[s] = key2[s];
                ok = ok2;
            }
        }
        PHASE(4);
    }
#ifdef FLOCK_PHASE_PROF
    if (__ballot(active && !ok) != 0) PHASE_COUNT(17, 1);
#endif
    if constexpr (SPL > 1) {  // split scan: every lane group takes 1 / SPL of the candidates, then the merge
        constexpr int Q = NC / SPL;
        const int q = t / NC, ia = t - q * NC;
        const bool live = p.env0 + (int)blockIdx.x < p.E;
        uint32_t part[L];
        if (live) {
            const float2 me = lpos[ia];  // published by the phase-2 barrier
            scan_range<L, PERIODIC>(part, lpos, q * Q, q * Q + Q, p.ib, me.x, me.y, p.box);
        }
        uint32_t* mk = reinterpret_cast<uint32_t*>(ext_all);  // [SPL - 1][L][NC] (no cell list here)
        if (q > 0 && live)
#pragma unroll
            for (int s = 0; s < L; ++s) mk[((q - 1) * L + s) * NC + ia] = part[s];
        __syncthreads();
        if (q == 0 && live) {
#pragma unroll
            for (int s = 0; s < L; ++s) key[s] = part[s];
            for (int r = 0; r < SPL - 1; ++r)
#pragma unroll
                for (int s = 0; s < L; ++s) key_insert<L>(key, mk[(r * L + s) * NC + ia]);
        }
        ok = true;
    }
    bool amb = false;
    if (active) {
        if (!ok) {
            scan_all<L, PERIODIC>(key, lpos + g * p.S, p.N, p.ib, kx, ky, p.box);
            R = 0;
        }
        amb = knn_finalize<L, PERIODIC>(key, lpos + g * p.S, p.N, p.k, p.ib, kx, ky, p.box, bd, bj, false);
#ifdef FLOCK_PHASE_PROF
        if (__ballot(amb) != 0) PHASE_COUNT(18, 1);
#endif
    }
#ifdef FLOCK_DIAG_NORESCAN  // diagnostics only: timing without the exact rescans (ambiguous lanes are wrong)
    amb = false;
#endif
    // lanes with an ambiguous (k+1) / (k+2) bucket: exact rescan by the whole wave (every lane of the wave is here;
    // with CELL, envs are wave-aligned) of rows cy-1..cy+1, columns cx-kRg..cx+kRg (cell lanes, R = 1) or of all N
    // agents (R = 0)
    if (__ballot(amb) != 0) {
#ifdef FLOCK_SERIAL_RESCAN  // A/B builds: the one-lane rescans
        if (amb && R == 0) knn_finalize<L, PERIODIC>(key, lpos + g * p.S, p.N, p.k, p.ib, kx, ky, p.box, bd, bj, true);
        if (CELL && amb && R == 1)
            exact_rescan_cells<L, PERIODIC, EVR>(bd, bj, ext_all + g * p.ecap, pre_all + g * npre, gx, gy, cx, cy, R, x, y,
                                            p.box);
#else
        exact_rescan_wave<L, PERIODIC, CELL, EVR>(bd, bj, amb, R, lpos, p.S, p.N, ext_all, pre_all, p.ecap, npre, g, gx, gy,
                                             cx, cy, kx, ky, p.box);
#endif
    }
    PHASE(5);

    // ---- phase 5: outputs -----------------------------------------------------------------------------
    int coll = 0;
    if (active) {
        float dv[L - 1];
#pragma unroll
        for (int s = 1; s < L - 1; ++s) {
            if (s <= p.k) {
                float d = sqrt_rn(bd[s]);
                if (p.clamp) d = clamp_t(d, 0.0f, p.sensor_range);  // gym_flock_v2.py:151
                dv[s - 1] = d;
                coll |= (d < p.cd);                                   // :212-215
                if (!(L - 2 == 4 && p.k == 4)) p.dnn[a * p.k + (s - 1)] = d;
                if (p.idx) p.idx[a * p.k + (s - 1)] = (int64_t)bj[s];
            }
        }
        if (L - 2 == 4 && p.k == 4)  // one 16-B store
            st_o<kNtOut>(reinterpret_cast<f32x4*>(p.dnn + a * p.k), f32x4{dv[0], dv[1 % (L - 1)], dv[2 % (L - 1)], dv[3 % (L - 1)]});
        if (CELL && p.seeds) {  // this step's neighbours: the next step's search seeds
            uint16_t* sp = p.seeds + a * p.k;
            if (L - 2 == 4 && p.k == 4)
                st_o<kNtOut>(reinterpret_cast<u32x2*>(sp), u32x2{(uint32_t)bj[1] | ((uint32_t)bj[2 % (L - 1)] << 16),
                                                         (uint32_t)bj[3 % (L - 1)] | ((uint32_t)bj[4 % (L - 1)] << 16)});
            else
#pragma unroll
                for (int s = 1; s < L - 1; ++s)
                    if (s <= p.k) sp[s - 1] = (uint16_t)bj[s];
        }
        if (variant == FLOCK_VARIANT_UW || variant == FLOCK_VARIANT_FLOCK) {  // torch.roll + insert (:120-123)
            float* mo = p.mem_out + a * kMem * p.k;
            if (kMemEarly && L - 2 == 4 && p.k == 4) {  // the prefetched frames, 4 x float4 stores
                float4* mo4 = reinterpret_cast<float4*>(mo);
                mo4[0] = make_float4(dv[0], dv[1 % (L - 1)], dv[2 % (L - 1)], dv[3 % (L - 1)]);
#pragma unroll
                for (int f = 0; f < (SPL > 1 ? 0 : kMem - 1); ++f)  // (split: the other lane groups rolled them)
                    mo4[f + 1] = make_float4(mrow[(f * (L - 2)) % kMemKeep], mrow[(f * (L - 2) + 1) % kMemKeep],
                                             mrow[(f * (L - 2) + 2) % kMemKeep], mrow[(f * (L - 2) + 3) % kMemKeep]);
            } else if (kMemEarly) {
#pragma unroll
                for (int f = 0; f < kMem - 1; ++f)
#pragma unroll
                    for (int c = 0; c < L - 2; ++c)
                        if (c < p.k) mo[(f + 1) * p.k + c] = mrow[(f * (L - 2) + c) % kMemKeep];
#pragma unroll
                for (int s = 0; s < L - 2; ++s)
                    if (s < p.k) mo[s] = dv[s];
            } else {
                const float* mi = p.mem_in + a * kMem * p.k;
                for (int c = 0; c < p.k; ++c) {
                    for (int s = kMem - 1; s >= 1; --s) mo[s * p.k + c] = mi[(s - 1) * p.k + c];
                }
#pragma unroll
                for (int s = 0; s < L - 2; ++s)
                    if (s < p.k) mo[s] = dv[s];
            }
        }
        if (variant != kSense) {
            st_o<kNtOut>(p.done + a, (uint8_t)coll);
            float r;
            if (variant == FLOCK_VARIANT_UW) {  // gym_flock_uw.py:206-221
                const float com_x = __fsub_rn(x, s0), com_y = __fsub_rn(y, s1);
                const float dist = sqrt_rn(__fadd_rn(__fmul_rn(com_x, com_x), __fmul_rn(com_y, com_y)));
                const float com = (dist < p.com_r) ? 0.01f : 0.0f;                  // :197
                const float prev = prev_h;
                const float angp = (fabsf(__fsub_rn(prev, h)) > 0.27f) ? -0.01f : 0.001f;  // :202-204
                p.prev_heading[a] = h;
                r = __fadd_rn(__fadd_rn(coll ? -5.0f : 0.01f, com), angp);          // :220
            } else if (variant == FLOCK_VARIANT_UW_DISCRETE) {  // gym_flock_uw_discrete.py:260-276
                const float err = fabsf(__fsub_rn(s0, h));                            // :256-257
                const float align = (err > 0.2f) ? 0.0f : 0.1f;                       // :258
                p.prev_heading[a] = h;                                                // :270 side effect
                r = __fadd_rn(coll ? -9.0f : 0.0f, align);                            // :237, :275
            } else {
                r = coll ? -5.0f : 0.01f;  // gym_flock_v2.py:217-220, gym_flock.py:142-145
            }
            st_o<kNtOut>(p.reward + a, r);
            if (p.r_state && r_unit >= p.r_skip) {  // fused replay insert: row (start + unit - skip) mod cap
                int64_t row = p.r_start + r_unit - p.r_skip;
                if (row >= p.r_cap) row -= p.r_cap;
                const int64_t e = row * p.r_group + r_slot;  // this agent's element of the row
                if (L - 2 == 4 && p.k == 4) {  // 16-B stores (the RNN-MADDPG ring's actor copies too)
                    const f32x4 so{prev_obs[0], prev_obs[1 % (L - 2)], prev_obs[2 % (L - 2)], prev_obs[3 % (L - 2)]};
                    const f32x4 sn{dv[0], dv[1 % (L - 1)], dv[2 % (L - 1)], dv[3 % (L - 1)]};
                    st_ring(reinterpret_cast<f32x4*>(p.r_state + e * p.k), so);
                    st_ring(reinterpret_cast<f32x4*>(p.r_new + e * p.k), sn);
                    if (p.r_astate) st_ring(reinterpret_cast<f32x4*>(p.r_astate + e * p.k), so);
                    if (p.r_anew) st_ring(reinterpret_cast<f32x4*>(p.r_anew + e * p.k), sn);
                } else {
#pragma unroll
                    for (int s = 0; s < L - 2; ++s)
                        if (s < p.k) {
                            p.r_state[e * p.k + s] = prev_obs[s];
                            p.r_new[e * p.k + s] = dv[s];
                            if (p.r_astate) p.r_astate[e * p.k + s] = prev_obs[s];
                            if (p.r_anew) p.r_anew[e * p.k + s] = dv[s];
                        }
                }
                if (p.r_ids)
                    st_ring(p.r_action + e, act_in.x);
                else
                    st_ring(reinterpret_cast<f32x2*>(p.r_action) + e, f32x2{act_in.x, act_in.y});
                st_ring(p.r_reward + e, r);
                if (!p.r_env_done) st_ring(p.r_term + e, (coll != 0) == (p.r_done != 0) ? 1.0f : 0.0f);
            }
        }
    }
    PHASE(6);
    if (variant != kSense) {  // _computeDone :306-315
        if (p.G == 1) {
            // one env per block: no trailing barrier. Each wave ORs its collisions into flags[0] and then adds its
            // agent count to the arrival counter (release); the wave that completes the count (acquire) has seen
            // every OR and publishes any_done
            const bool coll_w = __ballot(active && coll) != 0;
            const int na = __popcll(__ballot(active));
            if ((t & 63) == 0 && na) {
                if (coll_w) __hip_atomic_fetch_or(&flags[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int old = __hip_atomic_fetch_add(&flags[1], na, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (old + na == p.N) {
                    const int f = __hip_atomic_load(&flags[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    p.any_done[env] = (uint8_t)f;
                    env_done_row(p, env, f);
                }
            }
        } else {
            if (active && coll) atomicOr(&flags[g], 1);
            __syncthreads();
            if (active && i == 0) {
                p.any_done[env] = (uint8_t)flags[g];
                env_done_row(p, env, flags[g]);
            }
        }
    }
    PHASE(7);
    if (pf_on) asm volatile("" ::"v"(pf_sink));  // the L2 pull completes before the wave ends
    PHASE_FLUSH();
}

// ---------------------------------------------------------------------------------------------------------------
// K steps of gym_flock_uw in ONE launch (flock_rollout_uw; BASELINE config 2: 64 agents per env, k = 4, Euclidean kNN,
// 4-frame observation memory), for the random-action rollout regime where the K actions are known up front. One
// workgroup of 4 x 64 lanes owns one env for all K steps and keeps its state on chip: positions, previous headings and
// the memory frames in registers, each step's positions in LDS. A step's HBM traffic is then its action read and its
// observation / reward / done writes (77 B per agent-step; a single step also reads and rewrites the state and the
// memory: the 149 B of SURVEY §8(d)'s accounting), and the launch pays its dispatch and its first loads once per K steps.
// SPL lanes per agent (SPL waves per env; 2 by default): lane r of agent ia runs its kinematics redundantly, scans
// candidates [r N / SPL, (r + 1) N / SPL), and the SPL partial top-L key lists are merged by xor shuffles: the same key
// set, hence the same result, as the split step kernel's LDS merge. Lane r holds memory frames [r 4 / SPL, (r + 1) 4 /
// SPL), so the memory roll is one shuffle. The centre of mass is the step kernel's fixed power-of-two tree
// (r[i] += r[i + s], s = 32 .. 1) as wave shuffles: the same pairs in the same order, bitwise equal. One workgroup
// barrier per step (the positions are double-buffered in LDS, so a wave one step ahead never overwrites the positions
// another wave still scans). The results are bitwise those of K flock_step_uw calls (tests/test_gpu_rollout.py).
constexpr int kRollN = 64;
// SPL lanes per agent (2 or 4): SPL waves per env, each wave 64 / SPL agents; lane r of an agent scans candidates
// [r N / SPL, (r + 1) N / SPL) and holds memory frames [r 4 / SPL, (r + 1) 4 / SPL)
template <int SPL>
__global__ __launch_bounds__(SPL * kRollN) void rollout_uw_kernel(const Params p, int K,
                                                                  const float* __restrict__ actions,
                                                                  float* __restrict__ obs, float* __restrict__ rew_out,
                                                                  uint8_t* __restrict__ done_out,
                                                                  uint8_t* __restrict__ any_out) {
    constexpr int N = kRollN, L = 6, KN = L - 2, IB = 6;  // k = 4; IB = ceil_log2(N)
    constexpr int APW = 64 / SPL, Q = N / SPL, FPL = kMem / SPL;  // agents per wave, candidates / frames per lane
    static_assert(SPL == 2 || SPL == 4, "2 or 4 lanes per agent");
    __shared__ float2 lpos[2][N];
    __shared__ int flag[2];  // any_done of a step, by step parity
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int ia = APW * w + (l & (APW - 1)), r = l / APW;
    const int env = blockIdx.x;
    const size_t a = (size_t)env * N + ia;
    const size_t EN = (size_t)p.E * N;
    if (t < 2) flag[t] = 0;
    const f32x2 p0 = reinterpret_cast<const f32x2*>(p.pos)[a];
    float x = p0.x, y = p0.y;
    const float h = p.heading[a];
    float prev_h = p.prev_heading[a];
    float4 fr[FPL];  // memory frames r FPL .. r FPL + FPL - 1
#pragma unroll
    for (int f = 0; f < FPL; ++f) fr[f] = reinterpret_cast<const float4*>(p.mem_in)[a * kMem + r * FPL + f];
    f32x2 act = ld_i<true>(reinterpret_cast<const f32x2*>(actions) + a);
    float vx = 0.0f, vy = 0.0f, rw = 0.0f;
    float dv[KN];
    int bj[L - 1];
#pragma unroll
    for (int q = 0; q < KN; ++q) dv[q] = 0.0f;
#pragma unroll
    for (int q = 0; q < L - 1; ++q) bj[q] = 0;
    int coll = 0;
    for (int s = 0; s < K; ++s) {
        f32x2 nxt = act;  // the next step's action, in flight during this step
        if (s + 1 < K) nxt = ld_i<true>(reinterpret_cast<const f32x2*>(actions) + (size_t)(s + 1) * EN + a);
        // kinematics + check_boundary (gym_flock_uw.py:269-302; the step kernel's FLOCK_VARIANT_UW branch)
        const float n = sqrt_rn(__fadd_rn(__fmul_rn(act.x, act.x), __fmul_rn(act.y, act.y)));
        vx = __fmul_rn(nan_to_num(__fdiv_rn(act.x, n)), p.dt);
        vy = __fmul_rn(nan_to_num(__fdiv_rn(act.y, n)), p.dt);
        x = boundary(__fadd_rn(x, vx), p.box, p.rigid);
        y = boundary(__fadd_rn(y, vy), p.box, p.rigid);
        float2* lp = lpos[s & 1];
        if (r == 0) lp[ia] = make_float2(x, y);
        __syncthreads();
        if (t == 0 && s > 0) {  // the previous step's any_done: every wave ORed into it before this barrier
            any_out[(size_t)(s - 1) * p.E + env] = (uint8_t)flag[(s - 1) & 1];
            flag[(s - 1) & 1] = 0;  // reused by step s + 1, whose ORs come after the next barrier
        }
        // centre of mass (gym_flock_uw.py:206-210): every wave, lane = agent
        const float2 c = lp[l];
        float sx = c.x, sy = c.y;
#pragma unroll
        for (int o = N / 2; o >= 1; o >>= 1) {
            sx = __fadd_rn(sx, __shfl_down(sx, o));
            sy = __fadd_rn(sy, __shfl_down(sy, o));
        }
        const float s0 = __fdiv_rn(__shfl(sx, 0), (float)N), s1 = __fdiv_rn(__shfl(sy, 0), (float)N);
        // kNN (_computeDistances :155-175 + topk): 1 / SPL of the candidates per lane, the lists merged
        uint32_t key[L];
        scan_range<L, false>(key, lp, Q * r, Q * r + Q, IB, x, y, p.box);
#pragma unroll
        for (int m = APW; m < 64; m <<= 1) {
            uint32_t o[L];
#pragma unroll
            for (int q = 0; q < L; ++q) o[q] = (uint32_t)__shfl_xor((int)key[q], m);
#pragma unroll
            for (int q = 0; q < L; ++q) key_insert<L>(key, o[q]);
        }
        float bd[L - 1];
        const bool amb = knn_finalize<L, false>(key, lp, N, KN, IB, x, y, p.box, bd, bj, false) && r == 0;
        if (__ballot(amb) != 0)
            exact_rescan_wave<L, false, false, false>(bd, bj, amb, 0, lp, N, N, nullptr, nullptr, 0, 0, 0, 0, 0, 0,
                                                      0, x, y, p.box);
        // outputs of step s: distances of the agent's r == 0 lane (clamp, collisions: gym_flock_uw.py:120-123, 215)
        float d4[KN];
#pragma unroll
        for (int q = 0; q < KN; ++q) d4[q] = clamp_t(sqrt_rn(bd[q + 1]), 0.0f, p.sensor_range);
        coll = 0;
#pragma unroll
        for (int q = 0; q < KN; ++q) {
            dv[q] = __shfl(d4[q], l & (APW - 1));
            coll |= (dv[q] < p.cd);
        }
        // torch.roll + insert of the observation memory: frame j <- frame j - 1, frame 0 <- dv. The lane's first frame
        // comes from the previous lane of its agent (l - APW), its others from itself
        float4 in;
        in.x = __shfl(fr[FPL - 1].x, (l - APW) & 63);
        in.y = __shfl(fr[FPL - 1].y, (l - APW) & 63);
        in.z = __shfl(fr[FPL - 1].z, (l - APW) & 63);
        in.w = __shfl(fr[FPL - 1].w, (l - APW) & 63);
#pragma unroll
        for (int f = FPL - 1; f >= 1; --f) fr[f] = fr[f - 1];
        fr[0] = r == 0 ? make_float4(dv[0], dv[1], dv[2], dv[3]) : in;
#pragma unroll
        for (int f = 0; f < FPL; ++f)
            st_o<true>(reinterpret_cast<f32x4*>(obs) + ((size_t)s * EN + a) * kMem + r * FPL + f,
                       f32x4{fr[f].x, fr[f].y, fr[f].z, fr[f].w});
        if (r == 0) {  // reward (gym_flock_uw.py:206-221)
            const float com_x = __fsub_rn(x, s0), com_y = __fsub_rn(y, s1);
            const float dist = sqrt_rn(__fadd_rn(__fmul_rn(com_x, com_x), __fmul_rn(com_y, com_y)));
            const float com = (dist < p.com_r) ? 0.01f : 0.0f;
            const float angp = (fabsf(__fsub_rn(prev_h, h)) > 0.27f) ? -0.01f : 0.001f;
            rw = __fadd_rn(__fadd_rn(coll ? -5.0f : 0.01f, com), angp);
            st_o<true>(rew_out + (size_t)s * EN + a, rw);
            st_o<true>(done_out + (size_t)s * EN + a, (uint8_t)coll);
        }
        prev_h = h;
        if (__ballot(r == 0 && coll) != 0 && l == 0) atomicOr(&flag[s & 1], 1);
        act = nxt;
    }
    __syncthreads();
    if (t == 0) {
        const uint8_t f = (uint8_t)flag[(K - 1) & 1];
        any_out[(size_t)(K - 1) * p.E + env] = f;
        p.any_done[env] = f;
    }
    // the state after the last step, as K flock_step_uw calls leave it
#pragma unroll
    for (int f = 0; f < FPL; ++f) reinterpret_cast<float4*>(p.mem_out)[a * kMem + r * FPL + f] = fr[f];
    if (r == 0) {
        reinterpret_cast<f32x2*>(p.pos)[a] = f32x2{x, y};
        reinterpret_cast<f32x2*>(p.vel)[a] = f32x2{vx, vy};
        p.prev_heading[a] = prev_h;
        reinterpret_cast<f32x4*>(p.dnn)[a] = f32x4{dv[0], dv[1], dv[2], dv[3]};
        p.reward[a] = rw;
        p.done[a] = (uint8_t)coll;
        if (p.idx)
#pragma unroll
            for (int q = 0; q < KN; ++q) p.idx[a * KN + q] = (int64_t)bj[q + 1];
    }
}

// ---------------------------------------------------------------------------------------------------------------
// reset: bounded in-kernel rejection sampling (replaces the reference's unbounded recursion)

template <int L>
__global__ __launch_bounds__(1024) void reset_kernel(const Params p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float2* lpos = reinterpret_cast<float2*>(smem);
    int* flags = reinterpret_cast<int*>(lpos + p.G * p.S);  // [G] collision flag of the current attempt
    int* state = flags + p.G;                                // [G] 1 = still drawing
    int* mx = state + p.G;  // [G] normalize_distance: max |p| of the draw (bits of a float >= 0, ordered as ints)

    const int t = threadIdx.x;
    const int g = t / p.N;
    const int i = t - g * p.N;
    const int env = blockIdx.x * p.G + g;
    const bool in_group = g < p.G;
    const bool active = in_group && env < p.E;
    const size_t a = (size_t)env * p.N + i;
    if (in_group && i == 0) state[g] = (env < p.E) && (p.env_mask == nullptr || p.env_mask[env] != 0);
    __syncthreads();

    float x = 0.0f, y = 0.0f, h = 0.0f;
    float bd[L - 1];
    int bj[L - 1];
    for (int attempt = 0; attempt < p.max_attempts; ++attempt) {
        const bool drawing = in_group && state[g];
        if (in_group && i == 0) flags[g] = 0;
        if (active && drawing) {
            const uint64_t ctr = p.rng_offset + (uint64_t)attempt;
            const U4 r = philox(p.seed, (uint32_t)a, (uint32_t)(a >> 32), (uint32_t)ctr, (uint32_t)(ctr >> 32));
            // positions = (lo - hi) * U + hi  in (lo, hi]   (gym_flock_v2.py:87-89 and siblings)
            const float span = p.range_lo - p.range_hi;
            x = __fadd_rn(__fmul_rn(span, u01(r.x)), p.range_hi);
            y = __fadd_rn(__fmul_rn(span, u01(r.y)), p.range_hi);
            h = __fadd_rn(__fmul_rn(-p.head_hi, u01(r.z)), p.head_hi);  // headings (0 - c) * U + c  (:96)
            x = boundary(x, p.box, p.rigid);                             // :99
            y = boundary(y, p.box, p.rigid);
            lpos[g * p.S + i] = make_float2(x, y);
        }
        if (in_group && i == 0) mx[g] = 0;
        __syncthreads();
        float kx = x, ky = y;  // the kNN's coordinates: positions / max |p| under normalize_distance (:157-163)
        if (p.normalize) {
            if (active && drawing)
                atomicMax(&mx[g], __float_as_int(sqrt_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)))));
            __syncthreads();
            if (active && drawing) {
                const float m = __int_as_float(mx[g]);
                kx = __fdiv_rn(x, m);
                ky = __fdiv_rn(y, m);
                lpos[g * p.S + i] = make_float2(kx, ky);
            }
            __syncthreads();
        }
        if (active && drawing) {
            knn_scan<L, false>(lpos + g * p.S, p.N, p.k, p.ib, kx, ky, p.box, bd, bj);  // Euclidean (:100)
            int coll = 0;
#pragma unroll
            for (int s = 1; s < L - 1; ++s)
                if (s <= p.k) {
                    float d = sqrt_rn(bd[s]);
                    if (p.clamp) d = clamp_t(d, 0.0f, p.sensor_range);
                    coll |= (d < p.check_distance);
                }
            if (coll) atomicOr(&flags[g], 1);
        }
        __syncthreads();
        int more = 0;
        if (in_group && i == 0 && state[g]) {
            state[g] = flags[g];  // keep drawing while the draw has a collision (:105-108)
        }
        __syncthreads();
        if (in_group) more = state[g];
        if (!__syncthreads_or(more)) break;
    }
    // repair (p.repair > 0 rounds; flock_reset_ext): a swarm whose every whole-swarm draw collided (certain at
    // main.py density for N >= 256) keeps its last draw, and every agent closer than
    // check_distance to a LOWER-indexed agent re-draws its own position from a separate Philox stream, round after
    // round, until no pair is that close. The kNN + collision check of the reference then decides valid[] as for
    // a plain draw. Agent 0 never moves, so each round fixes at least the lowest conflicting index.
    if (p.repair > 0 && !p.normalize && __syncthreads_or(in_group && state[g])) {  // (host: repair 0 with normalize)
        const float2* lp = lpos + g * p.S;
        for (int round = 0; round < p.repair; ++round) {
            int bad = 0;
            if (active && state[g]) {
                for (int j = 0; j < i; ++j) {  // Euclidean distance with the kNN's op order
                    const float2 q = lp[j];
                    const float dx = __fsub_rn(x, q.x), dy = __fsub_rn(y, q.y);
                    const float d = sqrt_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)));
                    bad |= (d < p.check_distance);
                }
            }
            __syncthreads();  // every lane has read the round's positions before any rewrite
            if (bad) {
                const uint64_t ctr = p.rng_offset + (uint64_t)round;
                const U4 r = philox(p.seed, (uint32_t)a, (uint32_t)(a >> 32), (uint32_t)ctr,
                                    (uint32_t)(ctr >> 32) | 0x80000000u);
                const float span = p.range_lo - p.range_hi;
                x = boundary(__fadd_rn(__fmul_rn(span, u01(r.x)), p.range_hi), p.box, p.rigid);
                y = boundary(__fadd_rn(__fmul_rn(span, u01(r.y)), p.range_hi), p.box, p.rigid);
                lpos[g * p.S + i] = make_float2(x, y);
            }
            if (!__syncthreads_or(bad)) break;
        }
        if (in_group && i == 0) flags[g] = 0;
        __syncthreads();
        if (active && state[g]) {
            knn_scan<L, false>(lpos + g * p.S, p.N, p.k, p.ib, x, y, p.box, bd, bj);
            int coll = 0;
#pragma unroll
            for (int s = 1; s < L - 1; ++s)
                if (s <= p.k) {
                    float d = sqrt_rn(bd[s]);
                    if (p.clamp) d = clamp_t(d, 0.0f, p.sensor_range);
                    coll |= (d < p.check_distance);
                }
            if (coll) atomicOr(&flags[g], 1);
        }
        __syncthreads();
        if (in_group && i == 0 && state[g]) state[g] = flags[g];
        __syncthreads();
    }
    const bool touched = active && (p.env_mask == nullptr || p.env_mask[env] != 0);
    if (touched) {
        reinterpret_cast<float2*>(p.pos)[a] = make_float2(x, y);
        if (p.heading) p.heading[a] = h;
        if (p.prev_heading) p.prev_heading[a] = 0.0f;
        if (p.vel) reinterpret_cast<float2*>(p.vel)[a] = make_float2(0.0f, 0.0f);
#pragma unroll
        for (int s = 1; s < L - 1; ++s) {
            if (s <= p.k) {
                float d = sqrt_rn(bd[s]);
                if (p.clamp) d = clamp_t(d, 0.0f, p.sensor_range);
                p.dnn[a * p.k + (s - 1)] = d;
                if (p.idx) p.idx[a * p.k + (s - 1)] = (int64_t)bj[s];
                if (p.mem_out) {
                    float* mo = p.mem_out + a * kMem * p.k;
                    mo[s - 1] = d;
                    for (int f = 1; f < kMem; ++f) mo[f * p.k + (s - 1)] = 0.0f;
                }
            }
        }
        if (i == 0 && p.valid) p.valid[env] = (uint8_t)(state[g] == 0);
    }
}

// ---------------------------------------------------------------------------------------------------------------
// host side

int ceil_log2(int n) {
    int b = 0;
    while ((1 << b) < n) ++b;
    return b;
}

struct Cfg {
    int G, T, S, P, blocks;
    size_t lds;
};

// cell grid of the step kernel's cell list (N >= 128): about one agent per cell, rows about twice the typical
// (k+1)-th neighbour distance tall (0.38 sqrt N rows: 5 agents within r_typ means r_typ = box sqrt(5 / (pi N))), at
// least kRows distinct rows and gx >= 2 kRg + 4 columns (cand_d2x2). Returns false for the full-scan path.
bool cell_grid(int N, int variant, int* gx, int* gy) {
    if (variant == kSense || N < 128) return false;
    *gy = max(kRows, (int)(0.38f * sqrtf((float)N)));
    *gx = max(2 * kRg + 4, N / *gy);
    return true;
}

Cfg make_cfg(int E, int N, bool reset, int cells, int gx, int gy, int G = 0, bool evr = false) {
    Cfg c;
    c.S = (N + 1) & ~1;
    c.P = 1 << ceil_log2(N);
    c.G = G > 0 ? G : ((N <= 256) ? (256 / N) : 1);
    c.T = ((c.G * N + 63) / 64) * 64;
    c.blocks = (E + c.G - 1) / c.G;
    if (reset)
        c.lds = (size_t)c.G * c.S * sizeof(float2) + 3 * c.G * sizeof(int);
    else
        c.lds = (size_t)c.G * c.S * sizeof(float2) + (size_t)2 * c.G * c.P * sizeof(float) + 2 * c.G * sizeof(int);
    if (!reset && cells) {  // ext (2N + 2 float4, 16-B aligned) + cnt + pre per env
        c.lds = (c.lds + 15) & ~(size_t)15;
        c.lds += (size_t)c.G * ((size_t)ext_cap(N, gy, evr) * sizeof(float4) +
                                (size_t)(gx * gy + gy * row_stride(gx, evr) + 1 + 16) * 4);
    }
    return c;
}

int check_common(int E, int N, int k) {
    if (E < 0 || N < 1) return fail(FLOCK_E_ARG, "E must be >= 0 and N >= 1");
    if (k < 1 || k + 1 > N) return fail(FLOCK_E_K_RANGE, "selected index k out of range");
    if (k > 15) return fail(FLOCK_E_LIMIT, "this build supports k <= 15");
    if (N > 1024) return fail(FLOCK_E_LIMIT, "this build supports N <= 1024 agents per env");
    return FLOCK_OK;
}

// diagnostics knobs (flock_set_diag; A/B tests and tools): env_launches = n splits a step into n launches over
// consecutive env ranges; no_spec takes the generic instantiations; no_split the one-lane-per-agent scan of the split
// (SPL > 1) instantiations; no_cells the full scan instead of the cell list; pf = 0 turns off the env blocks' L2
// pull-ahead (step_kernel's PFM, compiled only into the shapes that use it; -1: on)
struct Knobs {
    int env_launches = 1;
    bool no_spec = false, no_split = false, no_cells = false;
    int pf = -1;
    int rollout_spl = 2;  // lanes per agent of the uw rollout kernel (2 or 4)
};
Knobs& knobs_mut() {
    static Knobs k;
    return k;
}
const Knobs& knobs() { return knobs_mut(); }
int env_launches(int blocks, int requested) {
    const int n = requested > 0 ? requested : knobs().env_launches;
    return n < 1 ? 1 : (n > blocks ? blocks : n);
}

// the specialised instantiations (step_kernel VAR / NC / SPL): the BASELINE configurations' per-GPU shapes
// resident blocks of a kernel on the current device (occupancy at T threads and lds bytes per block); 0 on error
int resident_blocks(const void* kernel, int T, size_t lds) {
    int dev = 0, per_cu = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, T, lds) != hipSuccess)
        return 0;
    return per_cu * cus;
}

template <int VAR, int NC, bool PERIODIC, bool CELL, int GXC, int GYC, int SPL = 1, int PF = 0, bool EVR = false>
bool launch_spec(const Cfg& c0, const Params& p0, hipStream_t s) {
    if (p0.variant != VAR || p0.N != NC || p0.k != 4 || (p0.periodic != 0) != PERIODIC || (p0.cells != 0) != CELL ||
        p0.normalize)
        return false;
    if (CELL && (p0.gx != GXC || p0.gy != GYC || p0.ecap != ext_cap(NC, GYC, false))) return false;
    if (knobs().no_spec) return false;  // A/B diagnostics: the generic instantiation
    Cfg c = c0;
    Params p = p0;
    if (EVR) {  // the even-row layout: row sentinels in ext (its capacity and the LDS size)
        static_assert(!EVR || CELL, "the even-row layout is a cell-list layout");
        c = make_cfg(p.E, NC, false, p.cells, GXC, GYC, 0, true);
        p.ecap = ext_cap(NC, GYC, true);
    }
    if (SPL > 1) {  // one env per block of SPL * NC lanes; LDS: the G = 1 layout + the merge lists in place of ext
        if (knobs().no_split) return false;
        c = make_cfg(p.E, NC, false, 0, 0, 0, 1);
        c.T = SPL * NC;
        c.lds = ((c.lds + 15) & ~(size_t)15) + (size_t)(SPL - 1) * 6 * NC * sizeof(uint32_t);
    }
    const int parts = env_launches(c.blocks, p.launches);
    if (PF != 0 && parts <= 1 && knobs().pf != 0) {  // each block pulls a later block's inputs into L2
        auto* kern = step_kernel<6, PERIODIC, CELL, VAR, NC, GXC, GYC, SPL, PF, EVR>;
        static int pf_lds = -1, pf_res = 0;  // per instantiation (the LDS size is fixed by NC, GXC, GYC)
        if (pf_lds != (int)c.lds) {
            pf_res = resident_blocks(reinterpret_cast<const void*>(kern), c.T, c.lds);
            pf_lds = (int)c.lds;
        }
        Params q = p;
        // one block generation ahead (two measured flat at config 5, round 4)
        q.pf_ahead = (pf_res > 0 && c.blocks > pf_res) ? pf_res : 0;
        hipLaunchKernelGGL(kern, dim3(c.blocks), dim3(c.T), c.lds, s, q);
        return true;
    }
    if (parts <= 1) {
        hipLaunchKernelGGL((step_kernel<6, PERIODIC, CELL, VAR, NC, GXC, GYC, SPL, 0, EVR>), dim3(c.blocks), dim3(c.T),
                           c.lds, s, p);
        return true;
    }
    // the step as `parts` back-to-back launches over consecutive env ranges (same results: envs are independent)
    const int per = (c.blocks + parts - 1) / parts;
    Params q = p;
    for (int b0 = 0; b0 < c.blocks; b0 += per) {
        q.env0 = b0 * c.G;
        hipLaunchKernelGGL((step_kernel<6, PERIODIC, CELL, VAR, NC, GXC, GYC, SPL, 0, EVR>), dim3(min(per, c.blocks - b0)),
                           dim3(c.T), c.lds, s, q);
    }
    return true;
}

template <int L>
void launch_step_L(const Cfg& c, const Params& p, hipStream_t s) {
    if constexpr (L == 6) {
        if (launch_spec<FLOCK_VARIANT_V2, 256, true, true, 42, 6, 1, 1>(c, p, s)) return;  // config 3 (+ L2 pull)
        if (launch_spec<FLOCK_VARIANT_V2, 1024, true, true, 85, 12, 1, 3, true>(c, p, s)) return;  // config 5 (+ L2 pull, late)
        // config 4: no pull (the config-5 pull + non-temporal streams measured 0.1954-0.1959 against 0.1929-0.1937 ms
        // per step, the kinematics pull 0.1952; profiles/r05/c4pf/). The even-row layout (EVR) in configs 4 and 5
        // only: 0.1929-0.1936 -> 0.1890-0.1907 and 0.7535-0.7570 -> 0.7393-0.7417 ms per step, config 3 0.0809-0.0815
        // -> 0.0820-0.0823 (profiles/r05/evenrows/)
        if (launch_spec<FLOCK_VARIANT_UW_DISCRETE, 512, false, true, 64, 8, 1, 0, true>(c, p, s)) return;  // config 4
        // config 2: the candidate scan split over 4 lanes per agent (2 lanes with the memory roll on one lane group:
        // 0.0096 against 0.0094-0.0096 ms per step; 8 lanes 0.0100; profiles/r05/c2spl/)
        if (launch_spec<FLOCK_VARIANT_UW, 64, false, false, 0, 0, 4>(c, p, s)) return;  // config 2
    }
    if (p.cells) {
        if (p.periodic)
            hipLaunchKernelGGL((step_kernel<L, true, true>), dim3(c.blocks), dim3(c.T), c.lds, s, p);
        else
            hipLaunchKernelGGL((step_kernel<L, false, true>), dim3(c.blocks), dim3(c.T), c.lds, s, p);
    } else {
        if (p.periodic)
            hipLaunchKernelGGL((step_kernel<L, true, false>), dim3(c.blocks), dim3(c.T), c.lds, s, p);
        else
            hipLaunchKernelGGL((step_kernel<L, false, false>), dim3(c.blocks), dim3(c.T), c.lds, s, p);
    }
}

template <int L>
void launch_reset_L(const Cfg& c, const Params& p, hipStream_t s) {
    hipLaunchKernelGGL((reset_kernel<L>), dim3(c.blocks), dim3(c.T), c.lds, s, p);
}

int dispatch(Params& p, hipStream_t s, bool reset) {
    if (p.E == 0) return FLOCK_OK;
    if (p.periodic) p.normalize = 0;  // the periodic kNN never normalises (gym_flock_v2.py:135-151)
    // normalize_distance runs on the generic full-scan instantiations (a runtime flag there; launch_spec declines)
    p.cells = (reset || knobs().no_cells || p.normalize) ? 0 : cell_grid(p.N, p.variant, &p.gx, &p.gy);
    if (p.cells) {
        p.ecap = ext_cap(p.N, p.gy, false);  // the generic instantiations: no row sentinels
        p.cwx = p.box / (float)p.gx;
        p.cwy = p.box / (float)p.gy;
        p.inv_cwx = (float)p.gx / p.box;
        p.inv_cwy = (float)p.gy / p.box;
        p.cell_eps = p.box * 1e-5f;
        p.r_lim = fminf(0.999f * p.cwy, (float)(kRg - 1) * p.cwx);  // kRows rows, kRg - 1 columns each side
        if (!(p.box > 0.0f)) p.cells = 0;
    }
    const Cfg c = make_cfg(p.E, p.N, reset, p.cells, p.gx, p.gy);
    p.G = c.G;
    p.S = c.S;
    p.P = c.P;
    p.ib = ceil_log2(p.N);
    if (p.ib < 1) p.ib = 1;
#define FLOCK_CASE(LL)                                   \
    case LL:                                             \
        if (reset)                                       \
            launch_reset_L<LL>(c, p, s);                 \
        else                                             \
            launch_step_L<LL>(c, p, s);                  \
        break;
    const int L = (p.k + 2 <= 12) ? p.k + 2 : 17;
    switch (L) {
        FLOCK_CASE(3)
        FLOCK_CASE(4)
        FLOCK_CASE(5)
        FLOCK_CASE(6)
        FLOCK_CASE(7)
        FLOCK_CASE(8)
        FLOCK_CASE(9)
        FLOCK_CASE(10)
        FLOCK_CASE(11)
        FLOCK_CASE(12)
        FLOCK_CASE(17)
        default:
            return fail(FLOCK_E_LIMIT, "unsupported k");
    }
#undef FLOCK_CASE
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FLOCK_E_LAUNCH, hipGetErrorString(e));
    return FLOCK_OK;
}

Params base(int E, int N, int k, float box) {
    Params p;
    memset(&p, 0, sizeof(p));
    p.E = E;
    p.N = N;
    p.k = k;
    p.box = box;
    p.clamp = 1;
    return p;
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
// C ABI

void flock_sc_diag_no_spec(bool v);       // flock_sc.hip
void flock_sc_diag_event_system(bool v);  // flock_sc.hip
void flock_sc_diag_free_events(bool v);   // flock_sc.hip

extern "C" {

int flock_abi_version(void) { return FLOCK_ABI_VERSION; }

int flock_set_diag(const char* name, int value) {
    if (!name) return fail(FLOCK_E_NULL, "flock_set_diag: NULL name");
    Knobs& k = knobs_mut();
    if (!strcmp(name, "env_launches"))
        k.env_launches = value;
    else if (!strcmp(name, "no_spec"))
        k.no_spec = value != 0;
    else if (!strcmp(name, "no_split"))
        k.no_split = value != 0;
    else if (!strcmp(name, "no_cells"))
        k.no_cells = value != 0;
    else if (!strcmp(name, "pf"))
        k.pf = value;
    else if (!strcmp(name, "rollout_spl") && (value == 2 || value == 4))
        k.rollout_spl = value;
    else if (!strcmp(name, "sc_no_spec"))
        flock_sc_diag_no_spec(value != 0);
    else if (!strcmp(name, "sc_event_system_scope"))
        flock_sc_diag_event_system(value != 0);
    else if (!strcmp(name, "sc_free_events"))
        flock_sc_diag_free_events(value != 0);
    else
        return fail(FLOCK_E_ARG, "flock_set_diag: unknown knob");
    return FLOCK_OK;
}

#ifdef FLOCK_PHASE_PROF
// diagnostics build only: copy out and clear the phase counters (32 x u64)
int flock_phase_read(unsigned long long* host) {
    static unsigned long long buf[64 * 32];
    if (hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_phase), sizeof(buf)) != hipSuccess) return 1;
    for (int q = 0; q < 32; ++q) {
        host[q] = 0;
        for (int s = 0; s < 64; ++s) host[q] += buf[s * 32 + q];
    }
    memset(buf, 0, sizeof(buf));
    return hipMemcpyToSymbol(HIP_SYMBOL(g_phase), buf, sizeof(buf)) != hipSuccess;
}
// diagnostics build only: per-block start / end (s_memrealtime) of the last launch (blocks < 4096)
int flock_blk_read(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_blk), sizeof(g_blk)) != hipSuccess;
}
int flock_blkph_read(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_blkph), sizeof(g_blkph)) != hipSuccess;
}
#endif

const char* flock_last_error(void) { return g_err; }

}  // extern "C"

namespace {

// ring (may be NULL): the fused replay insert; seeds (may be NULL): compact kNN search seeds
// the fused replay insert's targets (FlockRing) into the launch parameters, checked
int set_ring(Params& p, const FlockRing* ring, int E, int N, const char* who) {
    if (!ring) return FLOCK_OK;
    static thread_local char msg[160];
    auto bad = [&](int code, const char* what) {
        snprintf(msg, sizeof(msg), "%s: %s", who, what);
        return fail(code, msg);
    };
    if (E && (!ring->state || !ring->action || !ring->reward || !ring->new_state || !ring->terminal ||
              !ring->prev_obs))
        return bad(FLOCK_E_NULL, "NULL ring pointer");
    if (ring->group != 1 && ring->group != N)
        return bad(FLOCK_E_ARG, "ring group must be 1 (a row per agent) or N (a row per env)");
    if (ring->env_done && ring->group != N) return bad(FLOCK_E_ARG, "env_done needs group = N (a row per env)");
    const int64_t units = ring->group == 1 ? (int64_t)E * N : (int64_t)E;
    if (ring->skip < 0 || units - ring->skip > ring->capacity || ring->start < 0 || ring->start >= ring->capacity)
        return bad(FLOCK_E_ARG, "need skip >= 0, rows - skip <= capacity, 0 <= start < capacity");
    auto a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };  // k = 4: the observation rows move as 16 B
    if (E && p.k == 4 && !(a16(ring->state) && a16(ring->new_state) && a16(ring->prev_obs) &&
                           a16(ring->actor_state) && a16(ring->actor_new_state)))
        return bad(FLOCK_E_ARG, "k = 4 ring observation fields must be 16-B aligned");
    p.r_state = ring->state;
    p.r_action = ring->action;
    p.r_reward = ring->reward;
    p.r_new = ring->new_state;
    p.r_term = ring->terminal;
    p.r_prev = ring->prev_obs;
    p.r_cap = ring->capacity;
    p.r_start = ring->start;
    p.r_skip = ring->skip;
    p.r_astate = ring->actor_state;
    p.r_anew = ring->actor_new_state;
    p.r_group = (int)ring->group;
    p.r_done = ring->store_done;
    p.r_ids = ring->action_ids != 0;
    p.r_env_done = ring->env_done != 0;
    return FLOCK_OK;
}

int step_v2_impl(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance, float dt,
                 float v_min, float v_max, int periodic, int rigid_boundary, float* pos, float* heading,
                 const float* action, float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done,
                 uint8_t* any_done, const FlockRing* ring, uint16_t* seeds, int launches = 0, int normalize = 0) {
    int rc = check_common(E, N, k);
    if (rc) return rc;
    if (E && (!pos || !heading || !action || !vel || !dnn || !reward || !done || !any_done))
        return fail(FLOCK_E_NULL, "flock_step_v2: NULL pointer");
    Params p = base(E, N, k, box);
    if ((rc = set_ring(p, ring, E, N, "flock_step_v2_store"))) return rc;
    p.variant = FLOCK_VARIANT_V2;
    p.periodic = periodic != 0;
    p.rigid = rigid_boundary != 0;
    p.sensor_range = sensor_range;
    p.cd = collision_distance;
    p.dt = dt;
    p.v_min = v_min;
    p.v_max = v_max;
    p.pos = pos;
    p.heading = heading;
    p.action = action;
    p.vel = vel;
    p.dnn = dnn;
    p.idx = nn_idx;
    p.reward = reward;
    p.done = done;
    p.any_done = any_done;
    p.seeds = seeds;
    p.launches = launches;
    p.normalize = normalize != 0;  // Euclidean (periodic = 0, the RNN fork) only; dispatch clears it otherwise
    return dispatch(p, (hipStream_t)stream, false);
}

}  // namespace

extern "C" {

int flock_step_v2(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                  float dt, float v_min, float v_max, int periodic, int rigid_boundary, float* pos, float* heading,
                  const float* action, float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done,
                  uint8_t* any_done) {
    return step_v2_impl(stream, E, N, k, box, sensor_range, collision_distance, dt, v_min, v_max, periodic,
                        rigid_boundary, pos, heading, action, vel, dnn, nn_idx, reward, done, any_done, nullptr,
                        nullptr);
}

int flock_step_v2_store(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                        float dt, float v_min, float v_max, int periodic, int rigid_boundary, float* pos,
                        float* heading, const float* action, float* vel, float* dnn, int64_t* nn_idx, float* reward,
                        uint8_t* done, uint8_t* any_done, const FlockRing* ring) {
    if (E && !ring) return fail(FLOCK_E_NULL, "flock_step_v2_store: NULL pointer");
    return step_v2_impl(stream, E, N, k, box, sensor_range, collision_distance, dt, v_min, v_max, periodic,
                        rigid_boundary, pos, heading, action, vel, dnn, nn_idx, reward, done, any_done, ring,
                        nullptr);
}

int flock_step_v2_ext(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                      float dt, float v_min, float v_max, int periodic, int rigid_boundary, float* pos,
                      float* heading, const float* action, float* vel, float* dnn, int64_t* nn_idx, float* reward,
                      uint8_t* done, uint8_t* any_done, const FlockStepExt* ext) {
    return step_v2_impl(stream, E, N, k, box, sensor_range, collision_distance, dt, v_min, v_max, periodic,
                        rigid_boundary, pos, heading, action, vel, dnn, nn_idx, reward, done, any_done,
                        ext ? ext->ring : nullptr, ext ? ext->seeds : nullptr, ext ? ext->launches : 0,
                        ext ? ext->normalize_distance : 0);
}

int flock_step_uw_ext(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                      float dt, int rigid_boundary, float* pos, const float* heading, float* prev_heading,
                      const float* action, const float* mem_in, float* mem_out, float* vel, float* dnn,
                      int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done, const FlockStepExt* ext) {
    if (ext && ext->ring) return fail(FLOCK_E_ARG, "flock_step_uw_ext: the fused replay insert is v2 only");
    int rc = check_common(E, N, k);
    if (rc) return rc;
    if (E && (!pos || !heading || !prev_heading || !action || !mem_in || !mem_out || !vel || !dnn || !reward ||
              !done || !any_done))
        return fail(FLOCK_E_NULL, "flock_step_uw: NULL pointer");
    Params p = base(E, N, k, box);
    p.variant = FLOCK_VARIANT_UW;
    p.rigid = rigid_boundary != 0;
    p.sensor_range = sensor_range;
    p.cd = collision_distance;
    p.com_r = (float)((double)collision_distance * 4.0);  // collision_distance*4 (gym_flock_uw.py:197)
    p.seeds = ext ? ext->seeds : nullptr;
    p.launches = ext ? ext->launches : 0;
    p.normalize = ext && ext->normalize_distance;
    p.dt = dt;
    p.pos = pos;
    p.heading = const_cast<float*>(heading);
    p.prev_heading = prev_heading;
    p.action = action;
    p.mem_in = mem_in;
    p.mem_out = mem_out;
    p.vel = vel;
    p.dnn = dnn;
    p.idx = nn_idx;
    p.reward = reward;
    p.done = done;
    p.any_done = any_done;
    return dispatch(p, (hipStream_t)stream, false);
}

int flock_step_uw(void* stream, int E, int N, int k, float box, float sensor_range, float collision_distance,
                  float dt, int rigid_boundary, float* pos, const float* heading, float* prev_heading,
                  const float* action, const float* mem_in, float* mem_out, float* vel, float* dnn, int64_t* nn_idx,
                  float* reward, uint8_t* done, uint8_t* any_done) {
    return flock_step_uw_ext(stream, E, N, k, box, sensor_range, collision_distance, dt, rigid_boundary, pos, heading,
                             prev_heading, action, mem_in, mem_out, vel, dnn, nn_idx, reward, done, any_done,
                             nullptr);
}

int flock_rollout_uw(void* stream, int K, int E, int N, int k, float box, float sensor_range, float collision_distance,
                     float dt, int rigid_boundary, float* pos, const float* heading, float* prev_heading,
                     const float* actions, const float* mem_in, float* mem_out, float* vel, float* dnn,
                     int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done, float* obs_out,
                     float* reward_out, uint8_t* done_out, uint8_t* any_done_out, const FlockStepExt* ext) {
    if (ext && ext->ring) return fail(FLOCK_E_ARG, "flock_rollout_uw: the fused replay insert is v2 / uw_discrete only");
    int rc = check_common(E, N, k);
    if (rc) return rc;
    if (K < 0) return fail(FLOCK_E_ARG, "flock_rollout_uw: K must be >= 0");
    if (K == 0 || E == 0) return FLOCK_OK;
    if (!pos || !heading || !prev_heading || !actions || !mem_in || !mem_out || !vel || !dnn || !reward || !done ||
        !any_done || !obs_out || !reward_out || !done_out || !any_done_out)
        return fail(FLOCK_E_NULL, "flock_rollout_uw: NULL pointer");
    hipStream_t st = (hipStream_t)stream;
    const bool normalize = ext && ext->normalize_distance;
    const size_t EN = (size_t)E * N;
    if (N == kRollN && k == 4 && !normalize && !knobs().no_spec) {  // the one-launch kernel (config 2's shape)
        Params p = base(E, N, k, box);
        p.variant = FLOCK_VARIANT_UW;
        p.rigid = rigid_boundary != 0;
        p.sensor_range = sensor_range;
        p.cd = collision_distance;
        p.com_r = (float)((double)collision_distance * 4.0);  // collision_distance*4 (gym_flock_uw.py:197)
        p.dt = dt;
        p.pos = pos;
        p.heading = const_cast<float*>(heading);
        p.prev_heading = prev_heading;
        p.mem_in = mem_in;
        p.mem_out = mem_out;
        p.vel = vel;
        p.dnn = dnn;
        p.idx = nn_idx;
        p.reward = reward;
        p.done = done;
        p.any_done = any_done;
        if (knobs().rollout_spl == 4)
            hipLaunchKernelGGL(rollout_uw_kernel<4>, dim3(E), dim3(4 * kRollN), 0, st, p, K, actions, obs_out,
                               reward_out, done_out, any_done_out);
        else
            hipLaunchKernelGGL(rollout_uw_kernel<2>, dim3(E), dim3(2 * kRollN), 0, st, p, K, actions, obs_out,
                               reward_out, done_out, any_done_out);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? FLOCK_OK : fail(FLOCK_E_LAUNCH, hipGetErrorString(e));
    }
    // other shapes: K step launches writing the stacked outputs directly (step t's memory input is step t - 1's
    // observation), then the last step's memory / reward / done into the env buffers
    for (int s = 0; s < K; ++s) {
        const float* mi = s == 0 ? mem_in : obs_out + (size_t)(s - 1) * EN * kMem * k;
        if ((rc = flock_step_uw_ext(stream, E, N, k, box, sensor_range, collision_distance, dt, rigid_boundary, pos,
                                    heading, prev_heading, actions + (size_t)s * EN * 2, mi,
                                    obs_out + (size_t)s * EN * kMem * k, vel, dnn, nn_idx, reward_out + (size_t)s * EN,
                                    done_out + (size_t)s * EN, any_done_out + (size_t)s * E, ext)))
            return rc;
    }
    const size_t last = (size_t)(K - 1);
    if (hipMemcpyAsync(mem_out, obs_out + last * EN * kMem * k, EN * kMem * k * sizeof(float),
                       hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(reward, reward_out + last * EN, EN * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(done, done_out + last * EN, EN, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(any_done, any_done_out + last * E, E, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail(FLOCK_E_LAUNCH, "flock_rollout_uw: copy of the last step's outputs");
    return FLOCK_OK;
}

int flock_step_uw_discrete_ext(void* stream, int E, int N, int k, float box, float sensor_range,
                               float collision_distance, float dt, float v_max, int rigid_boundary, float* pos,
                               float* heading, float* prev_heading, const int64_t* action_id, const float* noise,
                               float noise_std, uint64_t seed, uint64_t rng_offset, const float* table,
                               int n_actions, float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done,
                               uint8_t* any_done, int* status, const FlockStepExt* ext) {
    int rc = check_common(E, N, k);
    if (rc) return rc;
    if (E && (!pos || !heading || !prev_heading || !action_id || !table || !vel || !dnn || !reward || !done ||
              !any_done))
        return fail(FLOCK_E_NULL, "flock_step_uw_discrete: NULL pointer");
    if (n_actions < 1) return fail(FLOCK_E_ARG, "n_actions must be >= 1");
    Params p = base(E, N, k, box);
    if ((rc = set_ring(p, ext ? ext->ring : nullptr, E, N, "flock_step_uw_discrete_ext"))) return rc;
    if (p.r_state && !p.r_ids)
        return fail(FLOCK_E_ARG, "flock_step_uw_discrete_ext: the ring stores action ids (action_ids = 1)");
    p.variant = FLOCK_VARIANT_UW_DISCRETE;
    p.rigid = rigid_boundary != 0;
    p.sensor_range = sensor_range;
    p.cd = collision_distance;
    p.dt = dt;
    p.v_max = v_max;
    p.noise_std = noise_std;
    p.seed = seed;
    p.rng_offset = rng_offset;
    p.pos = pos;
    p.heading = heading;
    p.prev_heading = prev_heading;
    p.action_id = action_id;
    p.noise = noise;
    p.table = table;
    p.n_actions = n_actions;
    p.vel = vel;
    p.dnn = dnn;
    p.idx = nn_idx;
    p.reward = reward;
    p.done = done;
    p.any_done = any_done;
    p.status = status;
    p.seeds = ext ? ext->seeds : nullptr;
    p.launches = ext ? ext->launches : 0;
    p.normalize = ext && ext->normalize_distance;
    return dispatch(p, (hipStream_t)stream, false);
}

int flock_step_uw_discrete(void* stream, int E, int N, int k, float box, float sensor_range,
                           float collision_distance, float dt, float v_max, int rigid_boundary, float* pos,
                           float* heading, float* prev_heading, const int64_t* action_id, const float* noise,
                           float noise_std, uint64_t seed, uint64_t rng_offset, const float* table, int n_actions,
                           float* vel, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done,
                           int* status) {
    return flock_step_uw_discrete_ext(stream, E, N, k, box, sensor_range, collision_distance, dt, v_max,
                                      rigid_boundary, pos, heading, prev_heading, action_id, noise, noise_std, seed,
                                      rng_offset, table, n_actions, vel, dnn, nn_idx, reward, done, any_done, status,
                                      nullptr);
}

int flock_step_flock_ext(void* stream, int E, int N, int k, float box, float collision_distance, float dt,
                         int rigid_boundary, float* pos, float* vel, const float* action, const float* mem_in,
                         float* mem_out, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done,
                         uint8_t* any_done, const FlockStepExt* ext) {
    if (ext && ext->ring) return fail(FLOCK_E_ARG, "flock_step_flock_ext: the fused replay insert is v2 only");
    int rc = check_common(E, N, k);
    if (rc) return rc;
    if (E && (!pos || !vel || !action || !mem_in || !mem_out || !dnn || !reward || !done || !any_done))
        return fail(FLOCK_E_NULL, "flock_step_flock: NULL pointer");
    Params p = base(E, N, k, box);
    p.variant = FLOCK_VARIANT_FLOCK;
    p.rigid = rigid_boundary != 0;
    p.clamp = 0;  // gym_flock.py:105: no clamp
    p.seeds = ext ? ext->seeds : nullptr;
    p.launches = ext ? ext->launches : 0;
    p.normalize = ext && ext->normalize_distance;
    p.cd = collision_distance;
    p.dt = dt;
    p.pos = pos;
    p.vel = vel;
    p.action = action;
    p.mem_in = mem_in;
    p.mem_out = mem_out;
    p.dnn = dnn;
    p.idx = nn_idx;
    p.reward = reward;
    p.done = done;
    p.any_done = any_done;
    return dispatch(p, (hipStream_t)stream, false);
}

int flock_step_flock(void* stream, int E, int N, int k, float box, float collision_distance, float dt,
                     int rigid_boundary, float* pos, float* vel, const float* action, const float* mem_in,
                     float* mem_out, float* dnn, int64_t* nn_idx, float* reward, uint8_t* done, uint8_t* any_done) {
    return flock_step_flock_ext(stream, E, N, k, box, collision_distance, dt, rigid_boundary, pos, vel, action,
                                mem_in, mem_out, dnn, nn_idx, reward, done, any_done, nullptr);
}

int flock_knn(void* stream, int E, int N, int k, float box, float sensor_range, int periodic, int clamp,
              const float* pos, float* dnn, int64_t* nn_idx) {
    int rc = check_common(E, N, k);
    if (rc) return rc;
    if (E && (!pos || !dnn)) return fail(FLOCK_E_NULL, "flock_knn: NULL pointer");
    Params p = base(E, N, k, box);
    p.variant = kSense;
    p.periodic = periodic != 0;
    p.clamp = clamp != 0;
    p.sensor_range = sensor_range;
    p.cd = 0.0f;
    p.pos = const_cast<float*>(pos);
    p.dnn = dnn;
    p.idx = nn_idx;
    return dispatch(p, (hipStream_t)stream, false);
}

int flock_reset(void* stream, int variant, int E, int N, int k, float range_lo, float range_hi, float box,
                float sensor_range, float check_distance, int rigid_boundary, int max_attempts, uint64_t seed,
                uint64_t rng_offset, const uint8_t* env_mask, float* pos, float* heading, float* prev_heading,
                float* vel, float* dnn, int64_t* nn_idx, float* mem, uint8_t* valid) {
    return flock_reset_ext(stream, variant, E, N, k, range_lo, range_hi, box, sensor_range, check_distance,
                           rigid_boundary, max_attempts, seed, rng_offset, env_mask, pos, heading, prev_heading, vel,
                           dnn, nn_idx, mem, valid, 0);
}

int flock_reset_ext(void* stream, int variant, int E, int N, int k, float range_lo, float range_hi, float box,
                    float sensor_range, float check_distance, int rigid_boundary, int max_attempts, uint64_t seed,
                    uint64_t rng_offset, const uint8_t* env_mask, float* pos, float* heading, float* prev_heading,
                    float* vel, float* dnn, int64_t* nn_idx, float* mem, uint8_t* valid, int repair_rounds) {
    return flock_reset_ext2(stream, variant, E, N, k, range_lo, range_hi, box, sensor_range, check_distance,
                            rigid_boundary, max_attempts, seed, rng_offset, env_mask, pos, heading, prev_heading, vel,
                            dnn, nn_idx, mem, valid, repair_rounds, 0);
}

int flock_reset_ext2(void* stream, int variant, int E, int N, int k, float range_lo, float range_hi, float box,
                     float sensor_range, float check_distance, int rigid_boundary, int max_attempts, uint64_t seed,
                     uint64_t rng_offset, const uint8_t* env_mask, float* pos, float* heading, float* prev_heading,
                     float* vel, float* dnn, int64_t* nn_idx, float* mem, uint8_t* valid, int repair_rounds,
                     int normalize_distance) {
    int rc = check_common(E, N, k);
    if (rc) return rc;
    if (E && (!pos || !dnn)) return fail(FLOCK_E_NULL, "flock_reset: NULL pointer");
    if (max_attempts < 1) return fail(FLOCK_E_ARG, "max_attempts must be >= 1");
    if (repair_rounds < 0) return fail(FLOCK_E_ARG, "repair_rounds must be >= 0");
    Params p = base(E, N, k, box);
    p.repair = normalize_distance ? 0 : repair_rounds;  // the repair stage works on raw distances
    p.normalize = normalize_distance != 0;
    p.variant = variant;
    p.rigid = rigid_boundary != 0;
    p.sensor_range = sensor_range;
    p.check_distance = check_distance;
    p.max_attempts = max_attempts;
    p.seed = seed;
    p.rng_offset = rng_offset;
    p.env_mask = env_mask;
    p.pos = pos;
    p.heading = heading;
    p.prev_heading = prev_heading;
    p.vel = vel;
    p.dnn = dnn;
    p.idx = nn_idx;
    p.mem_out = mem;
    p.valid = valid;
    p.clamp = (variant == FLOCK_VARIANT_FLOCK) ? 0 : 1;
    switch (variant) {  // position range and heading range per reference reset()
        case FLOCK_VARIANT_V2:  // gym_flock_v2.py:87-96
            p.range_lo = range_lo;
            p.range_hi = range_hi;
            p.head_hi = 4.71238898f;  // float(pi*1.5)
            break;
        case FLOCK_VARIANT_UW:  // gym_flock_uw.py:87-92: (r0 - r1//2) * U + r1//2, headings (0, 2pi]
            p.range_lo = range_lo;
            p.range_hi = (float)(long long)(range_hi / 2);
            p.head_hi = 6.28318548f;
            break;
        case FLOCK_VARIANT_UW_DISCRETE:  // gym_flock_uw_discrete.py:125-133: headings (0, pi/1.2]
            p.range_lo = range_lo;
            p.range_hi = range_hi;
            p.head_hi = 2.61799383f;
            break;
        case FLOCK_VARIANT_FLOCK:  // gym_flock.py:63
            p.range_lo = range_lo;
            p.range_hi = range_hi;
            p.head_hi = 0.0f;
            break;
        default:
            return fail(FLOCK_E_ARG, "unknown variant");
    }
    return dispatch(p, (hipStream_t)stream, true);
}

}  // extern "C"
