// flock_snap.h — the replay minibatch draw and the staging-row copy of the shared-critic learn() (device helpers shared
// by csrc/flock_sc.hip and csrc/flock_env.hip, whose step kernel can carry the snapshot in its first block).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flock_learn.h"
#include "flock_mem.h"

namespace flock_snap {

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

// the whole snapshot in one workgroup that publishes it through the device-side gate (sc_prep_snapshot_gate, and block
// 0 of a step launch that carries it: flock_step_v2_ext with FlockStepExt.snapshot): rows and agent stored `sc1`,
// every wave's stores waited for, a workgroup barrier, then one lane's agent-scope store of gate[0] = seq
// (MI355X_MICROARCH.md hand-off table, row 1; csrc/flock_mem.h)
__device__ __forceinline__ void snapshot_block(const FlockStepSnapshot& s) {
    if (threadIdx.x == 0) flock_mem::st_sc1(s.agent_out, s.agent);
    for (int r = threadIdx.x; r < s.B; r += blockDim.x)
        snapshot_row<true>(s.rows, s.seed, s.counter, nullptr, s.in_dim, s.n_actions, s.src, s.dst, s.vec, r);
    flock_mem::wait_vmem();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(s.gate, s.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace flock_snap
