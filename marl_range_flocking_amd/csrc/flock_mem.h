// flock_mem.h — memory-access flavours of the gfx950 kernels (device helpers shared by the .hip sources).
//
// Write-through (`sc1`) stores: the bytes leave the XCD's L2 at once and the line is dropped there; `sc1` loads bypass
// the CU's L1 (served by L2). Together with an `sc1` flag store issued after every storing wave's `s_waitcnt
// vmcnt(0)` and a workgroup barrier, and an `sc1` poll of that flag by the consumer, they form the inter-workgroup
// hand-off of MI355X_MICROARCH.md's visibility table (row 1: one lane of the storing workgroup signals for all its
// stores; the consumer's polling wave loads after its poll matched, the other waves after a workgroup barrier; every
// store and every load of the handed-off bytes `sc1`, 4-, 8- or 16-B; hipMalloc memory).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace flock_mem {

// one global_store of the element's width per lane, `sc1` (any trivially copyable 1, 2, 4, 8 or 16-byte element)
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    typedef float f32x4_t __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
    if constexpr (sizeof(T) == 16) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(__builtin_bit_cast(f32x4_t, v)) : "memory");
    } else if constexpr (sizeof(T) == 8) {
        asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(__builtin_bit_cast(u32x2_t, v)) : "memory");
    } else if constexpr (sizeof(T) == 4) {
        asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(__builtin_bit_cast(uint32_t, v)) : "memory");
    } else if constexpr (sizeof(T) == 2) {
        asm volatile("global_store_short %0, %1, off sc1" ::"v"(p), "v"((uint32_t)__builtin_bit_cast(uint16_t, v))
                     : "memory");
    } else {
        static_assert(sizeof(T) == 1, "st_sc1: 1, 2, 4, 8 or 16-byte elements");
        asm volatile("global_store_byte %0, %1, off sc1" ::"v"(p), "v"((uint32_t)__builtin_bit_cast(uint8_t, v))
                     : "memory");
    }
}

// `sc1` loads (relaxed agent-scope atomic loads lower to global_load_dword / dwordx2 ... sc1)
__device__ __forceinline__ float ld_sc1(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t ld_sc1(const int64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_sc1_f2(const float2* p) {
    return __builtin_bit_cast(float2, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT));
}

// every vector-memory operation of this wave has completed (stores acknowledged): the producer side of a hand-off
__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace flock_mem
