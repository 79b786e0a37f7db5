// Microbenchmark: issue throughput of the env step kernel's VALU opcodes on gfx950, in cycles per wave64
// instruction per SIMD, at 8 waves per SIMD (2048 blocks x 256 threads: the config-3 kernel's occupancy) and at
// 1 wave per SIMD (256 blocks). Each lane runs 8 independent chains of the instruction, so the numbers are issue
// throughput, not latency. The opcodes are the ones the config-3 step_kernel's ISA uses most (static histogram in
// profiles/ubench_valu.json); "class" is the SQ_INSTS_VALU_* counter the opcode is counted under.
//
// Build and run (writes JSON to stdout):
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu tools/ubench_valu.hip && tools/ubench_valu > out.json
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096

// one kernel per opcode: 8 independent chains per lane, ITERS x 8 instructions per wave
#define U32_OP(NAME, ASM)                                                                          \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned* out, unsigned seed) {                \
        unsigned a[8];                                                                             \
        for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + i);                               \
        const unsigned b = seed ^ 0x1234u, c = seed ^ 0x9876u;                                     \
        for (int it = 0; it < ITERS; ++it) {                                                       \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(a[i]) : "v"(b), "v"(c) : "vcc"); \
        }                                                                                          \
        unsigned acc = 0;                                                                          \
        for (int i = 0; i < 8; ++i) acc += a[i];                                                   \
        out[blockIdx.x * 256 + threadIdx.x] = acc;                                                 \
    }
#define F32_OP(NAME, ASM)                                                                          \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned* out, unsigned seed) {                \
        float f[8];                                                                                \
        for (int i = 0; i < 8; ++i) f[i] = (float)(seed * (threadIdx.x + i)) * 1e-9f;              \
        const float b = 0.999f, c = 1e-7f;                                                         \
        for (int it = 0; it < ITERS; ++it) {                                                       \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(f[i]) : "v"(b), "v"(c) : "vcc"); \
        }                                                                                          \
        unsigned acc = 0;                                                                          \
        for (int i = 0; i < 8; ++i) acc += __float_as_uint(f[i]);                                  \
        out[blockIdx.x * 256 + threadIdx.x] = acc;                                                 \
    }
// v_cndmask_b32 with its lane mask in an SGPR pair (reading VCC right after the previous statement's VCC clobber
// makes the compiler pad every instruction with hazard s_nops)
#define SEL_OP(NAME, ASM)                                                                          \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned* out, unsigned seed) {                \
        unsigned a[8];                                                                             \
        for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + i);                               \
        const unsigned b = seed ^ 0x1234u;                                                         \
        const uint64_t m = 0x5555aaaa3333ccccull ^ seed;                                           \
        for (int it = 0; it < ITERS; ++it) {                                                       \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(a[i]) : "v"(b), "s"(m)); \
        }                                                                                          \
        unsigned acc = 0;                                                                          \
        for (int i = 0; i < 8; ++i) acc += a[i];                                                   \
        out[blockIdx.x * 256 + threadIdx.x] = acc;                                                 \
    }
// compares writing an SGPR pair (the e64 form), one result register per chain
#define CMP_OP(NAME, ASM)                                                                          \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned* out, unsigned seed) {                \
        float f[8];                                                                                \
        uint64_t r[8];                                                                             \
        for (int i = 0; i < 8; ++i) f[i] = (float)(seed * (threadIdx.x + i)) * 1e-9f;              \
        const float b = 0.999f;                                                                    \
        for (int it = 0; it < ITERS; ++it) {                                                       \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "=s"(r[i]) : "v"(f[i]), "v"(b)); \
        }                                                                                          \
        unsigned acc = 0;                                                                          \
        for (int i = 0; i < 8; ++i) acc += (unsigned)r[i];                                         \
        out[blockIdx.x * 256 + threadIdx.x] = acc;                                                 \
    }
#define U64_OP(NAME, ASM)                                                                          \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned* out, unsigned seed) {                \
        uint64_t a[8];                                                                             \
        for (int i = 0; i < 8; ++i) a[i] = (uint64_t)seed * (threadIdx.x + i) * 0x10001ull;        \
        const uint64_t b = seed ^ 0x123456789ull;                                                  \
        const unsigned c = seed ^ 0x9876u, d = seed ^ 0x5555u;                                     \
        for (int it = 0; it < ITERS; ++it) {                                                       \
            _Pragma("unroll") for (int i = 0; i < 8; ++i)                                          \
                asm volatile(ASM : "+v"(a[i]) : "v"(b), "v"(c), "v"(d) : "vcc");                   \
        }                                                                                          \
        unsigned acc = 0;                                                                          \
        for (int i = 0; i < 8; ++i) acc += (unsigned)a[i] + (unsigned)(a[i] >> 32);                \
        out[blockIdx.x * 256 + threadIdx.x] = acc;                                                 \
    }

// class: the SQ_INSTS_VALU_* counter family (gfx950 counter_defs.yaml) the opcode falls under
#define OPS(X)                                                                                     \
    X(F32, v_add_f32, "ADD_F32", "v_add_f32 %0, %0, %1")                                           \
    X(F32, v_sub_f32, "ADD_F32", "v_sub_f32 %0, %1, %0")                                           \
    X(F32, v_sub_f32_abs, "ADD_F32", "v_sub_f32_e64 %0, %1, |%0|")                                 \
    X(F32, v_mul_f32, "MUL_F32", "v_mul_f32 %0, %0, %1")                                           \
    X(F32, v_fma_f32, "FMA_F32", "v_fma_f32 %0, %0, %1, %2")                                       \
    X(F32, v_min_f32, "other", "v_min_f32 %0, %0, %1")                                             \
    X(F32, v_max3_f32, "other", "v_max3_f32 %0, %0, %1, %2")                                       \
    X(F32, v_med3_f32, "other", "v_med3_f32 %0, %0, %1, %2")                                       \
    X(F32, v_floor_f32, "other", "v_floor_f32 %0, %0")                                             \
    X(F32, v_sqrt_f32, "TRANS_F32", "v_sqrt_f32 %0, %0")                                           \
    X(F32, v_sin_f32, "TRANS_F32", "v_sin_f32 %0, %0")                                             \
    X(F32, v_cmp_lt_f32, "other", "v_cmp_lt_f32 vcc, %0, %1")                                      \
    X(F32, v_cvt_i32_f32, "CVT", "v_cvt_i32_f32 %0, %0")                                           \
    X(SEL, v_cndmask_b32, "INT32", "v_cndmask_b32 %0, %0, %1, %2")                                 \
    X(CMP, v_cmp_lt_f32_e64, "other", "v_cmp_lt_f32_e64 %0, %1, %2")                               \
    X(F32, v_max_f32, "other", "v_max_f32 %0, %0, %1")                                             \
    X(F32, v_subrev_f32, "ADD_F32", "v_subrev_f32 %0, %0, %1")                                     \
    X(F32, v_fmac_f32, "FMA_F32", "v_fmac_f32 %0, %1, %2")                                         \
    X(U32, v_or_b32, "INT32", "v_or_b32 %0, %0, %1")                                               \
    X(U32, v_xor_b32, "INT32", "v_xor_b32 %0, %0, %1")                                             \
    X(U32, v_sub_u32, "INT32", "v_sub_u32 %0, %0, %1")                                             \
    X(U32, v_lshlrev_b32, "INT32", "v_lshlrev_b32 %0, 1, %0")                                      \
    X(U32, v_lshrrev_b32, "INT32", "v_lshrrev_b32 %0, 1, %0")                                      \
    X(U32, v_max_u32, "INT32", "v_max_u32 %0, %0, %1")                                             \
    X(U32, v_bfi_b32, "INT32", "v_bfi_b32 %0, %1, %0, %2")                                         \
    X(U32, v_bfe_u32, "INT32", "v_bfe_u32 %0, %0, 3, 9")                                           \
    X(U32, v_lshl_or_b32, "INT32", "v_lshl_or_b32 %0, %0, 1, %1")                                  \
    X(U32, v_alignbit_b32, "INT32", "v_alignbit_b32 %0, %0, %1, 7")                                \
    X(U32, v_mul_hi_u32, "INT32", "v_mul_hi_u32 %0, %0, %1")                                       \
    X(U32, v_cvt_f32_u32, "CVT", "v_cvt_f32_u32 %0, %0")                                           \
    X(U32, v_mov_b32, "INT32", "v_mov_b32 %0, %1")                                                 \
    X(U32, v_med3_u32, "INT32", "v_med3_u32 %0, %0, %1, %2")                                       \
    X(U32, v_min_u32, "INT32", "v_min_u32 %0, %0, %1")                                             \
    X(U32, v_min_i32, "INT32", "v_min_i32 %0, %0, %1")                                             \
    X(U32, v_add_u32, "INT32", "v_add_u32 %0, %0, %1")                                             \
    X(U32, v_add3_u32, "INT32", "v_add3_u32 %0, %0, %1, %2")                                       \
    X(U32, v_lshl_add_u32, "INT32", "v_lshl_add_u32 %0, %0, 2, %1")                                \
    X(U32, v_and_b32, "INT32", "v_and_b32 %0, %0, %1")                                             \
    X(U32, v_and_or_b32, "INT32", "v_and_or_b32 %0, %0, %1, %2")                                   \
    X(U32, v_bfrev_b32, "INT32", "v_bfrev_b32 %0, %0")                                             \
    X(U32, v_cmp_lt_u32, "INT32", "v_cmp_lt_u32 vcc, %0, %1")                                      \
    X(U32, v_mul_u32_u24, "INT32", "v_mul_u32_u24 %0, %0, %1")                                     \
    X(U32, v_mul_lo_u32, "INT32", "v_mul_lo_u32 %0, %0, %1")                                       \
    X(U64, v_pk_add_f32, "ADD_F32", "v_pk_add_f32 %0, %0, %1")                                     \
    X(U64, v_pk_mul_f32, "MUL_F32", "v_pk_mul_f32 %0, %0, %1")                                     \
    X(U64, v_pk_fma_f32, "FMA_F32", "v_pk_fma_f32 %0, %0, %1, %0")                                 \
    X(U64, v_mov_b64, "INT64", "v_mov_b64 %0, %1")                                                 \
    X(U64, v_lshl_add_u64, "INT64", "v_lshl_add_u64 %0, %0, 2, %1")                                \
    X(U64, v_lshlrev_b64, "INT64", "v_lshlrev_b64 %0, 2, %0")                                      \
    X(U64, v_mad_u64_u32, "INT64", "v_mad_u64_u32 %0, vcc, %2, %3, %0")

#define DEF(T, NAME, CLS, ASM) T##_OP(NAME, ASM)
OPS(DEF)

struct Op {
    const char* name;
    const char* cls;
    void (*fn)(unsigned*, unsigned);
};
#define ENTRY(T, NAME, CLS, ASM) {#NAME, CLS, k_##NAME},
static const Op ops[] = {OPS(ENTRY)};

int main() {
    unsigned* out;
    hipMalloc(&out, 2048 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int dev = 0, cus = 0, clk_khz = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
    const double simds = 4.0 * cus, clk = 2.4e9;
    printf("{\"device_cus\": %d, \"clock_attr_khz\": %d, \"clock_assumed_hz\": %.4g, \"iters\": %d,\n", cus, clk_khz,
           clk, ITERS);
    printf(" \"note\": \"cycles per wave64 instruction per SIMD = elapsed x %.3g Hz / (waves x %d x 8 / %d SIMDs); "
           "8 independent chains per lane; best of 3 launches\",\n \"ops\": [\n",
           clk, ITERS, (int)simds);
    const int n = sizeof(ops) / sizeof(ops[0]);
    for (int o = 0; o < n; ++o) {
        double cyc[2];
        const int blocks_of[2] = {2048, 256};  // 8 and 1 waves per SIMD on 256 CUs
        for (int w = 0; w < 2; ++w) {
            const int blocks = blocks_of[w];
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                hipEventRecord(e0);
                hipLaunchKernelGGL(ops[o].fn, dim3(blocks), dim3(256), 0, 0, out, 7u + rep);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep) best = ms < best ? ms : best;  // rep 0 warms up
            }
            const double winstr = (double)blocks * 4 * ITERS * 8 / simds;  // wave-instructions per SIMD
            cyc[w] = best * 1e-3 * clk / winstr;
        }
        printf("  {\"op\": \"%s\", \"class\": \"%s\", \"cyc_8waves\": %.3f, \"cyc_1wave\": %.3f}%s\n", ops[o].name,
               ops[o].cls, cyc[0], cyc[1], o + 1 < n ? "," : "");
    }
    printf(" ]}\n");
    hipFree(out);
    return 0;
}
