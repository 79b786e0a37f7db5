// Microbenchmark: issue throughput (cycles per wave64 instruction per SIMD) of the env kernel's inner-loop
// instruction types on gfx950. Each lane runs 8 independent chains; 2048 blocks x 256 threads (8 waves/SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 8192

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
    unsigned a[8];
    float f[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = seed * (threadIdx.x + i);
        f[i] = (float)a[i] * 1e-9f;
    }
    const unsigned b = seed ^ 0x1234u, c = seed ^ 0x9876u;
    const float fb = 0.999f, fc = 1e-7f;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
            if (OP == 1) asm volatile("v_min_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
            if (OP == 2) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fb), "v"(fc));
            if (OP == 3) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
            if (OP == 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fb), "v"(fc));
            if (OP == 5) asm volatile("v_sub_f32_e64 %0, %1, |%0|" : "+v"(f[i]) : "v"(fb));
            if (OP == 6) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if (OP == 7) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 8) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 9) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 10) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 11) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 12) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if (OP == 13) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if (OP == 14) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            if (OP == 15) asm volatile("v_mov_b32 %0, %1" : "+v"(a[i]) : "v"(b));
            if (OP == 16) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
        }
    }
    unsigned acc = 0;
    for (int i = 0; i < 8; ++i) acc += a[i] + __float_as_uint(f[i]);
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void kpk(unsigned* out, unsigned seed) {
    float2 f[8];
    for (int i = 0; i < 8; ++i) f[i] = make_float2(seed * 1e-9f + i, seed * 2e-9f);
    const float2 s = make_float2(0.999f, 1.001f);
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            double d = *reinterpret_cast<double*>(&f[i]);
            const double sd = *reinterpret_cast<const double*>(&s);
            asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(d) : "v"(sd));
            f[i] = *reinterpret_cast<float2*>(&d);
        }
    }
    unsigned acc = 0;
    for (int i = 0; i < 8; ++i) acc += __float_as_uint(f[i].x) + __float_as_uint(f[i].y);
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    unsigned* out;
    const int blocks = 2048;
    hipMalloc(&out, blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"v_add_f32", "v_min_f32", "v_med3_f32", "v_mul_f32", "v_fma_f32", "v_sub_f32_e64|abs|", "v_med3_u32", "v_min_u32", "v_min_i32", "v_add_u32", "v_and_b32", "v_or_b32", "v_and_or_b32", "v_bfi_b32", "v_or3_b32", "v_mov_b32", "v_cndmask_b32", "v_pk_mul_f32"};
    for (int op = 0; op < 18; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            switch (op) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 6: hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 7: hipLaunchKernelGGL(k<7>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 8: hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 9: hipLaunchKernelGGL(k<9>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 10: hipLaunchKernelGGL(k<10>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 11: hipLaunchKernelGGL(k<11>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 12: hipLaunchKernelGGL(k<12>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 13: hipLaunchKernelGGL(k<13>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 14: hipLaunchKernelGGL(k<14>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 15: hipLaunchKernelGGL(k<15>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 16: hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
                case 17: hipLaunchKernelGGL(kpk, dim3(blocks), dim3(256), 0, 0, out, 7u); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // wave-instructions per SIMD: blocks*4 waves * ITERS*8 / 1024 SIMDs
            const double winstr = (double)blocks * 4 * ITERS * 8 / 1024.0;
            if (rep) printf("%-20s %8.3f ms  %.2f cycles/wave-instr/SIMD @2.4GHz\n", names[op], ms,
                            ms * 1e-3 * 2.4e9 / winstr);
        }
    }
    return 0;
}
