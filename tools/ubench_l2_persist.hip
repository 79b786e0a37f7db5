// Does a line a kernel pulled into its XCD's L2 survive the kernel boundary? (verdict r4 item 4: map the producer and
// consumer blocks of consecutive learner launches to the same XCD so that operands are L2 hits.)
// touch<<<>>> : the blocks that find themselves on XCD X read a 2 MiB buffer (plain loads; it fits one XCD's 4 MiB L2).
// probe<<<>>> : the next launch, same stream: the blocks on XCD Y read the same buffer again, each timing its slice
//               (s_memrealtime, 100 MHz) with all of its loads in flight.
// Cases: Y == X (the lines would be L2 hits if L2 kept them), Y != X (cross-XCD: MALL or HBM), and "cold" (before
// the probe a 512 MiB sweep evicts the MALL too). Also probe -> probe inside ONE launch is the L2-hit reference (a
// second pass over the slice by the same block).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_l2_persist.hip -o tools/ubench_l2_persist
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xF;
}

constexpr int kBlocks = 512;       // 64 per XCD (blocks are dealt round-robin over the 8 XCDs)
constexpr int kPerXcd = 64;
constexpr size_t kBytes = 2u << 20;  // 2 MiB
constexpr int kSlice = (int)(kBytes / 16 / kPerXcd);  // float4 per block slice: 2048

__global__ __launch_bounds__(256) void touch(const float4* buf, int x, float* sink) {
    if (xcc_id() != x) return;
    // the slice of this block among the XCD's blocks: blockIdx.x / 8 (round-robin dealing; placement only for speed)
    const int b = blockIdx.x / 8;
    float4 acc = make_float4(0, 0, 0, 0);
    for (int i = threadIdx.x; i < kSlice; i += 256) {
        const float4 v = buf[(size_t)b * kSlice + i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (acc.x == 1234.5f) sink[blockIdx.x] = acc.y + acc.z + acc.w;
}

// two timed passes over the slice in one launch: pass 0 (whatever the caches hold), pass 1 (the same block's lines:
// L2 hits at least)
__global__ __launch_bounds__(256) void probe(const float4* buf, int y, unsigned long long* t, float* sink) {
    if (xcc_id() != y) return;
    const int b = blockIdx.x / 8;
    float acc = 0.0f;
    for (int pass = 0; pass < 2; ++pass) {
        __syncthreads();
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = buf[(size_t)b * kSlice + threadIdx.x + 256 * u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) t[(size_t)blockIdx.x * 2 + pass] = t1 - t0;
    }
    if (acc == 1234.5f) sink[blockIdx.x] = acc;
}

__global__ void sweep(float4* big, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) big[i].x += 1.0f;
}

int main() {
    float4 *buf, *big;
    float* sink;
    unsigned long long* t;
    const size_t nbig = (512u << 20) / 16;
    if (hipMalloc(&buf, kBytes) || hipMalloc(&big, nbig * 16) || hipMalloc(&sink, kBlocks * 4) ||
        hipMalloc(&t, kBlocks * 2 * 8))
        return 1;
    hipMemset(buf, 0, kBytes);
    hipMemset(big, 0, nbig * 16);
    unsigned long long ht[kBlocks * 2];
    const char* names[3] = {"same XCD (Y == X)", "other XCD (Y != X)", "cold (MALL swept)"};
    for (int rep = 0; rep < 3; ++rep)
        for (int c = 0; c < 3; ++c) {
            const int x = 3, y = c == 1 ? 6 : 3;
            hipMemset(t, 0, kBlocks * 2 * 8);
            sweep<<<4096, 256>>>(big, nbig);  // evict L2 and MALL
            if (c != 2) touch<<<kBlocks, 256>>>(buf, x, sink);
            probe<<<kBlocks, 256>>>(buf, y, t, sink);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
            double s0 = 0, s1 = 0;
            int n = 0;
            for (int b = 0; b < kBlocks; ++b)
                if (ht[2 * b]) {
                    s0 += ht[2 * b];
                    s1 += ht[2 * b + 1];
                    ++n;
                }
            printf("rep %d %-20s blocks %3d  first pass %.3f us  second pass (same block, same launch) %.3f us\n",
                   rep, names[c], n, n ? s0 / n / 100.0 : 0.0, n ? s1 / n / 100.0 : 0.0);
        }
    return 0;
}
