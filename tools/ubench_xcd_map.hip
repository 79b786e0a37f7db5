// Two facts the learner round's XCD-aware mapping depends on (verdict r4 item 4):
// 1. is the block -> XCD dealing the same in every launch (block b on XCD (b + c) mod 8 with one c per launch; does
//    c change between launches)?  whoami<<<>>> records s_getreg(HW_REG_XCC_ID) per block, five launches in a row.
// 2. what a read sees and costs across kernel boundaries after another XCD wrote the lines: k0 XCD Y reads a 1 MiB
//    buffer (its L2 holds the old lines), k1 XCD X writes new values (plain stores), k2 XCD Y reads it again (stale
//    words counted, time per block), k3 XCD X reads it (the writer's own L2).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_xcd_map.hip -o tools/ubench_xcd_map
#include <hip/hip_runtime.h>

#include <stdio.h>

__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xF;
}

__global__ void whoami(int* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

constexpr int kBlocks = 512, kPerXcd = 64;
constexpr size_t kFloats = (1u << 20) / 4;
constexpr int kSlice4 = (int)(kFloats / 4 / kPerXcd);  // float4 per block: 1024

__global__ __launch_bounds__(256) void rd(const float4* buf, int y, float want, unsigned* bad,
                                          unsigned long long* t) {
    if (xcc_id() != y) return;
    const int b = blockIdx.x / 8;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = buf[(size_t)b * kSlice4 + threadIdx.x + 256 * u];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    unsigned n = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) n += (v[u].x != want) + (v[u].y != want) + (v[u].z != want) + (v[u].w != want);
    if (n) atomicAdd(bad, n);
    if (threadIdx.x == 0) t[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(256) void wr(float4* buf, int x, float val) {
    if (xcc_id() != x) return;
    const int b = blockIdx.x / 8;
#pragma unroll
    for (int u = 0; u < 4; ++u) buf[(size_t)b * kSlice4 + threadIdx.x + 256 * u] = make_float4(val, val, val, val);
}

double mean_us(const unsigned long long* t) {
    double s = 0;
    int n = 0;
    for (int b = 0; b < kBlocks; ++b)
        if (t[b]) s += t[b], ++n;
    return n ? s / n / 100.0 : 0.0;
}

int main() {
    int *map, hmap[5][kBlocks];
    if (hipMalloc(&map, sizeof(hmap))) return 1;
    for (int l = 0; l < 5; ++l) whoami<<<kBlocks, 64>>>(map + l * kBlocks);
    if (hipMemcpy(hmap, map, sizeof(hmap), hipMemcpyDeviceToHost)) return 2;
    for (int l = 0; l < 5; ++l) {
        const int c = ((hmap[l][0] - 0) % 8 + 8) % 8;
        int rr = 0, per[8] = {0};
        for (int b = 0; b < kBlocks; ++b) {
            rr += hmap[l][b] == (b + c) % 8;
            per[hmap[l][b] & 7]++;
        }
        printf("launch %d: block 0 on XCD %d; blocks on XCD (b + %d) mod 8: %d / %d; per XCD:", l, hmap[l][0], c, rr,
               kBlocks);
        for (int x = 0; x < 8; ++x) printf(" %d", per[x]);
        printf("\n");
    }
    float4* buf;
    unsigned* bad;
    unsigned long long *t, ht[kBlocks];
    if (hipMalloc(&buf, kFloats * 4) || hipMalloc(&bad, 4) || hipMalloc(&t, kBlocks * 8)) return 1;
    for (int rep = 0; rep < 3; ++rep) {
        const float v0 = 1.0f + 2 * rep, v1 = v0 + 1.0f;
        const int X = 2, Y = 5;
        wr<<<kBlocks, 256>>>(buf, Y, v0);  // old values, written and cached on Y
        hipMemset(bad, 0, 4);
        hipMemset(t, 0, kBlocks * 8);
        rd<<<kBlocks, 256>>>(buf, Y, v0, bad, t);  // k0: Y reads (L2 of Y holds the lines)
        if (hipDeviceSynchronize()) return 3;
        hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
        const double t0 = mean_us(ht);
        wr<<<kBlocks, 256>>>(buf, X, v1);  // k1: X writes new values
        hipMemset(t, 0, kBlocks * 8);
        rd<<<kBlocks, 256>>>(buf, Y, v1, bad, t);  // k2: Y reads again
        if (hipDeviceSynchronize()) return 4;
        unsigned hbad = 0;
        hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost);
        hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
        const double t2 = mean_us(ht);
        hipMemset(t, 0, kBlocks * 8);
        rd<<<kBlocks, 256>>>(buf, X, v1, bad, t);  // k3: the writer's XCD reads
        if (hipDeviceSynchronize()) return 5;
        hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
        const double t3 = mean_us(ht);
        unsigned hbad2 = 0;
        hipMemcpy(&hbad2, bad, 4, hipMemcpyDeviceToHost);
        printf("rep %d: Y reads its own lines %.3f us; after X rewrote them: Y reads %.3f us (stale words %u), X reads "
               "%.3f us (stale words %u)\n", rep, t0, t2, hbad, t3, hbad2 - hbad);
    }
    // 3. lines WRITTEN by XCD X in the previous launch, read by X in the next (the learner round's producer ->
    //    consumer hand-off): k0 X writes (plain stores), k1 X reads; against k1' X re-reading lines it only read
    for (int rep = 0; rep < 3; ++rep) {
        const int X = 4;
        const float v0 = 100.0f + rep;
        wr<<<kBlocks, 256>>>(buf, X, v0);
        hipMemset(bad, 0, 4);
        hipMemset(t, 0, kBlocks * 8);
        rd<<<kBlocks, 256>>>(buf, X, v0, bad, t);  // X reads the lines it wrote one launch earlier
        if (hipDeviceSynchronize()) return 6;
        hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
        const double tw = mean_us(ht);
        hipMemset(t, 0, kBlocks * 8);
        rd<<<kBlocks, 256>>>(buf, X, v0, bad, t);  // and again (lines it read one launch earlier)
        if (hipDeviceSynchronize()) return 7;
        hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
        const double tr = mean_us(ht);
        hipMemset(t, 0, kBlocks * 8);
        rd<<<kBlocks, 256>>>(buf, (X + 3) & 7, v0, bad, t);  // another XCD reads them
        if (hipDeviceSynchronize()) return 8;
        hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
        const double to = mean_us(ht);
        unsigned hb = 0;
        hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
        printf("rep %d: X reads the lines it wrote last launch %.3f us; lines it read last launch %.3f us; another XCD "
               "%.3f us (stale words %u)\n", rep, tw, tr, to, hb);
    }
    return 0;
}
