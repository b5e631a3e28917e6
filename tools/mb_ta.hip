// mb_ta.hip — vector-memory (TA/TD/L1) cost of the load shapes the K1 parse
// uses, on an L2-resident buffer: wave64 loads per CU per cycle for
//   0 scattered dwordx4 at random byte offsets (the candidate loads)
//   1 scattered dwordx4 at random 16-byte-aligned offsets
//   2 dwordx4 at base + lane (16 overlapping unaligned windows per row: the window loads)
//   3 dword at base + 4*lane (coalesced, aligned)
//   4 scattered dwordx2 at random byte offsets
//   5 scattered dword at random byte offsets
//   6 scattered dwordx4 at random 4-byte-aligned offsets
//   7 dwordx4 at base + 16*lane (coalesced, aligned)
// usage: mb_ta [iters]; prints ns per wave-load and loads/CU/us per pattern.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint4 __attribute__((aligned(1))) u4u;
typedef uint2 __attribute__((aligned(1))) u2u;
typedef uint32_t __attribute__((aligned(1))) u1u;

__device__ __forceinline__ uint32_t rnd(uint32_t &s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

template <int P>
__global__ __launch_bounds__(64) void k(const uint8_t *buf0, uint32_t mask, int iters, uint32_t *out) {
    const uint32_t lane = threadIdx.x;
    // L1 mode (mask < 64 KiB): every CU's waves share one small region (L1-resident after the first pass)
    const uint8_t *buf = mask < 65536 ? buf0 + (size_t)(blockIdx.x % 256) * 65536 : buf0;
    uint32_t s = 0x9e3779b9u * (blockIdx.x * 64 + lane + 1);
    uint32_t acc = 0;
    for (int it = 0; it < iters; it++) {
        uint32_t r = rnd(s) & mask;
        const uint32_t base = __builtin_amdgcn_readfirstlane(r) & ~63u;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t q = (r + 977u * u) & mask;
            if (P == 0) { const uint4 v = *(const u4u *)(buf + q); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
            if (P == 1) { const uint4 v = *(const uint4 *)(buf + (q & ~15u)); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
            if (P == 2) { const uint4 v = *(const u4u *)(buf + ((base + 128 * u + lane) & mask)); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
            if (P == 3) { acc ^= *(const uint32_t *)(buf + ((base + 256 * u + 4 * lane) & mask)); }
            if (P == 4) { const uint2 v = *(const u2u *)(buf + q); acc ^= v.x ^ v.y; }
            if (P == 5) { acc ^= *(const u1u *)(buf + q); }
            if (P == 6) { const uint4 v = *(const u4u *)(buf + (q & ~3u)); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
            if (P == 7) { const uint4 v = *(const uint4 *)(buf + ((base + 1024 * u + 16 * lane) & mask)); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int P>
float run(const uint8_t *buf, uint32_t mask, int iters, uint32_t *out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k<P>, dim3(blocks), dim3(64), 0, 0, buf, mask, 4, out);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<P>, dim3(blocks), dim3(64), 0, 0, buf, mask, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const size_t bytes = 16u << 20;  // L2-resident per XCD after the first touch: 8 MiB spread over 8 XCDs
    uint8_t *buf;
    uint32_t *out;
    hipMalloc(&buf, bytes + 64);
    hipMalloc(&out, 64);
    hipMemset(buf, 1, bytes + 64);
    const int blocks = 256 * 20;  // 20 waves per CU, as the K1 parse
    const char *names[] = {"scatter dwordx4 byte-aligned", "scatter dwordx4 16B-aligned", "window dwordx4 base+lane",
                           "coalesced dword", "scatter dwordx2 byte-aligned", "scatter dword byte-aligned",
                           "scatter dwordx4 4B-aligned", "coalesced dwordx4"};
    float t[8];
    for (int mode = 0; mode < 2; mode++) {
    const uint32_t m = mode == 0 ? (uint32_t)(bytes - 1) : 16383u;  // 8 MiB (L2) or 16 KiB per CU (L1)
    printf(mode == 0 ? "-- 8 MiB buffer (L1 misses, L2 hits)\n" : "-- 16 KiB per CU (L1 hits)\n");
    t[0] = run<0>(buf, m, iters, out, blocks);
    t[1] = run<1>(buf, m, iters, out, blocks);
    t[2] = run<2>(buf, m, iters, out, blocks);
    t[3] = run<3>(buf, m, iters, out, blocks);
    t[4] = run<4>(buf, m, iters, out, blocks);
    t[5] = run<5>(buf, m, iters, out, blocks);
    t[6] = run<6>(buf, m, iters, out, blocks);
    t[7] = run<7>(buf, m, iters, out, blocks);
    for (int p = 0; p < 8; p++) {
        const double loads_per_cu = (double)blocks / 256 * iters * 4;
        printf("%d %-32s %8.3f ms  %7.1f wave-loads/CU/us  %6.1f ns per wave-load per CU\n", p, names[p], t[p],
               loads_per_cu / (t[p] * 1e3), t[p] * 1e6 / loads_per_cu);
    }
    }
    return 0;
}
