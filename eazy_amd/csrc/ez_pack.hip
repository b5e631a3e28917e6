// ez_pack.hip — K3: pack per-stream compressed slots densely.
//
// Replaces the reference's per-Write output buffer hand-off (w.b + flush,
// writer.go:379-401) for a batch: an exclusive scan of the per-stream sizes
// gives each stream's offset in one dense output buffer, then one wave per
// stream gathers its slot there.
//   scan1: per 1024-stream tile sum            (tile_sums)
//   scan2: one workgroup scans the tile sums   (tile_base)
//   scan3: per-tile exclusive scan + tile_base (packed_off)
//   gather: wave per stream, dword-wide where alignment allows
#include "ez_internal.h"
#include "ez_wave.h"

namespace ez {
namespace {

constexpr int kTile = 1024;
constexpr int kThreads = 256;
constexpr int kPer = kTile / kThreads;

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *sh, uint64_t *total) {
    // wave-level inclusive scan with shuffles, then across the 4 waves
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    uint64_t x = v;
    for (int d = 1; d < kWave; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, kWave);
        if (lane >= d) x += y;
    }
    if (lane == kWave - 1) sh[w] = x;
    __syncthreads();
    uint64_t wbase = 0, tot = 0;
    for (int k = 0; k < kThreads / kWave; k++) {
        if (k < w) wbase += sh[k];
        tot += sh[k];
    }
    __syncthreads();
    *total = tot;
    return wbase + x - v;
}

__global__ __launch_bounds__(kThreads) void k3_scan1(const uint64_t *sizes, uint64_t count, uint64_t *tile_sums) {
    __shared__ uint64_t sh[kThreads / kWave];
    const uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kPer;
    uint64_t v = 0;
    for (int k = 0; k < kPer; k++)
        if (base + k < count) v += sizes[base + k];
    uint64_t tot;
    block_exclusive_scan(v, sh, &tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kThreads) void k3_scan2(uint64_t *tile_sums, uint64_t ntiles) {
    __shared__ uint64_t sh[kThreads / kWave];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < ntiles; b += kThreads) {
        const uint64_t t = b + threadIdx.x;
        const uint64_t v = t < ntiles ? tile_sums[t] : 0;
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(v, sh, &tot);
        if (t < ntiles) tile_sums[t] = carry + ex;
        carry += tot;
    }
}

__global__ __launch_bounds__(kThreads) void k3_scan3(const uint64_t *sizes, uint64_t count, const uint64_t *tile_base,
                                                     uint64_t *packed_off) {
    __shared__ uint64_t sh[kThreads / kWave];
    const uint64_t base = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * kPer;
    uint64_t v[kPer];
    uint64_t sum = 0;
    for (int k = 0; k < kPer; k++) {
        v[k] = base + k < count ? sizes[base + k] : 0;
        sum += v[k];
    }
    uint64_t tot;
    uint64_t run = tile_base[blockIdx.x] + block_exclusive_scan(sum, sh, &tot);
    for (int k = 0; k < kPer; k++) {
        if (base + k < count) packed_off[base + k] = run;
        if (base + k + 1 == count) packed_off[count] = run + v[k];
        run += v[k];
    }
}

typedef uint4 __attribute__((aligned(4))) uint4_a4;  // 16 bytes at a dword-aligned address

__global__ __launch_bounds__(256) void k3_gather(const uint8_t *slots, const uint64_t *slot_off, const uint64_t *sizes,
                                                 uint64_t count, uint8_t *packed, const uint64_t *packed_off,
                                                 uint32_t split) {
    const int lane = lane_id();
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / kWave);
    const uint64_t work = count * split;
    for (uint64_t v = (uint64_t)blockIdx.x * (blockDim.x / kWave) + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
         v < work; v += waves) {
        // virtual wave v = stream s, part j of split: part j moves dwords
        // j*64 .. j*64+63 of every split*64-dword round; part 0 also the
        // head and tail bytes
        const uint64_t s = v / split;
        const uint32_t j = (uint32_t)(v - s * split);
        const uint8_t *src = slots + slot_off[s];
        uint8_t *dst = packed + packed_off[s];
        const uint64_t n = sizes[s];
        // head bytes until dst is 4-aligned, then whole dwords built from
        // two aligned source dwords, then the tail bytes
        const uint64_t head = ((4 - ((uintptr_t)dst & 3)) & 3) < n ? ((4 - ((uintptr_t)dst & 3)) & 3) : n;
        if (j == 0 && (uint64_t)lane < head) dst[lane] = src[lane];
        const uint64_t body = (n - head) / 4;
        const uint8_t *s2 = src + head;
        const uint32_t r = (uint32_t)((uintptr_t)s2 & 3);
        const uint32_t *sw = (const uint32_t *)(s2 - r);
        uint32_t *dw = (uint32_t *)(dst + head);
        // last source word index that holds a byte of this stream
        const uint64_t wlast = (r + (n - head) + 3) / 4 - 1;
        // 16 bytes per lane and step (four dwords built from five source dwords; the source is read
        // at dword granularity, never past its last word), the last < 4 dwords one at a time
        const uint64_t body4 = body / 4;
        for (uint64_t k = (uint64_t)j * kWave + lane; k < body4; k += (uint64_t)split * kWave) {
            const uint64_t q = 4 * k;
            const uint4 a = *(const uint4_a4 *)(sw + q);
            const uint32_t e = sw[q + 4 <= wlast ? q + 4 : wlast];
            *(uint4_a4 *)(dw + q) = make_uint4(__builtin_amdgcn_alignbyte(a.y, a.x, r), __builtin_amdgcn_alignbyte(a.z, a.y, r),
                                              __builtin_amdgcn_alignbyte(a.w, a.z, r), __builtin_amdgcn_alignbyte(e, a.w, r));
        }
        if (j == 0) {
            const uint64_t k = 4 * body4 + (uint64_t)lane;
            if (k < body) {
                const uint32_t w0 = sw[k];
                const uint32_t w1 = sw[k + 1 <= wlast ? k + 1 : wlast];
                dw[k] = __builtin_amdgcn_alignbyte(w1, w0, r);
            }
        }
        const uint64_t t0 = head + body * 4;
        if (j == 0 && (uint64_t)lane < n - t0) dst[t0 + lane] = src[t0 + lane];
    }
}

}  // namespace

size_t pack_workspace(uint64_t count) {
    const uint64_t tiles = (count + kTile - 1) / kTile;
    return (size_t)(tiles ? tiles : 1) * sizeof(uint64_t);
}

hipError_t launch_pack(const uint8_t *slots, const uint64_t *slot_off, const uint64_t *sizes, uint64_t count,
                       uint8_t *packed, uint64_t *packed_off, void *workspace, hipStream_t st) {
    if (count == 0) return hipMemsetAsync(packed_off, 0, sizeof(uint64_t), st);
    const uint64_t tiles = (count + kTile - 1) / kTile;
    uint64_t *tile_sums = (uint64_t *)workspace;
    hipLaunchKernelGGL(k3_scan1, dim3((unsigned)tiles), dim3(kThreads), 0, st, sizes, count, tile_sums);
    hipLaunchKernelGGL(k3_scan2, dim3(1), dim3(kThreads), 0, st, tile_sums, tiles);
    hipLaunchKernelGGL(k3_scan3, dim3((unsigned)tiles), dim3(kThreads), 0, st, sizes, count, tile_sums, packed_off);
    // few (long) streams: several waves per stream so the gather fills the
    // chip (64 streams of 4 MiB were 64 waves, 7.3 ms); 16 Ki waves in all
    uint32_t split = 1;
    if (count < 16384) split = (uint32_t)(16384 / count);
    if (split > 1024) split = 1024;
    uint64_t blocks = (count * split + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k3_gather, dim3((unsigned)blocks), dim3(256), 0, st, slots, slot_off, sizes, count, packed,
                       packed_off, split);
    return hipGetLastError();
}

}  // namespace ez
