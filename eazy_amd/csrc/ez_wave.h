// ez_wave.h — wave64 helpers and byte views shared by the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ez {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ uint64_t wballot(bool p) { return (uint64_t)__ballot(p); }

__device__ __forceinline__ int32_t rl32(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

__device__ __forceinline__ int64_t rl64(int64_t v, int l) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// inclusive prefix sum over the wave's 64 lanes by DPP (row_shr 1/2/4/8 within each row of 16,
// then row_bcast 15/31 across the rows): VALU only, no LDS round trip per step as ds_bpermute has
__device__ __forceinline__ int32_t wscan_add(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 into rows 2, 3
    return v;
}
// lane l gets v of lane l-1, lane 0 gets `first` (DPP wave_shr:1)
__device__ __forceinline__ int32_t wshr1(int32_t v, int32_t first) {
    return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false);
}

// first set lane of a ballot mask (mask != 0)
__device__ __forceinline__ int ffs64(uint64_t m) { return (int)__builtin_ctzll(m); }

// 4 bytes at byte address a (any alignment) of a dword-aligned word array
__device__ __forceinline__ uint32_t words_u32(const uint32_t *w, uint64_t a) {
    const uint32_t w0 = w[a >> 2];
    const uint32_t w1 = w[(a >> 2) + 1];
    return __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(a & 3));
}

// Token-header accumulator: up to 16 bytes built in two 64-bit words
// (uniform values), written to memory by lanes 0..n-1.
struct Hdr {
    uint64_t lo = 0, hi = 0;
    int n = 0;
    __device__ __forceinline__ void put(uint32_t b) {
        const uint64_t v = (uint64_t)(b & 0xff);
        if (n < 8) lo |= v << (8 * n);
        else hi |= v << (8 * (n - 8));
        n++;
    }
    __device__ __forceinline__ uint8_t byte(int k) const {
        return (uint8_t)((k < 8 ? lo : hi) >> (8 * (k & 7)));
    }
};

// Encoder.Tag (writer.go:537-563) into a header; false = panic.
__device__ __forceinline__ bool hdr_tag(Hdr &h, int tag, int64_t l) {
    if (l < 124) { h.put(tag | (int)l); return true; }
    l -= 124;
    if (l < 0x100) { h.put(tag | 124); h.put((uint32_t)l); return true; }
    l -= 0x100;
    if (l < 0x10000) { h.put(tag | 125); h.put((uint32_t)l); h.put((uint32_t)(l >> 8)); return true; }
    l -= 0x10000;
    if (l < 0x100000000LL - 8) {
        h.put(tag | 126);
        h.put((uint32_t)l); h.put((uint32_t)(l >> 8)); h.put((uint32_t)(l >> 16)); h.put((uint32_t)(l >> 24));
        return true;
    }
    return false;
}

// Encoder.Offset (writer.go:565-597) into a header; false = panic.
__device__ __forceinline__ bool hdr_offset(Hdr &h, int64_t off, int64_t l) {
    if (off >= l) off -= l;
    else h.put(255);
    if (off < 252) { h.put((uint32_t)off); return true; }
    off -= 252;
    if (off < 0x100) { h.put(252); h.put((uint32_t)off); return true; }
    off -= 0x100;
    if (off < 0x10000) { h.put(253); h.put((uint32_t)off); h.put((uint32_t)(off >> 8)); return true; }
    off -= 0x10000;
    if (off < 0x100000000LL - 8) {
        h.put(254);
        h.put((uint32_t)off); h.put((uint32_t)(off >> 8)); h.put((uint32_t)(off >> 16)); h.put((uint32_t)(off >> 24));
        return true;
    }
    return false;
}

}  // namespace ez
