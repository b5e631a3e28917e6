// ez_k1_common.h — pieces of the group-per-stream K1 kernels (ez_compress_split.hip):
// the byte view of a stream read through L1/L2, group
// ballots/broadcasts, the branch-free Encoder.Tag / Encoder.Offset
// (writer.go:537-597) and the cooperative exact match count.
#pragma once

#include "ez_format.h"
#include "ez_wave.h"
#include "ez_bytes.h"

namespace ez {
namespace k1 {

template <int G>
__device__ __forceinline__ uint32_t gball(bool p, int g) {
    return (uint32_t)(((uint64_t)__ballot(p) >> (G * g)) & (G == 32 ? 0xffffffffull : ((1ull << G) - 1)));
}
__device__ __forceinline__ int32_t bcast(int32_t v, int src_lane) { return __shfl(v, src_lane, 64); }

// byte view of a stream read straight from HBM (through L1/L2): p = the
// stream's first byte, [blo, bhi) = the batch (>= 16 bytes), loads never leave
// it; bytes before the stream start read 0 (the fresh ring),
// bytes past its end are the next stream's (every use masks or caps them).
struct GW {
    const uint8_t *p, *blo, *bhi;
    __device__ __forceinline__ uint32_t u32(int32_t y) const {
        const uint8_t *a = p + y;
        if (y >= 0 && a + 4 <= bhi) return *(const uint32_t __attribute__((aligned(1))) *)a;
        uint64_t lo, hi;
        around(y + 8, lo, hi);  // lo = bytes y .. y+7
        return (uint32_t)lo;
    }
    __device__ __forceinline__ uint32_t b(int32_t y) const { return u32(y) & 0xff; }
    __device__ __forceinline__ void around(int32_t y, uint64_t &before, uint64_t &from) const {
        const uint8_t *a = p + y - 8;
        V16 v;
        if (a >= blo && a + 16 <= bhi) {
            v = ld16v(a);  // the common case: one unaligned 16-byte load
            if (y < 8) {   // near the stream start: the bytes before it read 0
                const int32_t k = 8 - y;
                v.lo &= k >= 8 ? 0ull : ~0ull << (8 * k);
                v.hi &= k >= 16 ? 0ull : (k <= 8 ? ~0ull : ~0ull << (8 * (k - 8)));
            }
        } else {
            v = V16{0, 0};
            if (bhi - blo >= 16) {
                v = ld_clamped(a, blo, bhi);
            } else {  // a batch shorter than one 16-byte load: byte by byte
                for (int t = 0; t < 16; t++) {
                    const uint8_t *q = a + t;
                    const uint64_t x = q >= blo && q < bhi ? *q : 0;
                    if (t < 8) v.lo |= x << (8 * t);
                    else v.hi |= x << (8 * (t - 8));
                }
            }
            if (y < 8) {  // zero the bytes before the stream start
                const int32_t k = 8 - y;
                v.lo &= k >= 8 ? 0ull : ~0ull << (8 * k);
                v.hi &= k >= 16 ? 0ull : (k <= 8 ? ~0ull : ~0ull << (8 * (k - 8)));
            }
        }
        before = v.lo;
        from = v.hi;
    }
};

__device__ __forceinline__ uint64_t low_bytes(uint64_t x, int32_t k) {
    return k >= 8 ? x : (k <= 0 ? 0ull : (x & ((1ull << (8 * k)) - 1)));
}
__device__ __forceinline__ uint32_t low_bytes32(uint32_t x, int32_t k) {
    return k >= 4 ? x : (k <= 0 ? 0u : (x & (0xffffffffu >> (8 * (4 - k)))));
}
__device__ __forceinline__ int32_t ctz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_ctzll(d) >> 3) : 8; }
__device__ __forceinline__ int32_t clz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_clzll(d) >> 3) : 8; }

// Encoder.Tag (writer.go:537-563), branch-free: bytes in the low bits, count in *n
__device__ __forceinline__ uint64_t tag_bytes(uint32_t tag, int32_t l, int32_t *n) {
    const bool a = l < 124, b = l < 380, c = l < 65916;
    *n = a ? 1 : (b ? 2 : (c ? 3 : 5));
    const uint32_t b0 = tag | (uint32_t)(a ? l : (b ? 124 : (c ? 125 : 126)));
    const uint64_t v = (uint64_t)(uint32_t)(b ? l - 124 : (c ? l - 380 : l - 65916));
    return a ? (uint64_t)b0 : ((uint64_t)b0 | (v << 8));
}
// Encoder.Offset (writer.go:565-597), branch-free
__device__ __forceinline__ uint64_t off_bytes(int32_t off, int32_t l, int32_t *n) {
    const bool lg = off < l;
    const int32_t o = lg ? off : off - l;
    const bool a = o < 252, b = o < 508, c = o < 66044;
    int32_t k = a ? 1 : (b ? 2 : (c ? 3 : 5));
    const uint32_t b0 = (uint32_t)(a ? o : (b ? 252 : (c ? 253 : 254)));
    const uint64_t v = (uint64_t)(uint32_t)(b ? o - 252 : (c ? o - 508 : o - 66044));
    uint64_t r = a ? (uint64_t)b0 : ((uint64_t)b0 | (v << 8));
    if (lg) { r = 0xff | (r << 8); k += 1; }
    *n = k;
    return r;
}

// Cooperative exact match count of one group, starting `from` bytes in
// (the capped 8 already known equal), 4*G bytes per step, up to lim.
// mode: 0 zeros (a vs 0), 1 plain (a vs b), 2 ring (b's bytes from done on read 0).
// FWD: a+k vs b+k for k = from, from+1, ...; else a-1-k vs b-1-k.
template <int G, bool FWD, class SRC>
__device__ __forceinline__ int32_t gcount(const SRC &P, bool run, int g, int lj, int32_t a, int32_t b, int mode,
                                          int32_t done, int32_t from, int32_t lim) {
    int32_t res = from < lim ? from : lim;
    bool go = run && from < lim;
    int32_t base = from;
    while (__ballot(go) != 0) {
        int32_t mb = 4;
        if (go) {
            const int32_t k = base + 4 * lj;  // bytes k .. k+3 of the scan
            if (k < lim) {
                const int32_t ya = FWD ? a + k : a - k - 4, yb = FWD ? b + k : b - k - 4;
                uint32_t vb = mode == 0 ? 0u : P.u32(yb < -4 ? -4 : yb);
                if (mode == 2) {
                    // ring image: bytes from done on and before the stream start read 0 (fresh window)
                    vb = FWD ? low_bytes32(vb, done - yb) : (yb + 4 <= 0 ? 0u : (yb < 0 ? P.u32(0) << (8 * -yb) : vb));
                }
                const uint32_t d = P.u32(ya) ^ vb;
                if (d) mb = FWD ? (int32_t)(__builtin_ctz(d) >> 3) : (int32_t)(__builtin_clz(d) >> 3);
                if (mb > lim - k) mb = lim - k;
            } else {
                mb = 0;
            }
        }
        const uint32_t badm = gball<G>(go && mb < 4, g);
        const int l = badm ? __builtin_ctz(badm) : 0;
        const int32_t mbl = bcast(mb, G * g + l);
        if (go) {
            if (badm) {
                res = base + 4 * l + mbl;
                if (res > lim) res = lim;
                go = false;
            } else {
                base += 4 * G;
                if (base >= lim) { res = lim; go = false; }
            }
        }
    }
    return res;
}

}  // namespace k1
}  // namespace ez
