// ez_k2_ring.h — the LDS output ring of the wave-per-stream decoders (K2w, K2t): output
// position p lives at ring slot p & (R - 1); the ring is laid out as [16-byte guard][R bytes]
// [16-byte mirror of the first 16][16-byte guard] so that every 16-byte read at any slot is one
// contiguous LDS access.
#pragma once

#include "ez_bytes.h"

namespace ez {

typedef uint64_t __attribute__((aligned(1))) u64_ua;

// 16 bytes of position p from a ring of R bytes
template <int32_t R>
__device__ __forceinline__ V16 rld(const uint8_t *ring, int32_t p) {
    const uint8_t *q = ring + (p & (R - 1));
    return V16{*(const u64_ua *)q, *(const u64_ua *)(q + 8)};
}
// 16 bytes of position p into the ring: a write that wraps is written again R bytes lower (its
// head lands in the front guard), one into the first 16 bytes again R bytes higher (its tail
// lands in the back guard) -- whole 16-byte LDS writes only
template <int32_t R>
__device__ __forceinline__ void rst(uint8_t *ring, int32_t p, V16 v) {
    const int32_t r = p & (R - 1);
    *(u64_ua *)(ring + r) = v.lo;
    *(u64_ua *)(ring + r + 8) = v.hi;
    if (r > R - 16 || r < 16) {
        const int32_t r2 = r < 16 ? r + R : r - R;
        *(u64_ua *)(ring + r2) = v.lo;
        *(u64_ua *)(ring + r2 + 8) = v.hi;
    }
}
// the first n bytes (1..16) of v at d
__device__ __forceinline__ void put_n(uint8_t *d, V16 v, uint32_t n) {
    if (n >= 16) {
        *(u64_ua *)d = v.lo;
        *(u64_ua *)(d + 8) = v.hi;
    } else {
        put_small(d, v, n);
    }
}
// n bytes (1..16) of position p into the ring, exact (pieces of one instruction never overlap)
template <int32_t R>
__device__ __forceinline__ void rput(uint8_t *ring, int32_t p, V16 v, uint32_t n) {
    const int32_t r = p & (R - 1);
    put_n(ring + r, v, n);
    if (r + (int32_t)n > R || r < 16) put_n(ring + (r < 16 ? r + R : r - R), v, n);
}

// Long literals (C4: a whole fp32 bucket is one literal) are not moved by the stream's one wave:
// the decoder records them (DeferLit) and kd_copy moves their bytes with the whole chip afterwards.
// A far copy reading from such a literal before kd_copy has run reads its bytes from the input.
constexpr int32_t kDeferMin = 16384;  // literals this long are deferred

// the 16 output bytes at sq (< the ring's reach) from HBM, or from the input where they lie in one
// of the nd deferred literals (defs: {output position, input position, length} each, in LDS)
__device__ __forceinline__ V16 far16_def(const uint8_t *out, int32_t cap, const uint8_t *b, int32_t sq, int nd, const int32_t *defs) {
    V16 v{0, 0};
    for (int t = 0; t < 16; t++) {
        const int32_t y = sq + t;
        uint64_t c = y >= 0 ? out[y] : 0;
        for (int k = 0; k < nd; k++)
            if (y >= defs[3 * k] && y < defs[3 * k] + defs[3 * k + 2]) c = b[defs[3 * k + 1] + (y - defs[3 * k])];
        if (t < 8) v.lo |= c << (8 * t);
        else v.hi |= c << (8 * (t - 8));
    }
    return v;
}
__device__ __forceinline__ V16 far16(const uint8_t *out, int32_t cap, const uint8_t *b, int32_t sq, int nd, const int32_t *defs) {
    bool hit = false;
    for (int k = 0; k < nd; k++)
        if (sq < defs[3 * k] + defs[3 * k + 2] && sq + 16 > defs[3 * k]) hit = true;
    if (!hit) return ld_clamped16(out + sq, out, out + cap);
    return far16_def(out, cap, b, sq, nd, defs);
}

}  // namespace ez
