// ez_bytes.h — 16-byte values in VGPR pairs and the byte shifts, clamped
// loads and small stores the lane-per-stream kernels (K1 lane, K2 fast) use.
// Shifts saturate to zero with selects instead of branches, so lanes that sit
// at different points of different streams run the same instructions.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ez_format.h"

namespace ez {

typedef uint4 __attribute__((aligned(1))) uint4_u;

struct V16 {
    uint64_t lo, hi;
};

EZ_HD V16 ld16v(const uint8_t *p) {
    const uint4 v = *(const uint4_u *)p;
    return {(uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z | ((uint64_t)v.w << 32)};
}
EZ_HD void st16v(uint8_t *p, V16 v) {
    *(uint4_u *)p = make_uint4((uint32_t)v.lo, (uint32_t)(v.lo >> 32), (uint32_t)v.hi, (uint32_t)(v.hi >> 32));
}
// shifts that saturate to 0 at >= 64 bits (selects, no branches)
EZ_HD uint64_t shr64(uint64_t a, uint32_t n) { return n >= 64 ? 0 : a >> (n & 63); }
EZ_HD uint64_t shl64(uint64_t a, uint32_t n) { return n >= 64 ? 0 : a << (n & 63); }
// bytes s .. s+7 of the 16 bytes (a, b), 0 <= s <= 7
EZ_HD uint64_t fun8(uint64_t a, uint64_t b, uint32_t s) {
    return (a >> (8 * s)) | shl64(b, 64 - 8 * s);
}
// v shifted towards lower addresses by k bytes (k >= 0), zeros shifted in
EZ_HD V16 shr16(V16 v, uint32_t k) {
    const uint32_t n = 8 * (k < 16 ? k : 16);
    const uint64_t lo = n < 64 ? shr64(v.lo, n) | shl64(v.hi, 64 - n) : shr64(v.hi, n - 64);
    return {lo, n < 64 ? shr64(v.hi, n) : 0};
}
// v shifted towards higher addresses by k bytes (k >= 0), zeros shifted in
EZ_HD V16 shl16(V16 v, uint32_t k) {
    const uint32_t n = 8 * (k < 16 ? k : 16);
    const uint64_t hi = n < 64 ? shl64(v.hi, n) | shr64(v.lo, 64 - n) : shl64(v.lo, n - 64);
    return {n < 64 ? shl64(v.lo, n) : 0, hi};
}
// 16 bytes at y, clamped into [lo, hi): bytes outside read as 0 (a range shorter than 16 bytes
// is read byte by byte: one 16-byte load would leave it)
EZ_HD V16 ld_clamped(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    if (hi - lo < 16) {  // a batch of < 16 bytes: a rolled byte loop (few registers)
        V16 v{0, 0};
#pragma unroll 1
        for (int t = 0; t < 16; t++) {
            const uint64_t b = (y + t >= lo && y + t < hi) ? y[t] : 0;
            if (t < 8) v.lo |= b << (8 * t);
            else v.hi |= b << (8 * (t - 8));
        }
        return v;
    }
    const uint8_t *yc = y < lo ? lo : (y > hi - 16 ? hi - 16 : y);
    const V16 v = ld16v(yc);
    const int64_t d = y - yc;
    const V16 r = shr16(v, (uint32_t)(d > 0 ? d : 0)), l = shl16(v, (uint32_t)(d < 0 ? -d : 0));
    return d >= 0 ? r : l;
}
// ld_clamped for a range known to hold at least 16 bytes (no byte loop in the code)
EZ_HD V16 ld_clamped16(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    const uint8_t *yc = y < lo ? lo : (y > hi - 16 ? hi - 16 : y);
    const V16 v = ld16v(yc);
    const int64_t d = y - yc;
    const V16 r = shr16(v, (uint32_t)(d > 0 ? d : 0)), l = shl16(v, (uint32_t)(d < 0 ? -d : 0));
    return d >= 0 ? r : l;
}
// the low `per` bytes of v (1 <= per < 16) repeated over 16 bytes
EZ_HD V16 run_pattern(V16 v, uint32_t per) {
    V16 x = per >= 8 ? V16{v.lo, per == 8 ? 0 : v.hi & ((1ull << (8 * (per - 8))) - 1)} : V16{v.lo & ((1ull << (8 * per)) - 1), 0};
#pragma unroll
    for (int t = 0; t < 4; t++) {  // span = per << t; shl16 by >= 16 bytes is a no-op (zero)
        const V16 y = shl16(x, per << t);
        x.lo |= y.lo;
        x.hi |= y.hi;
    }
    return x;
}
// k < 16 bytes of v at d: 8/4/2/1-byte stores, no loop
EZ_HD void put_small(uint8_t *d, V16 v, uint32_t k) {
    typedef uint64_t __attribute__((aligned(1))) u64_u;
    typedef uint32_t __attribute__((aligned(1))) u32_u;
    typedef uint16_t __attribute__((aligned(1))) u16_u;
    uint32_t o = 0;
    uint64_t x = v.lo;
    if (k & 8) { *(u64_u *)(d + o) = x; x = v.hi; o += 8; }
    if (k & 4) { *(u32_u *)(d + o) = (uint32_t)x; x >>= 32; o += 4; }
    if (k & 2) { *(u16_u *)(d + o) = (uint16_t)x; x >>= 16; o += 2; }
    if (k & 1) d[o] = (uint8_t)x;
}


}  // namespace ez
