// ez_format.h — eazy wire format: constants and the token codec, shared by
// the host C-ABI (ez_encode_* / ez_decode_*) and the gfx950 kernels.
//
// Restates writer.go:49-122 (constants), writer.go:537-621 (Encoder) and
// reader.go:346-514 (Decoder).  Values are written for a 64-bit `int`
// (Go's int on the reference's 64-bit targets).
#pragma once

#include <stdint.h>

#include "../../include/eazy.h"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define EZ_HD __host__ __device__ __forceinline__
#else
#define EZ_HD static inline
#endif

namespace ez {

constexpr int kLiteral = 0x00, kCopy = 0x80, kMeta = 0x80;
constexpr int kTagMask = 0x80, kTagLenMask = 0x7f;
constexpr int kLen1 = 124, kLen2 = 125, kLen4 = 126, kLenAlt = 127;
constexpr int kOff1 = 252, kOff2 = 253, kOff4 = 254, kOffAlt = 255, kOffLong = 255;
constexpr int kMetaMagic = 0 << 3, kMetaVer = 1 << 3, kMetaReset = 2 << 3, kMetaBreak = 3 << 3;
constexpr int kMetaTagMask = 0xf8, kMetaLenMask = 0x07, kMetaLenWide = 6, kMetaLen0 = 7;
constexpr int kMinCopyChunk = 6;
constexpr int64_t kReserve = 8;
constexpr uint32_t kHashMul = 0x1e35a7bdu;

// Encoder.Tag (writer.go:537-563): writes <= 5 bytes, returns count, -1 = panic.
EZ_HD int enc_tag(uint8_t *b, int tag, int64_t l) {
    if (l < kLen1) { b[0] = (uint8_t)(tag | l); return 1; }
    l -= kLen1;
    if (l < 0x100) { b[0] = (uint8_t)(tag | kLen1); b[1] = (uint8_t)l; return 2; }
    l -= 0x100;
    if (l < 0x10000) { b[0] = (uint8_t)(tag | kLen2); b[1] = (uint8_t)l; b[2] = (uint8_t)(l >> 8); return 3; }
    l -= 0x10000;
    if (l < 0x100000000LL - kReserve) {
        b[0] = (uint8_t)(tag | kLen4);
        b[1] = (uint8_t)l; b[2] = (uint8_t)(l >> 8); b[3] = (uint8_t)(l >> 16); b[4] = (uint8_t)(l >> 24);
        return 5;
    }
    return -1;
}

// Encoder.Offset (writer.go:565-597): writes <= 6 bytes, returns count, -1 = panic.
EZ_HD int enc_offset(uint8_t *b, int64_t off, int64_t l) {
    int k = 0;
    if (off >= l) off -= l;
    else b[k++] = kOffLong;
    if (off < kOff1) { b[k++] = (uint8_t)off; return k; }
    off -= kOff1;
    if (off < 0x100) { b[k++] = kOff1; b[k++] = (uint8_t)off; return k; }
    off -= 0x100;
    if (off < 0x10000) { b[k++] = kOff2; b[k++] = (uint8_t)off; b[k++] = (uint8_t)(off >> 8); return k; }
    off -= 0x10000;
    if (off < 0x100000000LL - kReserve) {
        b[k++] = kOff4;
        b[k++] = (uint8_t)off; b[k++] = (uint8_t)(off >> 8); b[k++] = (uint8_t)(off >> 16); b[k++] = (uint8_t)(off >> 24);
        return k;
    }
    return -1;
}

// Encoder.Meta (writer.go:599-621): writes <= 8 bytes, returns count, -1 = panic.
EZ_HD int enc_meta(uint8_t *b, int64_t meta, int64_t l) {
    if (meta & ~(int64_t)kMetaTagMask) return -1;
    if (l == 0) { b[0] = kMeta; b[1] = (uint8_t)(meta | kMetaLen0); return 2; }
    if (l < kMetaLenWide && (l & (l - 1)) == 0) {
        int lg = 0;
        while ((int64_t)1 << (lg + 1) <= l) lg++;
        b[0] = kMeta; b[1] = (uint8_t)(meta | lg);
        return 2;
    }
    if (l < kOff1) { b[0] = kMeta; b[1] = (uint8_t)(meta | kMetaLenWide); b[2] = (uint8_t)l; return 3; }
    b[0] = kMeta; b[1] = (uint8_t)(meta | kMetaLenWide);
    int k = enc_offset(b + 2, l, 0);
    return k < 0 ? -1 : k + 2;
}

// Decoder.Tag (reader.go:346-392).  Returns EZ_* ; *i = st on error.
EZ_HD int dec_tag(const uint8_t *b, int64_t n, int64_t st, int *tag, int64_t *l, int64_t *i) {
    *tag = 0; *l = 0; *i = st;
    if (st >= n) return EZ_ESHORTBUF;
    int64_t j = st;
    uint32_t t0 = b[j];
    *tag = (int)(t0 & kTagMask);
    int64_t v = t0 & kTagLenMask;
    j++;
    *l = v;
    if (v == kLen1) {
        if (j + 1 > n) return EZ_ESHORTBUF;
        v = kLen1 + (int64_t)b[j];
        j++;
    } else if (v == kLen2) {
        if (j + 2 > n) return EZ_ESHORTBUF;
        v = kLen1 + 0x100 + ((int64_t)b[j] | (int64_t)b[j + 1] << 8);
        j += 2;
    } else if (v == kLen4) {
        if (j + 4 > n) return EZ_ESHORTBUF;
        v = kLen1 + 0x100 + 0x10000 +
            ((int64_t)b[j] | (int64_t)b[j + 1] << 8 | (int64_t)b[j + 2] << 16 | (int64_t)b[j + 3] << 24);
        j += 4;
    } else if (v == kLenAlt) {
        return EZ_EOVERFLOW;
    }
    *l = v;
    *i = j;
    return EZ_OK;
}

// Decoder.basicOffset (reader.go:422-472).
EZ_HD int dec_basic_offset(const uint8_t *b, int64_t n, int64_t st, int64_t *off, int64_t *i) {
    *off = 0; *i = st;
    if (st == n) return EZ_ESHORTBUF;
    int64_t j = st;
    int64_t v = b[j];
    j++;
    *off = v;
    if (v == kOff1) {
        if (j + 1 > n) return EZ_ESHORTBUF;
        v = kOff1 + (int64_t)b[j];
        j++;
    } else if (v == kOff2) {
        if (j + 2 > n) return EZ_ESHORTBUF;
        v = kOff1 + 0x100 + ((int64_t)b[j] | (int64_t)b[j + 1] << 8);
        j += 2;
    } else if (v == kOff4) {
        if (j + 4 > n) return EZ_ESHORTBUF;
        v = kOff1 + 0x100 + 0x10000 +
            ((int64_t)b[j] | (int64_t)b[j + 1] << 8 | (int64_t)b[j + 2] << 16 | (int64_t)b[j + 3] << 24);
        j += 4;
    } else if (v == kOffAlt) {
        return EZ_EOVERFLOW;
    }
    *off = v;
    *i = j;
    return EZ_OK;
}

// Decoder.Offset (reader.go:394-420).
EZ_HD int dec_offset(const uint8_t *b, int64_t n, int64_t st, int64_t l, int64_t *off, int64_t *i) {
    *off = 0; *i = st;
    if (st == n) return EZ_ESHORTBUF;
    int64_t j = st;
    bool lng = b[j] == kOffLong;
    if (lng) j++;
    int64_t k;
    int e = dec_basic_offset(b, n, j, off, &k);
    if (e) return e;
    if (!lng) *off += l;
    *i = k;
    return EZ_OK;
}

// Decoder.Meta (reader.go:474-514).
EZ_HD int dec_meta(const uint8_t *b, int64_t n, int64_t st, int64_t *meta, int64_t *l, int64_t *i) {
    *meta = 0; *l = 0; *i = st;
    if (st == n) return EZ_ESHORTBUF;
    int64_t j = st;
    int64_t m = b[j];
    j++;
    *meta = m & kMetaTagMask;
    int64_t v = m & kMetaLenMask;
    if (v == kMetaLen0) { *i = j; return EZ_OK; }
    if (v < kMetaLenWide) { *l = (int64_t)1 << v; *i = j; return EZ_OK; }
    if (j == n) return EZ_ESHORTBUF;
    v = b[j];
    j++;
    if (v < kOff1) { *l = v; *i = j; return EZ_OK; }
    int64_t k;
    int e = dec_basic_offset(b, n, j - 1, &v, &k);
    *l = v;
    if (e) return e;
    *i = k;
    return EZ_OK;
}

// Upper bound of one Write's output (header included).  Derivation
// (DESIGN.md §Bound): a copy token never costs more than it covers, every
// literal costs its bytes + a tag of <= 5 bytes, and there are at most
// n/6 + n/24 + 1 literal tags (copies are >= 6 bytes, cut literals >= 24).
EZ_HD uint64_t compress_bound(uint64_t n) { return n + (n >> 2) + 32; }

}  // namespace ez
