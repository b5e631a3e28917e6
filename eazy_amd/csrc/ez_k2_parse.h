// ez_k2_parse.h — the token parse shared by the batch decoders K2r (lane per
// stream) and K2w (wave per stream): one step of Reader.read's readTag for the
// common case, from the 16 input bytes at the parse position.
//
// readTag reader.go:218-270 (padding :221-224), continueMetaTag :272-325 for
// the header metas (magic, version 0, MetaReset before any output) and breaks,
// Decoder.Tag :346-392 and Decoder.Offset :394-420.  Everything else — an
// error of any kind, an unsupported or wide meta, a reset after output, a
// length over BlockSizeLimit, a token past the output slot or the input, a
// 4-byte length or offset of 2^30 or more — is "hand over": the exact decoder
// (ez_decompress.hip) recomputes the stream from scratch.
#pragma once

#include "ez_bytes.h"
#include "ez_format.h"

namespace ez {

struct K2Tok {
    int32_t adv;    // input bytes the step consumes
    int32_t L;      // token length (0: padding or a meta)
    int32_t j;      // literal: its bytes start at i + j
    uint32_t D;     // copy distance (0: zero region)
    bool cp;        // copy (else literal)
    uint32_t marg;  // kScanReset: log2 of the window
};

enum { kParseSkip = 0, kParseToken = 1, kParseHandOver = -1 };
enum { kScanReset = 2 };  // k2_scan only: a MetaReset, valid only before any output
// k2_scan with partial (a Reader's buffered input, which may end inside a token): the step at i runs
// past the input's end.  t.adv = 0: its header (or meta) is incomplete, nothing of it is consumed
// (readTag / continueMetaTag return ErrShortBuffer at i, reader.go:218-325); else a literal whose
// header is whole and whose body runs past the end (read copies the bytes there are, :166-168)
enum { kScanTail = 3 };

// The checks that do not depend on the decoder's state, for a step at input position
// i: returns kParseSkip (padding, break, version, magic), kScanReset, kParseToken or
// kParseHandOver.  h = input bytes i .. i+15 (zeros past the batch); nb = stream
// bytes; lim32 = BlockSizeLimit clamped to 32 bits (0x7fffffff: none), limit = the 64-bit one
__host__ __device__ __forceinline__ int k2_scan(V16 h, int32_t i, int32_t nb, int32_t lim32, int64_t limit, K2Tok &t,
                                                bool partial = false) {
    const uint64_t lo = h.lo;
    const uint32_t t0 = (uint32_t)lo & 0xff, l7 = t0 & 0x7f;
    t.L = 0;
    t.j = 0;
    t.D = 0;
    t.cp = false;
    t.marg = 0;
    if (t0 == 0) {  // padding, a run of zero bytes at once
        t.adv = lo ? (int32_t)(__builtin_ctzll(lo) >> 3) : (h.hi ? 8 + (int32_t)(__builtin_ctzll(h.hi) >> 3) : 16);
        if (partial && i + t.adv > nb) t.adv = nb - i;  // (readTag skips the zeros up to the input's end)
        return kParseSkip;
    }
    if (t0 == 0x80) {
        // meta: header metas and breaks only
        const uint32_t mb = (uint32_t)(lo >> 8) & 0xff, mt = mb & 0xf8, ml = mb & 7;
        const int32_t mln = ml == 7 ? 0 : (1 << ml);
        const uint32_t marg = (uint32_t)(lo >> 16) & 0xff;
        const bool m_brk = mt == kMetaBreak && mln == 0;
        const bool m_rst = mt == kMetaReset && mln == 1 && marg <= 32 && (limit == 0 || (1ll << marg) <= limit);
        const bool m_ver = mt == kMetaVer && mln == 1 && marg == 0;
        const bool m_mag = mt == kMetaMagic && mln == 4 && (uint32_t)(lo >> 16) == 0x797a6165u;
        if (partial && ml != 6 && i + 2 + mln > nb) {
            t.adv = 0;
            return kScanTail;
        }
        if (ml == 6 || i + 2 + mln > nb || !(m_brk || m_rst || m_ver || m_mag)) return kParseHandOver;
        t.adv = 2 + mln;
        t.marg = marg;
        return m_rst ? kScanReset : kParseSkip;
    }
    // Tag and Offset in 32 bits, branch-free: a length byte l7 >= 124 is followed by
    // 1 << (l7 - 124) little-endian bytes over the base 124 / 380 / 65916, an offset
    // byte o >= 252 by 1 << (o - 252) bytes over 252 / 508 / 66044
    const uint32_t lx = (uint32_t)(lo >> 8);
    const bool lw = l7 >= 124;
    const uint32_t ln = lw ? 1u << (l7 - 124 < 2 ? l7 - 124 : 2) : 0u;  // extra length bytes (1, 2, 4; 127 is bad)
    const uint32_t lmask = ln == 4 ? 0x3fffffffu : (1u << (8 * ln)) - 1;  // (4 bytes >= 2^30 are bad)
    const int32_t L = lw ? 124 + (l7 >= 125 ? 256 : 0) + (l7 >= 126 ? 65536 : 0) + (int32_t)(lx & lmask) : (int32_t)l7;
    const uint32_t j = 1 + ln;
    const bool cp = (t0 & 0x80) != 0;
    const bool lng = ((uint32_t)(lo >> (8 * j)) & 0xff) == 0xff;  // byte j (j <= 5, in lo)
    const uint32_t jo = j + (lng ? 1 : 0);
    const uint64_t y = (lo >> (8 * jo)) | (h.hi << (64 - 8 * jo));  // bytes from the offset on (1 <= jo <= 6)
    const uint32_t o = (uint32_t)y & 0xff, ox = (uint32_t)(y >> 8);
    const bool ow = o >= 252;
    const uint32_t on = ow ? 1u << (o - 252 < 2 ? o - 252 : 2) : 0u;
    const uint32_t omask = on == 4 ? 0x3fffffffu : (1u << (8 * on)) - 1;
    const int32_t D0 = ow ? 252 + (o >= 253 ? 256 : 0) + (o >= 254 ? 65536 : 0) + (int32_t)(ox & omask) : (int32_t)o;
    const uint32_t k = 1 + on;
    const uint32_t D = lng ? (uint32_t)D0 : (uint32_t)D0 + (uint32_t)L;  // < 2^32
    const int32_t adv = cp ? (int32_t)(jo + k) : (int32_t)j + L;
    if (partial && (uint32_t)i + (cp ? (uint32_t)adv : j) > (uint32_t)nb) {  // the header runs past the input
        t.adv = 0;
        return kScanTail;
    }
    const bool past = (uint32_t)i + (uint32_t)adv > (uint32_t)nb;
    const bool bad = l7 == 127 || (l7 == 126 && lx >= (1u << 30)) || (cp && o >= 254 && (o == 255 || ox >= (1u << 30))) || L > lim32 ||
                     (past && !partial) || (cp && D >= (1u << 30));
    if (bad) return kParseHandOver;
    if (past) {  // (partial) a literal whose body runs past the input
        t.adv = adv;
        t.L = L;
        t.j = (int32_t)j;
        return kScanTail;
    }
    t.adv = adv;
    t.L = L;
    t.j = (int32_t)j;
    t.D = cp ? D : 0;
    t.cp = cp;
    return kParseToken;
}

// The common token forms from the header's first 8 bytes, in 32-bit arithmetic without
// branches: a 1-byte tag (length 1..123; not padding, not a meta) and, for a copy, a 1..3-byte
// offset (plain, Off1 or Off2, reader.go:422-472) after an optional long prefix (:394-420).
// Returns a value < 0 for another form (k2_parse decides); D is the copy distance, adv the
// input bytes taken.  (Conditions as sign bits of one integer: compares would each become a
// lane mask and every && a scalar instruction.)
__host__ __device__ __forceinline__ int32_t fast_tok(uint64_t lo, int32_t &L, int32_t &adv, uint32_t &D, bool &cp) {
    const uint32_t w0 = (uint32_t)lo;
    const uint32_t l7 = w0 & 0x7f;
    cp = (w0 & 0x80) != 0;
    L = (int32_t)l7;
    const bool lng = (w0 & 0xff00) == 0xff00;
    const uint32_t y = (uint32_t)(lo >> (lng ? 16 : 8));  // the offset's bytes
    const uint32_t o = y & 0xff;
    const bool w = o >= 252, w2 = o == 253;
    const uint32_t ext = w2 ? 256 + ((y >> 8) & 0xffff) : (y >> 8) & 0xff;
    const uint32_t D0 = w ? 252 + ext : o;
    D = lng ? D0 : D0 + l7;
    adv = cp ? 2 + (int32_t)lng + (int32_t)w + (int32_t)w2 : 1 + L;
    return (L - 1) | (122 - (L - 1)) | (cp ? 253 - (int32_t)o : 0);
}

// the checks on the decoder's state: output position pos in a slot of cap bytes and
// bsl = log2 of the window after MetaReset (-1: none yet; updated here)
__host__ __device__ __forceinline__ int k2_check(int r, const K2Tok &t, int32_t pos, int32_t cap, int32_t &bsl) {
    if (r == kScanReset) {
        if (pos != 0) return kParseHandOver;
        bsl = (int32_t)t.marg;
        return kParseSkip;
    }
    if (r == kParseToken &&
        (bsl < 0 || (uint32_t)pos + (uint32_t)t.L > (uint32_t)cap || (t.cp && bsl < 30 && t.D > (1u << bsl))))
        return kParseHandOver;
    return r;
}

// one step at input position i with the decoder at output position pos
__host__ __device__ __forceinline__ int k2_parse(V16 h, int32_t i, int32_t nb, int32_t pos, int32_t cap, int32_t lim32, int64_t limit,
                                                 int32_t &bsl, K2Tok &t) {
    return k2_check(k2_scan(h, i, nb, lim32, limit, t), t, pos, cap, bsl);
}

}  // namespace ez
