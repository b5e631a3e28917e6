// ez_decompress_small.hip — K2s: batch decompression of small streams (output slots of at most
// 4 KiB: the C1 / C3 configurations) in two kernels, a parse and a move.
//
// Restates Reader.Read to EOF for NewReaderBytes (reader.go:116-216 read, readTag :218-270,
// continueMetaTag :272-325, reset :327-344, Decoder :346-514) for the common case through the
// token parse K2r uses (ez_k2_parse.h); anything else hands the stream to the exact decoder
// (ez_decompress.hip).
//
// Why two kernels.  K2r (a lane per stream, ez_decompress_ring.hip) runs Reader.read's token chain
// with every header and every far copy source a 64-address gather on the chain: at C1 the chip
// holds one such wave per SIMD and waits on those loads in every iteration.  Here the chain is
// split from the bytes:
//
//  K2p (k2_pre), a lane per stream: only the token walk — every step the parse of K2r (fast_tok,
//    k2_parse for padding, metas and long forms, every check: window, slot room, block size
//    limit) — from an LDS ring of the lane's input, refilled 128 bytes at a time one step ahead
//    (the loads of step k+1 are in flight while step k parses), so no global load sits on the
//    chain.  It writes one bit per input byte: the token starts (literal and copy tokens only),
//    in a per-stream region of the workspace, and the token count (or "hand over").
//  K2q (k2_small), 16 lanes per stream, 4 streams per wave: the whole output of a stream in LDS;
//    the bitmap becomes a list of token starts (popcount prefix sum), then rounds of 16 tokens,
//    one per lane: each lane parses its token from the 32 input bytes at its start (loaded one
//    round ahead), a prefix sum over the 16 lanes (DPP) gives every token's output position,
//    the literals are written at once, the copies in batches (every copy up to the first one
//    whose source reaches into the batch's own output; copies whose source is final at the
//    round's start run in any batch), and the finished output leaves LDS in 256-byte pieces.
//    No copy ever reads HBM: a 4 KiB stream's history is all in LDS.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"
#include "ez_k2_parse.h"

#ifndef EZ_EXP
#define EZ_EXP 0  // timing builds only: 2^21 no copies, 2^22 no literals, 2^23 no rounds, 2^24 no store
#endif

namespace ez {

namespace {

typedef uint64_t __attribute__((aligned(1))) u64_ua;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef uint16_t __attribute__((aligned(1))) u16_ua;

constexpr uint32_t kSHandOver = 0xffffffffu;

// whether c holds on any lane of the wave
__device__ __forceinline__ bool any_lane(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0; }

__device__ __forceinline__ V16 lds16(const uint8_t *p) { return V16{*(const u64_ua *)p, *(const u64_ua *)(p + 8)}; }

// 16 bytes at y of the batch [lo, hi) (hi - lo >= 16; bytes from hi on read as 0)
__device__ __forceinline__ V16 ld_batch(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    return y + 16 <= hi ? ld16v(y) : ld_clamped16(y, lo, hi);
}

// ---------------------------------------------------------------------------------------------
// K2p: the token walk, a lane per stream
// ---------------------------------------------------------------------------------------------
// The walk's chain is one LDS byte read per token: a table holds, for every input position of the
// lane's window, the input bytes a token starting there takes (SWAR over 4 positions a word, the
// common forms only: a 1-byte tag with a plain, Off1 or Off2 offset for a copy; 0 for the rest,
// which the walk parses in full) with bit 7 set when the position holds a tag (not padding).  The
// table is built when a refill lands, so the walk itself is a byte read, a mark and an add.
// Everything that needs the output position (slot room, the window, BlockSizeLimit) is checked
// by K2q, which parses every token anyway.
constexpr int kPBlock = 256;
constexpr int32_t kPRing = 256;                // input ring bytes per lane
constexpr int32_t kPStride = kPRing + 16;      // + a mirror of its first 16 bytes
constexpr int32_t kPTab = kPBlock * kPStride;  // the step tables after the rings (kPRing bytes per lane)
constexpr int32_t kPRefill = 128;              // bytes a lane's refill brings
constexpr int kPStep = 8;                      // tokens walked per refill step (<= 16 bytes each)

// the refill of one lane: 128 bytes of the stream from input position at
struct Refill {
    V16 v[kPRefill / 16];
};

__device__ __forceinline__ void refill_issue(Refill &r, const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    // (loads past the batch's last 16 bytes clamp and shift; only the batch's last stream reaches them)
    const bool edge = y + kPRefill > hi;
    if (any_lane(edge)) {
#pragma unroll
        for (int k = 0; k < kPRefill / 16; k++) r.v[k] = ld_batch(y + 16 * k, lo, hi);
    } else {
#pragma unroll
        for (int k = 0; k < kPRefill / 16; k++) r.v[k] = ld16v(y + 16 * k);
    }
}

__device__ __forceinline__ uint32_t fanout(uint32_t f) { return f | (f - (f >> 7)); }  // bit 7 of a byte -> 0xff

// Step-table bytes of 4 positions: X = bytes x .. x+3, Y = bytes x+1 .. x+4.  The input bytes a
// token starting there takes for the common forms (reader.go:346-392, 422-472): a literal with a
// 1-byte tag (length < 124; a zero byte is padding, one byte), a copy with a 1-byte tag and a
// plain, Off1 or Off2 offset; 0 for the others (Len1/Len2/Len4 tags, metas, Off4 and OffLong
// offsets).  Bit 7: the byte is a tag (not padding).
__device__ __forceinline__ uint32_t swar_step(uint32_t X, uint32_t Y) {
    const uint32_t X7 = X & 0x7f7f7f7fu, Y7 = Y & 0x7f7f7f7fu;
    const uint32_t isc = X & 0x80808080u;                         // a copy's (or a meta's) tag
    const uint32_t lit = X7 + 0x01010101u;                         // 1 + length
    const uint32_t ge252 = (Y7 + 0x04040404u) & Y & 0x80808080u;  // offset byte >= 252
    const uint32_t ge254 = (Y7 + 0x02020202u) & Y & 0x80808080u;  // >= 254: Off4, OffLong
    const uint32_t cpy = 0x02020202u + (((Y & 0x03030303u) + 0x01010101u) & fanout(ge252));
    const uint32_t mc = fanout(isc);
    const uint32_t adv = (cpy & mc) | (lit & ~mc);
    const uint32_t lwide = (X7 + 0x04040404u) & 0x80808080u;      // length byte >= 124
    const uint32_t nz = (X7 + 0x7f7f7f7fu) & 0x80808080u;         // low 7 bits nonzero (else 0x80: meta)
    const uint32_t rare = lwide | (isc & ~nz) | (isc & ge254);
    const uint32_t tag = (nz | isc) & ~rare;                       // a token's tag: bit 7 of its byte
    return (adv & ~fanout(rare)) | tag;
}

// a refill landed: its 128 bytes into the ring, and the step table of positions at - 8 .. at + 119
// (the 8 bytes before it are in the ring already; positions at + 120 .. at + 127 need bytes of the
// next refill and are written with it)
__device__ __forceinline__ void refill_commit(const Refill &r, uint8_t *ring, uint8_t *tab, int32_t at) {
    const uint64_t before = *(const u64_ua *)(ring + ((at - 8) & (kPRing - 1)));  // (garbage at a restart: never read)
#pragma unroll
    for (int k = 0; k < kPRefill / 16; k++) {
        const int32_t slot = (at + 16 * k) & (kPRing - 1);
        *(u64_ua *)(ring + slot) = r.v[k].lo;
        *(u64_ua *)(ring + slot + 8) = r.v[k].hi;
        if (slot == 0) {  // the mirror: a 16-byte read at any slot is one contiguous access
            *(u64_ua *)(ring + kPRing) = r.v[k].lo;
            *(u64_ua *)(ring + kPRing + 8) = r.v[k].hi;
        }
    }
    // dwords d[0..33]: bytes at - 8 .. at + 127
    uint32_t d[34];
    d[0] = (uint32_t)before;
    d[1] = (uint32_t)(before >> 32);
#pragma unroll
    for (int k = 0; k < kPRefill / 16; k++) {
        d[2 + 4 * k] = (uint32_t)r.v[k].lo;
        d[3 + 4 * k] = (uint32_t)(r.v[k].lo >> 32);
        d[4 + 4 * k] = (uint32_t)r.v[k].hi;
        d[5 + 4 * k] = (uint32_t)(r.v[k].hi >> 32);
    }
#pragma unroll
    for (int k = 0; k < kPRefill / 16; k++) {  // 16 positions (4 words) per store
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int x = 4 * k + q;
            w[q] = swar_step(d[x], __builtin_amdgcn_alignbyte(d[x + 1], d[x], 1));
        }
        // (8-byte pieces at 8-aligned slots: at - 8 + 16 k is 8 mod 16, so a 16-byte store at the
        // last slot would run past the lane's table)
        *(uint64_t *)(tab + ((at - 8 + 16 * k) & (kPRing - 1))) = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
        *(uint64_t *)(tab + ((at + 16 * k) & (kPRing - 1))) = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    }
}

// the token walk of stream s (valid: s < count) with `ring` (kPStride bytes of LDS) as its input
// window and `tab` (kPRing bytes) as its step table; writes its region of the bitmap workspace
// (kSmallRegion words: [0] the token count | log2 of the window << 16, or kSHandOver; then one bit
// per input byte, set at every literal or copy token's first byte)
__device__ __forceinline__ void pre_one(const DecompressArgs &A, const uint64_t s, const bool valid, uint8_t *ring, uint8_t *tab,
                                        uint32_t *bm) {
    const uint64_t sc = valid ? s : 0;
    const uint8_t *b = A.in + A.in_off[sc];
    const int64_t nb64 = (int64_t)(A.in_off[sc + 1] - A.in_off[sc]);
    const uint8_t *in_end = A.in + A.in_off[A.count];
    const int64_t cap64 = (int64_t)(A.out_off[sc + 1] - A.out_off[sc]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;  // 0: no limit
    uint32_t *reg = bm + sc * (uint64_t)kSmallRegion;
    // what K2s takes: slots of <= 4 KiB, streams of <= kSmallIn bytes, batches of >= 16 bytes
    const bool fits = in_end - A.in >= 16 && nb64 <= kSmallIn && cap64 <= kSmallOut;
    bool live = valid && fits, ho = valid && !fits;
    const int32_t nb = live ? (int32_t)nb64 : 0;
    int32_t i = 0, bsl = -1, ntok = 0;
    int32_t F = 0;       // the ring holds input [F - kPRing, F) (what has been committed)
    int32_t cw = 0;      // bitmap word being built
    uint32_t acc = 0;
    live = live && nb > 0;
    Refill r;
    // prologue: the first 128 bytes, waited for
    if (any_lane(live)) {
        refill_issue(r, b, A.in, in_end);
        if (live) refill_commit(r, ring, tab, 0);
        F = live ? kPRefill : 0;
    }
    while (any_lane(live)) {
        // a lane whose next header lies past its window restarts it there; a lane with at most
        // 128 bytes ahead (the oldest half of its ring is behind it) refills the next 128
        if (live && i >= F) F = i & ~15;
        const bool rf = live && F - i <= kPRing - kPRefill && F < nb + 16;
        if (any_lane(rf)) {
            if (rf) refill_issue(r, b + F, A.in, in_end);
        }
        // up to kPStep tokens while the refill is in flight
#pragma unroll 1
        for (int st = 0; st < kPStep; st++) {
            const bool rd = live && i + 16 <= F;
            if (!any_lane(rd)) break;
            const uint32_t e = tab[i & (kPRing - 1)];
            int32_t adv = (int32_t)(e & 0x7f);
            bool tok = (e & 0x80) != 0, bad = false;
            if (any_lane(rd && adv == 0)) {  // a rare form: the full parse of its 16 bytes
                if (rd && adv == 0) {
                    K2Tok t;
                    const int rr = k2_scan(lds16(ring + (i & (kPRing - 1))), i, nb, lim32, limit, t);
                    adv = t.adv;
                    tok = rr == kParseToken;
                    if (rr == kScanReset) {
                        if (ntok != 0) bad = true;  // MetaReset only before any output (k2_check)
                        bsl = (int32_t)t.marg;
                    }
                    bad = bad || rr == kParseHandOver;
                }
            }
            bad = bad || (tok && bsl < 0);  // a token before the window is set
            const bool go = rd && !bad;
            const bool mark = go && tok;
            // the bitmap: a word is stored when the walk leaves it (the words it jumps over are 0)
            const int32_t wi = i >> 5;
            const bool nw = mark && wi != cw;
            if (any_lane(nw)) {
                if (nw) {
                    reg[1 + cw] = acc;
#pragma unroll 1
                    for (int32_t x = cw + 1; x < wi; x++) reg[1 + x] = 0;
                    cw = wi;
                    acc = 0;
                }
            }
            acc = mark ? acc | (1u << (i & 31)) : acc;
            ntok += mark ? 1 : 0;
            i = go ? i + adv : i;
            ho = ho || (rd && bad);
            live = live && !(rd && bad) && i < nb;
        }
        if (any_lane(rf)) {
            if (rf) refill_commit(r, ring, tab, F);
        }
        F = rf ? F + kPRefill : F;
    }
    ho = ho || (valid && fits && i > nb);  // the last token runs past the input
    if (valid && !ho) {  // the last word, the words after it, the count and the window
        const int32_t nw = (nb + 31) >> 5;
        if (nw > 0) reg[1 + cw] = acc;
        for (int32_t x = cw + 1; x < nw; x++) reg[1 + x] = 0;
        reg[0] = (uint32_t)ntok | ((uint32_t)(bsl < 0 ? 0 : bsl) << 16);
    }
    if (ho) {
        reg[0] = kSHandOver;
        const uint32_t at = atomicAdd(&A.slow[0], 1u);
        A.slow[1 + at] = (uint32_t)s;
    }
}

__global__ __launch_bounds__(kPBlock) void k2_pre(DecompressArgs A, uint32_t *bm) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *ring = smem + threadIdx.x * kPStride, *tab = smem + kPTab + threadIdx.x * kPRing;
    for (uint64_t s0 = (uint64_t)blockIdx.x * kPBlock; s0 < A.count; s0 += (uint64_t)gridDim.x * kPBlock) {
        const uint64_t s = s0 + threadIdx.x;
        pre_one(A, s, s < A.count, ring, tab, bm);
    }
}

// ---------------------------------------------------------------------------------------------
// K2q: the moves, 16 lanes per stream (one DPP row), the stream's whole output in LDS
// ---------------------------------------------------------------------------------------------
constexpr int kQBlock = 256;
constexpr int kQG = 16;                        // lanes per stream: one DPP row
constexpr int kQPer = kQBlock / kQG;           // streams per block
constexpr int32_t kQList = 256;                // token starts per 512-position chunk at most (tokens take >= 2 bytes)
// per stream: [16 zero bytes: the history before the stream][output][token list u16][trash 8 B per lane]
constexpr int32_t kQOut = 16, kQListAt = kQOut + kSmallOut, kQTrash = kQListAt + 2 * kQList;
constexpr int32_t kQStride = kQTrash + 8 * kQG;
static_assert(kQStride % 16 == 0, "16-byte aligned groups");

// DPP within a row of 16 lanes
__device__ __forceinline__ int32_t row_shr(int32_t v, int n) {  // lane k gets lane k - n's value, 0 below the row
    switch (n) {
        case 1: return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
        case 2: return __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
        case 4: return __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
        default: return __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
    }
}
__device__ __forceinline__ int32_t row_ror(int32_t v, int n) {  // rotate within the row
    switch (n) {
        case 1: return __builtin_amdgcn_update_dpp(v, v, 0x121, 0xf, 0xf, false);
        case 2: return __builtin_amdgcn_update_dpp(v, v, 0x122, 0xf, 0xf, false);
        case 4: return __builtin_amdgcn_update_dpp(v, v, 0x124, 0xf, 0xf, false);
        default: return __builtin_amdgcn_update_dpp(v, v, 0x128, 0xf, 0xf, false);
    }
}
__device__ __forceinline__ int32_t row_incl_sum(int32_t v) {
    v += row_shr(v, 1);
    v += row_shr(v, 2);
    v += row_shr(v, 4);
    v += row_shr(v, 8);
    return v;
}
__device__ __forceinline__ int32_t row_last(int32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x15F, 0xf, 0xf, false); }  // row_newbcast:15
__device__ __forceinline__ int32_t row_min(int32_t v) {
    v = min(v, row_ror(v, 1));
    v = min(v, row_ror(v, 2));
    v = min(v, row_ror(v, 4));
    v = min(v, row_ror(v, 8));
    return v;
}

// the first n bytes (0..16) of v at d, without branches: the absent pieces go to trash (8 bytes)
__device__ __forceinline__ void put_exact(uint8_t *d, V16 v, uint32_t n, uint8_t *trash) {
    const bool b8 = n >= 8;
    *(u64_ua *)(b8 ? d : trash) = v.lo;
    *(u64_ua *)(n == 16 ? d + 8 : trash) = v.hi;
    uint64_t x = b8 ? v.hi : v.lo;
    uint8_t *t = d + (n & 8);
    *(u32_ua *)((n & 4) ? t : trash) = (uint32_t)x;
    x = (n & 4) ? x >> 32 : x;
    t += n & 4;
    *(u16_ua *)((n & 2) ? t : trash) = (uint16_t)x;
    x = (n & 2) ? x >> 16 : x;
    t += n & 2;
    *(uint8_t *)((n & 1) ? t : trash) = (uint8_t)x;
}

// bytes j .. j+15 of the 32 bytes (a, b), 0 <= j <= 16
__device__ __forceinline__ V16 at32(V16 a, V16 b, uint32_t j) {
    const V16 x = shr16(a, j), y = shl16(b, 16 - j);
    return V16{x.lo | y.lo, x.hi | y.hi};
}

// 16 output bytes at position x (x >= -16 reads the zero history before the stream from the guard)
__device__ __forceinline__ V16 out16(const uint8_t *ob, int32_t x) {
    const V16 v = lds16(ob + (x < -16 ? -16 : x));
    return x < -16 ? V16{0, 0} : v;
}

__device__ __forceinline__ int32_t run_step_of(int32_t per) { return per * (16 / per); }

// the 64 input bytes at y (clamped into the batch near its end: bytes past it read 0)
struct In64 {
    V16 v[4];
};
__device__ __forceinline__ In64 ld64(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    In64 r;
    if (any_lane(y + 64 > hi)) {
#pragma unroll
        for (int q = 0; q < 4; q++) r.v[q] = ld_batch(y + 16 * q, lo, hi);
    } else {
#pragma unroll
        for (int q = 0; q < 4; q++) r.v[q] = ld16v(y + 16 * q);
    }
    return r;
}
// bytes j + o .. j + o + 15 of the 64 (o = 0, 16, 32, 48; bytes past the 64 read 0), j <= 16
__device__ __forceinline__ V16 at64(const In64 &a, uint32_t j, int o) {
    const V16 x = a.v[o / 16];
    const V16 y = o / 16 + 1 < 4 ? a.v[o / 16 + 1] : V16{0, 0};
    return at32(x, y, j);
}

// the streams base .. base+3 of a wave, one per row (s = base + row); ob: the row's LDS output
// (16 zero bytes before it), list: its token list, trash: 8 bytes of this lane's
__device__ __forceinline__ void small_one(const DecompressArgs &A, const uint32_t *bm, const uint64_t s, const int k, uint8_t *ob,
                                          uint16_t *list, uint8_t *trash) {
    const bool v0 = s < A.count;
    const uint64_t sc = v0 ? s : 0;
    const uint32_t *reg = bm + sc * (uint64_t)kSmallRegion;
    const uint32_t w0r = reg[0];
    bool valid = v0 && w0r != kSHandOver;
    const uint8_t *b = A.in + A.in_off[sc];
    const uint8_t *in_end = A.in + A.in_off[A.count];
    const int32_t nb = valid ? (int32_t)(A.in_off[sc + 1] - A.in_off[sc]) : 0;
    const int32_t cap = valid ? (int32_t)(A.out_off[sc + 1] - A.out_off[sc]) : 0;  // (<= kSmallOut: K2p)
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;
    const uint32_t bsl = (w0r >> 16) & 63;
    const int32_t win = bsl >= 30 ? 0x7fffffff : 1 << bsl;
    const int32_t nwd = (nb + 31) >> 5;  // bitmap words
    const uint32_t rsh = (uint32_t)(threadIdx.x & 48);
    int32_t pos = 0;
    uint32_t wnext = k < nwd ? reg[1 + k] : 0;
#pragma unroll 1
    for (int32_t w0 = 0; any_lane(w0 < nwd); w0 += kQG) {
        // ---- the chunk's token starts (512 input positions): a row prefix sum of the popcounts
        uint32_t word = wnext;
        wnext = w0 + kQG + k < nwd ? reg[1 + w0 + kQG + k] : 0;  // (the next chunk's words, in flight)
        const int32_t c = __builtin_popcount(word);
        const int32_t ci = row_incl_sum(c);
        const int32_t nt = valid ? row_last(ci) : 0;
        int32_t e = ci - c;
        const int32_t wbase = (w0 + k) << 5;
        while (any_lane(word != 0)) {
            if (word != 0) {
                list[e++] = (uint16_t)(wbase + (int32_t)__builtin_ctz(word));
                word &= word - 1;
            }
        }
        // ---- rounds of 16 tokens, one per lane; the next round's 64 bytes load during this one
        In64 nx = ld64(b + (k < nt ? (int32_t)list[k] : 0), A.in, in_end);
#pragma unroll 1
        for (int32_t t0 = 0; !(EZ_EXP & (1 << 23)) && any_lane(t0 < nt); t0 += kQG) {
            const bool has = valid && t0 + k < nt;
            const int32_t q = has ? (int32_t)list[t0 + k] : 0;
            const In64 a = nx;
            nx = ld64(b + (t0 + kQG + k < nt ? (int32_t)list[t0 + kQG + k] : 0), A.in, in_end);
            // ---- the token (K2p found it: the common forms branch-free, the long ones by k2_scan)
            int32_t L, fadv, j = 1;
            uint32_t Du;
            bool cp;
            const int32_t ft = fast_tok(a.v[0].lo, L, fadv, Du, cp);
            if (any_lane(has && ft < 0)) {
                if (has && ft < 0) {
                    K2Tok t;
                    (void)k2_scan(a.v[0], q, nb, 0x7fffffff, 0, t);
                    L = t.L;
                    j = t.j;
                    Du = t.D;
                    cp = t.cp;
                }
            }
            L = has ? L : 0;
            cp = has && cp;
            const int32_t D = cp ? (int32_t)Du : 0;
            const int32_t incl = row_incl_sum(L);
            const int32_t total = row_last(incl);
            const int32_t dst = pos + incl - L;
            // the checks on the output position (k2_check, reader.go:251-263): room in the slot, the
            // block size limit, the window; a stream failing one goes to the exact decoder whole
            const bool bad = has && ((uint32_t)pos + (uint32_t)incl > (uint32_t)cap || L > lim32 || (cp && D > win));
            if ((uint32_t)(__builtin_amdgcn_ballot_w64(bad) >> rsh) & 0xffffu) {
                if (valid && k == 0) {
                    const uint32_t at = atomicAdd(&A.slow[0], 1u);
                    A.slow[1 + at] = (uint32_t)s;
                }
                valid = false;
            }
            const bool live = valid && has;
            // ---- literals: up to 64 - j bytes from the loaded ones, the rest from the input
            const bool lit = live && !cp && !(EZ_EXP & (1 << 22));
            put_exact(lit ? ob + dst : trash, at64(a, (uint32_t)j, 0), lit ? (uint32_t)(L < 16 ? L : 16) : 0u, trash);
            if (any_lane(lit && L > 16)) {
#pragma unroll
                for (int o = 16; o < 64; o += 16) {
                    const bool act = lit && L > o;
                    if (any_lane(act)) put_exact(act ? ob + dst + o : trash, at64(a, (uint32_t)j, o), act ? (uint32_t)(L - o < 16 ? L - o : 16) : 0u, trash);
                }
#pragma unroll 1
                for (int32_t o = 64 - j; any_lane(lit && o < L); o += 16) {  // (past the loaded bytes: rare)
                    const bool act = lit && o < L;
                    if (act) {
                        const V16 v = ld_batch(b + q + j + o, A.in, in_end);
                        put_exact(ob + dst + o, v, (uint32_t)(L - o < 16 ? L - o : 16), trash);
                    }
                }
            }
            // ---- copies in batches: a batch runs from the first pending copy up to the first one
            // whose source reaches past that copy's output position (the output before it is final);
            // a copy whose source ends before the round's first byte (or a zero region) is final now
            const int32_t cs = dst - D;
            const int32_t need = cs + (D < L ? D : L);
            const bool fre = cp && (D == 0 || need <= pos);
            bool pend = live && cp && !(EZ_EXP & (1 << 21));
#pragma unroll 1
            while (any_lane(pend)) {
                const int32_t oa = row_min(pend ? dst : 0x7fffffff);
                const bool br = pend && !fre && dst > oa && need > oa;
                const uint32_t bb = (uint32_t)(__builtin_amdgcn_ballot_w64(br) >> rsh) & 0xffffu;
                const int32_t bnd = (int32_t)__builtin_ctz(bb | 0x10000u);
                const bool ex = pend && (fre || k < bnd);
                pend = pend && !ex;
                // a copy that does not read its own output (D >= L, or a zero region): up to 64 bytes
                // read before any is written; a self-overlapping one 16 bytes at a time (D >= 16), or
                // a run of period D < 16 as its 16-byte pattern every run_step bytes
                const bool run = ex && D > 0 && D < 16;
                const bool wide = D >= L || D == 0;
                int32_t stp = wide ? 64 : 16;
                V16 pv{0, 0};
                if (any_lane(run)) {
                    if (run) {
                        pv = run_pattern(shr16(out16(ob, dst - 16), (uint32_t)(16 - D)), (uint32_t)D);
                        stp = run_step_of(D);
                    }
                }
                const bool src = D >= 16;
                int32_t o = 0;
                while (any_lane(ex && o < L)) {
                    const bool act = ex && o < L;
                    V16 v[4];
#pragma unroll
                    for (int p = 0; p < 4; p++) v[p] = src ? out16(ob, cs + o + 16 * p) : pv;
                    put_exact(act ? ob + dst + o : trash, v[0], act ? (uint32_t)(L - o < 16 ? L - o : 16) : 0u, trash);
#pragma unroll
                    for (int p = 1; p < 4; p++) {
                        const bool ap = act && wide && L > o + 16 * p;
                        if (any_lane(ap)) put_exact(ap ? ob + dst + o + 16 * p : trash, v[p], ap ? (uint32_t)(L - o - 16 * p < 16 ? L - o - 16 * p : 16) : 0u, trash);
                    }
                    o += stp;
                }
            }
            pos += total;
        }
    }
    // ---- the output to its slot, 256 bytes per row and step
    if (valid && !(EZ_EXP & (1 << 24))) {
        uint8_t *out = A.out + A.out_off[sc];
        for (int32_t x = 16 * k; x < pos; x += 16 * kQG) {
            const V16 v = lds16(ob + x);
            if (x + 16 <= pos) st16v(out + x, v);
            else put_small(out + x, v, (uint32_t)(pos - x));
        }
        if (k == 0) {
            A.out_size[sc] = (uint64_t)pos;
            if (A.status) A.status[sc] = EZ_OK;
        }
    }
}

__global__ __launch_bounds__(kQBlock) void k2_small(DecompressArgs A, const uint32_t *bm) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int row = (int)(threadIdx.x >> 4), k = (int)(threadIdx.x & 15);
    uint8_t *g = smem + row * kQStride;
    if (k == 0) {  // the zero history before every stream
        *(u64_ua *)g = 0;
        *(u64_ua *)(g + 8) = 0;
    }
    for (uint64_t base = (uint64_t)blockIdx.x * kQPer; base < A.count; base += (uint64_t)gridDim.x * kQPer)
        small_one(A, bm, base + row, k, g + kQOut, (uint16_t *)(g + kQListAt), g + kQTrash + 8 * k);
}

}  // namespace

hipError_t launch_decompress_small(const DecompressArgs &a, uint32_t *bm, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k2_pre, hipFuncAttributeMaxDynamicSharedMemorySize, kPTab + kPBlock * kPRing);
        (void)hipFuncSetAttribute((const void *)k2_small, hipFuncAttributeMaxDynamicSharedMemorySize, kQPer * kQStride);
        attr_done = true;
    }
    const uint64_t gp = (a.count + kPBlock - 1) / kPBlock;
    hipLaunchKernelGGL(k2_pre, dim3((unsigned)(gp < (1u << 30) ? gp : (1u << 30))), dim3(kPBlock), kPTab + kPBlock * kPRing, st, a, bm);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint64_t gq = (a.count + kQPer - 1) / kQPer;
    hipLaunchKernelGGL(k2_small, dim3((unsigned)(gq < (1u << 30) ? gq : (1u << 30))), dim3(kQBlock), kQPer * kQStride, st, a, bm);
    return hipGetLastError();
}

}  // namespace ez
