// ez_decompress_tok.hip — K2t: token-parallel batch decompression, one wave per
// stream, every lane busy on the stream's tokens.
//
// Restates Reader.Read to EOF for NewReaderBytes (reader.go:116-216 read,
// readTag :218-270, continueMetaTag :272-325, Decoder :346-514) for the common
// case through k2_scan (ez_k2_parse.h); anything else hands the stream to the
// exact decoder (ez_decompress.hip), as K2r and K2w do.
//
// Why.  Reader.read walks its tokens one after another; a lane per stream (K2r)
// keeps that chain on one lane and leaves the chip one wave per SIMD at C1, and a
// wave per stream that walks the tokens on the scalar unit and moves each one
// with the whole wave (K2w) pays a scalar parse and a wave-wide step per token.
// Here the walk is split into what is parallel and what is not:
//
//  1. scan: the stream's compressed input is staged 1 KiB at a time (a window)
//     and every lane computes, for each of its 16 input positions, how many input
//     bytes a token starting there would take (SWAR over 4 positions a word; the
//     common forms only, 0 for the others);
//  2. walk: each lane follows the chain through its own 16 positions from every
//     entry offset (backwards, so each position's exit from the lane's segment
//     is one lookup: ex[p]); the scalar unit then crosses the window segment to
//     segment through those exits (64 steps per window, the rare forms parsed in
//     full when the walk reaches them), and every lane marks the real token starts
//     of its segment from the entry the walk gave it;
//  3. tokens: the starts are compacted into a list; each round gives 64 tokens
//     one lane each: the full parse (k2_scan), a wave prefix sum of the output
//     lengths (every token's output position at once), every literal written at
//     once, and the copies in batches: a batch runs every copy up to the first one
//     whose source reaches past the batch's first output byte (copies of log lines
//     mostly read output decoded a few hundred bytes earlier: ~26 batches for the
//     ~210 copies of a C1 stream).
//
// Output goes through an LDS ring of R bytes (R = 4 KiB or 8 KiB) and leaves it
// 1 KiB at a time; copies reaching past the ring read the output already in HBM.
// A token longer than kTBig bytes is moved alone by the whole wave, HBM to HBM.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"
#include "ez_k2_parse.h"
#include "ez_k2_ring.h"

namespace ez {
namespace {

#ifndef EZ_EXP
#define EZ_EXP 0  // timing builds only: 256 no copy batches, 512 no literal pass, 1024 no rounds, 2048 no walk
#endif

constexpr int32_t kTWin = 1024;          // input positions scanned per window (16 per lane)
constexpr int32_t kTStage = kTWin + 96;  // staged input bytes: a header at the window's end reads 16 more
constexpr int32_t kTBig = 512;           // tokens longer than this are moved alone by the whole wave

template <int32_t R>
struct TLayout {
    static constexpr int32_t ring = 16;          // [16 guard][R][16 mirror][16 guard]
    static constexpr int32_t inb = R + 48;       // the staged input window
    // tab: the scan's advances (kTWin bytes; per-lane write trash during the rounds), the segment
    // exits (u16 x kTWin; then the token list), the segment entries (u16 x 64)
    static constexpr int32_t tab = inb + kTStage;
    static constexpr int32_t defs = tab + 3 * kTWin + 2 * kWave;  // the stream's deferred literals (3 x int32 each)
    static constexpr int32_t bytes = defs + 12 * kDefSlots;
    // output bytes of one round at most: the round's writes never reach a ring slot it reads, and
    // a source farther back than the ring is already in HBM (unflushed output stays < 1 KiB)
    static constexpr int32_t budget = R - 1024 - 64;
    static_assert(budget >= kTBig, "a round must hold any token that is not moved alone");
    static_assert(kDeferMin > R, "a deferred literal refills the whole ring");
};

__device__ __forceinline__ uint32_t fanout(uint32_t f) { return f | (f - (f >> 7)); }  // bit 7 of a byte -> 0xff

// Input bytes a token starting at each of 4 positions takes: X = bytes x .. x+3, Y = bytes
// x+1 .. x+4.  The common forms (reader.go:346-392, 422-472): a literal with a 1-byte tag
// (length < 124; a zero byte is padding, one byte), a copy with a 1-byte tag and a plain, Off1
// or Off2 offset.  0 for the others (Len1/Len2/Len4 tags, metas, Off4 and OffLong offsets).
__device__ __forceinline__ uint32_t swar_adv(uint32_t X, uint32_t Y) {
    const uint32_t X7 = X & 0x7f7f7f7fu, Y7 = Y & 0x7f7f7f7fu;
    const uint32_t isc = X & 0x80808080u;                         // a copy's (or meta's) tag
    const uint32_t lit = X7 + 0x01010101u;                         // 1 + length
    const uint32_t ge252 = (Y7 + 0x04040404u) & Y & 0x80808080u;  // offset byte >= 252
    const uint32_t ge254 = (Y7 + 0x02020202u) & Y & 0x80808080u;  // >= 254: Off4, OffLong
    const uint32_t cpy = 0x02020202u + (((Y & 0x03030303u) + 0x01010101u) & fanout(ge252));
    const uint32_t mc = fanout(isc);
    const uint32_t adv = (cpy & mc) | (lit & ~mc);
    const uint32_t lwide = (X7 + 0x04040404u) & 0x80808080u;      // length byte >= 124
    const uint32_t nz = (X7 + 0x7f7f7f7fu) & 0x80808080u;         // low 7 bits nonzero (else 0x80: meta)
    const uint32_t rare = lwide | (isc & ~nz) | (isc & ge254);
    return adv & ~fanout(rare);
}

template <int32_t R>  // (R unused)
__device__ __forceinline__ V16 lds16(const uint8_t *p) {
    return V16{*(const u64_ua *)p, *(const u64_ua *)(p + 8)};
}

// the bytes of v before position x + k (k < 16) that lie before the stream start read 0
__device__ __forceinline__ V16 zero_before_start(V16 v, int32_t x) {
    if (x >= 0) return v;
    const uint32_t nz = (uint32_t)(-x);
    return shl16(shr16(v, nz), nz);
}

typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef uint16_t __attribute__((aligned(1))) u16_ua;

// the first n bytes (1..16) of v at d, without branches: five stores, the absent ones to trash
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
// n bytes (1..16) of position p into the ring, exact; the mirror / wrapped copy only when needed
template <int32_t R>
__device__ __forceinline__ void rput_fast(uint8_t *ring, int32_t p, V16 v, uint32_t n, uint8_t *trash) {
    const int32_t r = p & (R - 1);
    put_exact(ring + r, v, n, trash);
    const bool mir = r < 16 || r + (int32_t)n > R;
    if (__ballot(mir)) {
        if (mir) put_n(ring + (r < 16 ? r + R : r - R), v, n);
    }
}

// bytes a run of period per (1..15) advances per 16-byte pattern store
__device__ __forceinline__ int32_t run_step_of(int32_t per) { return per * (16 / per); }

// the advance of a rare form at input position p (h: its 16 bytes, the same on every lane):
// the full parse; 2^30 (past any stream) when the stream goes to the exact decoder
__device__ __attribute__((noinline)) int32_t rare_adv(const uint8_t *h, int32_t p, int32_t nb, int32_t lim32, int64_t limit) {
    K2Tok t;
    const int rr = k2_scan(lds16<0>(h), p, nb, lim32, limit, t);
    return __builtin_amdgcn_readfirstlane(rr == kParseHandOver ? (1 << 30) : t.adv);
}

// hand the stream over; debug builds (EZ_EXP & 4096) record where (status 100 + code, out_size = pos)
#if (EZ_EXP & 4096)
#define HANDOVER(code)                                                   \
    do {                                                                 \
        if (lane == 0) {                                                 \
            A.out_size[s] = (uint64_t)pos | ((uint64_t)w << 32);         \
            if (A.status) A.status[s] = 100 + (code);                    \
        }                                                                \
        return false;                                                    \
    } while (0)
#else
#define HANDOVER(code) return false
#endif

// a hand-over because the output needs more than the slot: marked for a caller that sizes the slot
// itself (a Reader handle's whole-stream decode retries with a larger one, and the exact decoder does
// not re-decode the stream just to find the slot too small)
#define HANDOVER_ROOM(code)                                   \
    do {                                                      \
        if (A.end_state && lane == 0) A.end_state[0] = -2;    \
        HANDOVER(code);                                       \
    } while (0)

// stream s by the whole wave; false = hand it over to the exact decoder
template <int32_t R>
__device__ bool tok_one(const DecompressArgs &A, const uint64_t s, uint8_t *smem, const int lane) {
    using Lay = TLayout<R>;
    uint8_t *ring = smem + Lay::ring, *inb = smem + Lay::inb, *tab = smem + Lay::tab;
    uint8_t *trash = tab + 16 * lane;  // (the advances are dead during the rounds)
    int32_t *defs = (int32_t *)(smem + Lay::defs);
    int nd = 0;  // deferred literals of this stream (kd_copy moves them after the decoders)
    const uint8_t *b = A.in + A.in_off[s];
    const int64_t nb64 = (int64_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint8_t *in_end = A.in + A.in_off[A.count];
    uint8_t *out = A.out + A.out_off[s];
    const int64_t cap64 = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;
    int32_t w = 0, pos = 0, fl = 0, bsl = -1;  // w: the chain's entry into the next window; fl: output below is in HBM
    if (in_end - A.in < 16 || nb64 >= (1ll << 30) || cap64 >= (1ll << 30) || cap64 < 16) HANDOVER(1);
    const int32_t nb = (int32_t)nb64, cap = (int32_t)cap64;

    while (w < nb) {
        const int32_t base = w & ~15;
        // ---- stage the window [base, base + kTStage) (bytes past the batch read 0)
        for (int32_t k = 16 * lane; k < kTStage; k += 16 * kWave) {
            const uint8_t *y = b + base + k;
            const V16 v = y + 16 <= in_end ? ld16v(y) : ld_clamped(y, A.in, in_end);
            *(u64_ua *)(inb + k) = v.lo;
            *(u64_ua *)(inb + k + 8) = v.hi;
        }
        __syncthreads();
        // ---- scan: the advance of every position base + 16 * lane + j (lane's segment)
        uint32_t ad[4];
        {
            const uint4 a0 = *(const uint4 *)(inb + 16 * lane);
            const uint4 a1 = *(const uint4 *)(inb + 16 * lane + 16);
            ad[0] = swar_adv(a0.x, __builtin_amdgcn_alignbyte(a0.y, a0.x, 1));
            ad[1] = swar_adv(a0.y, __builtin_amdgcn_alignbyte(a0.z, a0.y, 1));
            ad[2] = swar_adv(a0.z, __builtin_amdgcn_alignbyte(a0.w, a0.z, 1));
            ad[3] = swar_adv(a0.w, __builtin_amdgcn_alignbyte(a1.x, a0.w, 1));
            *(uint4 *)(tab + 16 * lane) = make_uint4(ad[0], ad[1], ad[2], ad[3]);
        }
        // ---- segment exits, backwards through the lane's 16 positions: ex[p] = the first
        // position at or past the segment's end (or the window's) that a chain through p
        // reaches, or the first rare form on the way (p itself when it is one); offsets from base
        uint16_t *ex = (uint16_t *)(tab + kTWin), *ent = (uint16_t *)(tab + 3 * kTWin);
        uint16_t *tp = ex;  // (the token list, once the exits are used)
        const int32_t s0 = 16 * lane, se = s0 + 16;
        const int32_t limr = (nb < base + kTWin ? nb : base + kTWin) - base;  // positions walked this window
        const int32_t sx = se < limr ? se : limr;  // the chain stops at the segment's end or the window's
        ent[lane] = 0xffff;
#pragma unroll
        for (int j = 15; j >= 0; j--) {
            const int32_t a = (int32_t)((ad[j >> 2] >> (8 * (j & 3))) & 0xff);
            const int32_t pj = s0 + j, n = pj + a;
            const int32_t in_seg = ex[n < sx ? n : pj];  // (written already when n < sx)
            ex[pj] = (uint16_t)(a == 0 ? pj : (n >= sx ? n : in_seg));
        }
        __syncthreads();
        // ---- walk (uniform) from segment to segment through the exits, resolving the rare forms
        // on the way (their advance stored back into ex for the marking below); each segment's
        // first chain position is its entry
        int32_t e = w - base, sl = -1;
#if (EZ_EXP & 2048)
        e = limr;
#endif
#if !(EZ_EXP & 1048576)
        // exits two steps on, in place: the exit y of p, then the exit of y when y lies in the window
        // and the chain through y leaves y's segment (no rare form on the way), else y -- the walk
        // then crosses two segments per LDS round trip; the entries of the segments it steps over
        // are filled in by the marking below (each is the exit of the segment before it)
        {
            uint32_t e2[8];
            const uint4 r0 = *(const uint4 *)(ex + s0), r1 = *(const uint4 *)(ex + s0 + 8);
            const uint32_t e1[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
            for (int t = 0; t < 8; t++) {
                uint32_t v = 0;
#pragma unroll
                for (int hh = 0; hh < 2; hh++) {
                    const int32_t y = (int32_t)((e1[t] >> (16 * hh)) & 0xffffu);
                    const int32_t z = y < limr ? (int32_t)ex[y] : y;
                    v |= (uint32_t)(y < limr && z >= (y | 15) + 1 ? z : y) << (16 * hh);
                }
                e2[t] = v;
            }
            __syncthreads();  // (every lane has read the exits it needs)
            *(uint4 *)(ex + s0) = make_uint4(e2[0], e2[1], e2[2], e2[3]);
            *(uint4 *)(ex + s0 + 8) = make_uint4(e2[4], e2[5], e2[6], e2[7]);
            __syncthreads();
        }
#endif
        while (e < limr) {  // (e, x, sl uniform)
            const int32_t sg = e >> 4;
            if (sg != sl) {
                if (lane == 0) ent[sg] = (uint16_t)e;
                sl = sg;
            }
            int32_t x = __builtin_amdgcn_readfirstlane((int32_t)ex[e]);
            if (x == e) {  // a rare form: the full parse (2^30: hand over)
                x = e + __builtin_amdgcn_readfirstlane(rare_adv(inb + e, base + e, nb, lim32, limit));
                if (lane == 0) ex[e] = (uint16_t)(x < 0xffff ? x : 0xffff);
            }
            e = x;
        }
        if (base + e > nb) HANDOVER(2);  // the last token runs past the input, or a form to hand over
        const int32_t p = base + e;
        __syncthreads();
        // ---- every lane marks the chain's token starts in its segment, from the entry
        const int32_t sm = se < limr ? se : limr;
        int32_t q2 = (int32_t)ent[lane];
        const bool had = q2 != 0xffff;
        q2 = had ? q2 : se;
        uint32_t m16 = 0;
        while (__ballot(q2 < sm)) {
            if (q2 < sm) {
                m16 |= 1u << (q2 - s0);
                int32_t a = (int32_t)tab[q2];
                if (a == 0) a = (int32_t)ex[q2] - q2;  // a rare form (resolved by the walk)
                q2 += a;
            }
        }
#if !(EZ_EXP & 1048576)
        // the segments the walk stepped over: a marked segment's exit is the entry of the segment it
        // lands in when that one has none yet (the chain's exits lie in distinct segments)
        __syncthreads();
        if (had && q2 < limr && ent[q2 >> 4] == 0xffff) ent[q2 >> 4] = (uint16_t)q2;
        __syncthreads();
        if (!had) {
            q2 = (int32_t)ent[lane];
            q2 = q2 == 0xffff ? se : q2;
        }
        while (__ballot(!had && q2 < sm)) {
            if (!had && q2 < sm) {
                m16 |= 1u << (q2 - s0);
                int32_t a = (int32_t)tab[q2];
                if (a == 0) a = (int32_t)ex[q2] - q2;
                q2 += a;
            }
        }
#endif
        // ---- the token list in input order: a wave prefix sum of the counts, then each lane's starts
        const int32_t mc = __builtin_popcount(m16);
        int32_t ic = mc;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int32_t v = __shfl_up(ic, d, kWave);
            if (lane >= d) ic += v;
        }
        int32_t cnt = __builtin_amdgcn_readlane(ic, kWave - 1);
        __syncthreads();  // (the exits are read; the list overwrites them)
        int32_t at = ic - mc;
        while (__ballot(m16 != 0)) {
            if (m16 != 0) {
                tp[at++] = (uint16_t)(s0 + (int32_t)__builtin_ctz(m16));
                m16 &= m16 - 1;
            }
        }
        __syncthreads();
        // ---- rounds of up to 64 tokens, one per lane
#if (EZ_EXP & 1024)
        cnt = 0;
#endif
        for (int32_t t0 = 0; t0 < cnt;) {
            const bool has = t0 + lane < cnt;
            const int32_t q = base + (has ? (int32_t)tp[t0 + lane] : 0);
            // the common forms branch-free (fast_tok); the others (padding, metas, long tags and
            // offsets) take the full parse
            const V16 h = lds16<R>(inb + (q - base));
            K2Tok tk;
            tk.j = 1;
            tk.marg = 0;
            int32_t fadv;
            const int32_t ft = fast_tok(h.lo, tk.L, fadv, tk.D, tk.cp);
            tk.D = tk.cp ? tk.D : 0;
            int rr = kParseToken;
            if (__ballot(has && (ft < 0 || tk.L > lim32))) {
                if (has && (ft < 0 || tk.L > lim32)) rr = k2_scan(h, q, nb, lim32, limit, tk);
            }
            rr = has ? rr : kParseSkip;
            if (__ballot(rr == kParseHandOver)) HANDOVER(3);
            const uint64_t rsts = __ballot(rr == kScanReset);
            if (rsts) {  // MetaReset: only before any output (k2_check), once
                const int f = (int)__builtin_ctzll(rsts);
                if (pos != 0 || __builtin_popcountll(rsts) > 1 || __ballot(rr == kParseToken && lane < f)) HANDOVER(4);
                bsl = __builtin_amdgcn_readlane((int)tk.marg, f);
            }
            const bool tok = rr == kParseToken;
            if (bsl < 0 && __ballot(tok)) HANDOVER(5);  // a token before the window is set
            int32_t L = tok ? tk.L : 0;
            int32_t incl = L;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const int32_t v = __shfl_up(incl, d, kWave);
                if (lane >= d) incl += v;
            }
            // the round: up to the first token moved alone, within the output budget
            const uint64_t cut = __ballot(has && ((tok && L > kTBig) || incl > Lay::budget));
            const int32_t nr = cut ? (int32_t)__builtin_ctzll(cut) : (cnt - t0 < kWave ? cnt - t0 : kWave);
            if (nr == 0) {
                // ---- lane 0's token alone (longer than kTBig): HBM to HBM by the whole wave
                const int32_t L0 = __builtin_amdgcn_readlane(L, 0), D0 = __builtin_amdgcn_readlane((int)tk.D, 0);
                const bool cp0 = __builtin_amdgcn_readlane((int)tk.cp, 0) != 0;
                const int32_t src0 = __builtin_amdgcn_readlane(q + tk.j, 0);
                if ((uint32_t)pos + (uint32_t)L0 > (uint32_t)cap) HANDOVER_ROOM(6);
                if (cp0 && bsl < 30 && (uint32_t)D0 > (1u << bsl)) HANDOVER(6);
                for (int32_t x = fl + 16 * lane; x < pos; x += 16 * kWave) {  // everything before it to HBM
                    const V16 v = rld<R>(ring, x);
                    if (x + 16 <= pos) st16v(out + x, v);
                    else put_small(out + x, v, (uint32_t)(pos - x));
                }
                __builtin_amdgcn_s_waitcnt(0);  // (stores done before the copy reads them back)
                if (!cp0 && L0 >= kDeferMin && nd < kDefSlots && A.defer) {
                    // a long literal: recorded for kd_copy (the chip moves it after the decoders); the
                    // ring gets its last bytes from the input
                    if (lane == 0) {
                        const uint32_t at = atomicAdd(&A.defer[0], 1u);
                        if (at < A.defer_cap)
                            ((DeferLit *)(A.defer + 4))[at] = DeferLit{A.in_off[s] + (uint64_t)src0, A.out_off[s] + (uint64_t)pos, (uint64_t)L0};
                        defs[3 * nd] = pos;
                        defs[3 * nd + 1] = src0;
                        defs[3 * nd + 2] = L0;
                    }
                    nd++;
                    for (int32_t x = L0 - R + 16 * lane; x < L0; x += 16 * kWave) {  // (L0 > R)
                        const uint8_t *y = b + src0 + x;
                        rput<R>(ring, pos + x, y + 16 <= in_end ? ld16v(y) : ld_clamped(y, A.in, in_end), (uint32_t)(L0 - x < 16 ? L0 - x : 16));
                    }
                    pos += L0;
                    fl = pos;
                    t0 += 1;
                    __syncthreads();
                    continue;
                }
                if (!cp0 || D0 == 0 || D0 >= 16) {
                    // passes of W bytes: a copy's reads stay below the bytes its pass writes
                    const int32_t W = !cp0 || D0 == 0 ? 16 * kWave : ((D0 & ~15) < 16 * kWave ? (D0 & ~15) : 16 * kWave);
                    for (int32_t done = 0; done < L0; done += W) {
                        const int32_t k = done + 16 * lane;
                        if (16 * lane < W && k < L0) {
                            V16 v{0, 0};
                            if (!cp0) {
                                const uint8_t *y = b + src0 + k;
                                v = y + 16 <= in_end ? ld16v(y) : ld_clamped(y, A.in, in_end);
                            } else if (D0 != 0) {
                                v = far16(out, cap, b, pos - D0 + k, nd, defs);  // before the stream: 0
                            }
                            if (k + 16 <= L0) st16v(out + pos + k, v);
                            else put_small(out + pos + k, v, (uint32_t)(L0 - k));
                        }
                        __builtin_amdgcn_s_waitcnt(0);
                    }
                } else {  // a short-period run: its 16-byte pattern every step bytes
                    V16 v = zero_before_start(rld<R>(ring, pos - 16), pos - 16);
                    const V16 pv = run_pattern(shr16(v, (uint32_t)(16 - D0)), (uint32_t)D0);
                    const int32_t stp = run_step_of(D0);
                    for (int32_t k = stp * lane; k < L0; k += stp * kWave) {
                        if (k + 16 <= L0) st16v(out + pos + k, pv);
                        else put_small(out + pos + k, pv, (uint32_t)(L0 - k));
                    }
                    __builtin_amdgcn_s_waitcnt(0);
                }
                // the ring gets the token's last bytes back (what later copies may read from it)
                const int32_t np = pos + L0;
                const int32_t lo = np - R > pos ? np - R : pos;
                for (int32_t x = lo + 16 * lane; x < np; x += 16 * kWave)
                    rput<R>(ring, x, ld_clamped16(out + x, out, out + cap), (uint32_t)(np - x < 16 ? np - x : 16));
                pos = np;
                fl = np;
                t0 += 1;
                __syncthreads();
                continue;
            }
            const bool in = lane < nr && tok;
            const int32_t total = __builtin_amdgcn_readlane(incl, nr - 1);
            const int32_t dst = pos + incl - L;
            // a Break meta (0x80, MetaBreak | MetaLen0) of the round: its output position, for a Reader
            // handle's Reads (which stop there with ErrBreak, reader.go:312-313)
            if (A.breaks && __ballot(has && lane < nr && rr == kParseSkip && ((uint32_t)h.lo & 0xffffu) == (0x80u | ((kMetaBreak | kMetaLen0) << 8)))) {
                if (has && lane < nr && rr == kParseSkip && ((uint32_t)h.lo & 0xffffu) == (0x80u | ((kMetaBreak | kMetaLen0) << 8))) {
                    const uint64_t at = atomicAdd((unsigned long long *)A.breaks, 1ull);
                    if (at < A.breaks_cap) A.breaks[1 + at] = (uint64_t)dst;
                }
            }
            if ((uint32_t)pos + (uint32_t)total > (uint32_t)cap) HANDOVER_ROOM(7);
            if (__ballot(in && tk.cp && bsl < 30 && tk.D > (1u << bsl))) HANDOVER(8);
            // ---- literals: all at once (their bytes from the staged window, or HBM past it)
            const bool lit = in && !tk.cp;
            const int32_t src = q + tk.j;
            for (int32_t k = 0; !(EZ_EXP & 512) && __ballot(lit && 16 * k < L); k++) {
                if (lit && 16 * k < L) {
                    const int32_t x = src + 16 * k;
                    const bool staged = x + 16 <= base + kTStage;
                    V16 v = lds16<R>(inb + (staged ? x - base : 0));
                    if (__ballot(!staged)) {
                        if (!staged) {
                            const uint8_t *y = b + x;
                            v = y + 16 <= in_end ? ld16v(y) : ld_clamped(y, A.in, in_end);
                        }
                    }
                    rput_fast<R>(ring, dst + 16 * k, v, (uint32_t)(L - 16 * k < 16 ? L - 16 * k : 16), trash);
                }
            }
            // ---- copies, in batches: every copy up to the first one whose source reaches past
            // the batch's first output byte (its sources are final; the writes never overlap)
            const bool cpy = in && tk.cp;
            const int32_t D = (int32_t)tk.D;
            const int32_t cs = dst - D;
            const int32_t need = D == 0 ? -0x7fffffff : cs + (D < L ? D : L);
            const int32_t ringlo = pos + total - R + 16;  // sources from here on are in the ring
            uint64_t cm = (EZ_EXP & 256) ? 0 : __ballot(cpy);
            // ---- sources final at the round's start (every copy marked fre may run in any batch):
            // zero regions, sources before the round, sources inside one literal of the round (all
            // written above); a copy (D >= 16, not overlapping itself) whose source lies inside an
            // earlier copy of the round reads that copy's source instead (the same bytes),
            // repeated while it lands in a copy.  The token holding a position: the last lane whose
            // output starts at or before it (dst is non-decreasing over the lanes; a lane with no
            // output shares its dst with the next one)
            int32_t ys = cs;  // the copy's (redirected) source
            bool fre = cpy && (D == 0 || need <= pos);
#if !(EZ_EXP & 8192)
            // only in rounds with >= 16 copies reading the round's own output: there the searches
            // pay (C4s: 26 -> 22 batches per round, K2 101 -> 94 ms); on C2's logs (10 such copies per
            // round on average, 4.1 -> 3.0 batches) they cost more than the batches they save
            // (4.44 -> 4.55 ms), and 2 % of its rounds reach 16
            if (__builtin_popcountll(__ballot(cpy && !fre)) >= 16) {
                const int32_t tend = in ? dst + L : 0;
                const int32_t tinf = !in ? 0 : (!tk.cp ? -1 : D);  // -1 literal, D > 0 a copy, 0 neither
                int32_t ye = need;
                bool open = cpy && !fre;
                const bool redir = D >= 16 && D >= L;
                // (two steps resolve 72 % of what any number would on C2's logs: a simulation of
                // the rounds; each step a 4-way search, three dependent LDS round trips)
                for (int it = 0; it < 2 && __ballot(open); it++) {
                    const int32_t y = open ? ys : pos;
                    int t = 0;
#pragma unroll
                    for (int st = 16; st > 0; st >>= 2) {
                        const int32_t d1 = __builtin_amdgcn_ds_bpermute(4 * (t + st), dst);
                        const int32_t d2 = __builtin_amdgcn_ds_bpermute(4 * (t + 2 * st), dst);
                        const int32_t d3 = __builtin_amdgcn_ds_bpermute(4 * (t + 3 * st), dst);
                        t += (d1 <= y ? st : 0) + (d2 <= y ? st : 0) + (d3 <= y ? st : 0);
                    }
                    const int32_t te = __builtin_amdgcn_ds_bpermute(4 * t, tend);
                    const int32_t ti = __builtin_amdgcn_ds_bpermute(4 * t, tinf);
                    if (open) {
                        if (ys < pos || ye > te || t >= lane) {
                            open = false;  // straddles tokens or the round's start: the batches decide
                        } else if (ti < 0) {
                            fre = true;  // inside a literal of the round
                            open = false;
                        } else if (ti > 0 && redir) {
                            ys -= ti;
                            ye -= ti;
                            if (ye <= pos) {
                                fre = true;
                                open = false;
                            }
                        } else {
                            open = false;
                        }
                    }
                }
                if (open) ys = cs;  // unresolved: the batches' rule, on the copy's own source
            }
#endif
            // a copy reading output flushed to HBM: the flush stores complete first (same CU: its
            // L1 then serves the bytes stored)
            if (__ballot(cpy && D >= 16 && ys < ringlo)) __builtin_amdgcn_s_waitcnt(0);
            while (cm) {
                const int a = (int)__builtin_ctzll(cm);
                const int32_t oa = __builtin_amdgcn_readlane(dst, a);
                const bool pend = (cm >> lane) & 1;
                const uint64_t brk = __ballot(pend && !fre && lane > a && need > oa);
                const int bnd = brk ? (int)__builtin_ctzll(brk) : kWave;
                const bool ex = pend && (fre || lane < bnd);
                // the common copy (D >= 16, source in the ring, after the stream start): 16-byte
                // ring reads and exact writes; the others (runs and zero regions, sources before
                // the start or past the ring) below
                const bool slow = ex && (D < 16 || ys < 0 || ys < ringlo);
                if (__ballot(slow)) {
                    V16 pv{0, 0};
                    int32_t stp = 16;
                    if (slow && D > 0 && D < 16) {
                        const V16 v = zero_before_start(rld<R>(ring, dst - 16), dst - 16);
                        pv = run_pattern(shr16(v, (uint32_t)(16 - D)), (uint32_t)D);
                        stp = run_step_of(D);
                    }
                    for (int32_t k = 0; __ballot(slow && stp * k < L); k++) {
                        const int32_t o = stp * k;
                        if (slow && o < L) {
                            V16 v = pv;  // a run's pattern; a zero region's zeros
                            if (D >= 16) {
                                const int32_t x = ys + o;
                                if (x >= ringlo) v = zero_before_start(rld<R>(ring, x), x);
                                else v = far16(out, cap, b, x, nd, defs);  // flushed already (or deferred)
                            }
                            rput<R>(ring, dst + o, v, (uint32_t)(L - o < 16 ? L - o : 16));
                        }
                    }
                }
                const bool fast = ex && !slow;
                for (int32_t k = 0; __ballot(fast && 16 * k < L); k++) {
                    if (fast && 16 * k < L)
                        rput_fast<R>(ring, dst + 16 * k, rld<R>(ring, ys + 16 * k), (uint32_t)(L - 16 * k < 16 ? L - 16 * k : 16), trash);
                }
                cm &= ~__ballot(ex);
            }
            pos += total;
            t0 += nr;
            while (pos >= fl + 16 * kWave) {
                st16v(out + fl + 16 * lane, rld<R>(ring, fl + 16 * lane));
                fl += 16 * kWave;
            }
        }
        w = p;
        __syncthreads();
    }
    for (int32_t x = fl + 16 * lane; x < pos; x += 16 * kWave) {  // the last partial chunk, exact bytes
        const V16 v = rld<R>(ring, x);
        if (x + 16 <= pos) st16v(out + x, v);
        else put_small(out + x, v, (uint32_t)(pos - x));
    }
    if (lane == 0) {
        A.out_size[s] = (uint64_t)pos;
        if (A.status) A.status[s] = EZ_OK;
        if (A.end_state) {  // (one MetaReset, before any output: r.pos is the output since the start)
            A.end_state[0] = bsl < 0 ? 0 : (int64_t)1 << bsl;
            A.end_state[1] = pos;
        }
    }
    return true;
}

template <int32_t R>
__global__ __launch_bounds__(64) void k2_tok(DecompressArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)threadIdx.x;
    for (uint64_t s = blockIdx.x; s < A.count; s += gridDim.x)
        if (!tok_one<R>(A, s, smem, lane) && lane == 0) {
            const uint32_t at = atomicAdd(&A.slow[0], 1u);
            A.slow[1 + at] = (uint32_t)s;
        }
}

}  // namespace

// R: an 8 KiB ring keeps more copies in LDS, a 4 KiB one fits more waves per CU (TLayout<4096>
// ~8.6 KiB, <8192> ~12.7 KiB of LDS).  A batch with more streams than the chip holds runs in
// rounds of resident waves, the last one partly empty, so R = 4096 is taken whenever it needs
// fewer such rounds (C2, 4,096 x 256 KiB: 3,072 resident waves at 8 KiB, all 4,096 at 4 KiB:
// K2 7.06 -> 4.93 ms), and always when the whole stream fits it.
static uint64_t resident_waves(const void *kernel, size_t lds) {
    int dev = 0, ncu = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 64, lds) != hipSuccess || per <= 0 || ncu <= 0)
        return 1;
    return (uint64_t)per * (uint64_t)ncu;
}
hipError_t launch_decompress_tok(const DecompressArgs &a, hipStream_t st) {
    const uint64_t grid = a.count < (1u << 30) ? a.count : (1u << 30);
    static const int force_r = knob("EZ_K2T_R", 0);  // A/B (experiment builds): 4096 / 8192
    static const uint64_t res4 = resident_waves((const void *)k2_tok<4096>, TLayout<4096>::bytes);
    static const uint64_t res8 = resident_waves((const void *)k2_tok<8192>, TLayout<8192>::bytes);
    const bool fits = a.max_out != 0 && a.max_out <= 4096;  // the whole stream fits the ring
    const bool fewer_rounds = (grid + res4 - 1) / res4 < (grid + res8 - 1) / res8;
    if (force_r == 4096 || (force_r == 0 && (fits || fewer_rounds))) {
        hipLaunchKernelGGL(k2_tok<4096>, dim3((unsigned)grid), dim3(64), TLayout<4096>::bytes, st, a);
    } else {
        hipLaunchKernelGGL(k2_tok<8192>, dim3((unsigned)grid), dim3(64), TLayout<8192>::bytes, st, a);
    }
    return hipGetLastError();
}

}  // namespace ez
