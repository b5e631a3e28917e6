// ez_compress.hip — K1: bit-exact eazy compression on gfx950.
//
// Restates Writer.Write (writer.go:206-337) with writeRunlen (:441-489),
// writeZeros (:407-439), hash (:491-493), the header (:495-517) and the
// Encoder (:537-597).  One wave64 per stream.
//
// Speculative window parse: the greedy loop visits position
// i, inserts ht[hash(i)] = start+i and judges the previous entry.  Judging
// depends only on (done, w.pos, ring, ht-before-insert), and none of these
// change until the first ACCEPT.  So the wave judges 64 consecutive
// positions at once:
//   * lane j hashes position i+j; its candidate is the latest earlier lane
//     of the window with the same hash (an LDS bucket mask + exact check),
//     else ht[hash];
//   * every lane evaluates its branch (far skip / runlen / zero run / cut /
//     window match) with extensions capped at kCap bytes — acceptance is
//     monotone in the extension lengths, so a capped result is either a
//     certain reject, a certain accept, or "maybe";
//   * the first lane that can accept is resolved exactly with wave-wide
//     64-byte extension steps (ballot + ctz); if it rejects, the next one;
//   * hash inserts of lanes <= a are applied last-writer-wins, then lane a's
//     action is emitted and the next window starts at the new i (which may
//     be smaller than before: SURVEY A.7).
// The ring (block) is never materialised for fresh streams: a linear view
// reproduces block[x & mask] exactly:
//   q = w.pos - bs + ((x - w.pos) mod bs);  byte = q >= start ? p[q-start]
//                                                  : (ring ? ring[q & mask] : 0)
#include <atomic>
#include <string>
#include <type_traits>

#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"

#include <stdlib.h>

namespace ez {
namespace {

constexpr int kCap = 8;          // per-lane speculative extension cap (>= kMinCopyChunk)
constexpr int kBuckets = 256;    // intra-window hash bucket masks
constexpr int kMaskBytes = kBuckets * 8;
constexpr int kHashBytes = kWave * 4;
constexpr int64_t kPLdsMax = 16 * 1024;  // stage streams up to this size in LDS
constexpr int64_t kHtLdsMax = 4096;      // hash tables up to this many entries in LDS
constexpr uint32_t kWinBytes = 32768;    // LDS window of a long stream (EZ_K1W_WIN, 0: none)

enum Kind : int { kReject = 0, kWin = 1, kRun = 2, kCut = 3, kZero = 4 };

// Stream input view: LDS-staged (PL) or global.
template <bool PL>
struct InView {
    static constexpr bool kLds = PL;
    const uint8_t *g;      // global bytes of the stream
    const uint8_t *lo, *hi;  // the batch's input bytes (16-byte loads stay inside)
    const uint32_t *gw;    // global aligned words covering g
    uint64_t gr;           // g - gw (bytes)
    uint64_t glast;        // last valid word index of gw
    const uint32_t *lw;    // LDS words (PL)
    uint32_t lr;           // byte misalignment inside lw (PL)
    // !PL, long streams: an LDS window of the stream around the parse position, so that the
    // reads near i (the next window's bytes, zero runs, literals) are LDS reads, not one HBM
    // round trip each: ww[k] = gw-relative bytes wa0 + 4k .. (wnb bytes held)
    const uint32_t *ww = nullptr;
    int64_t wa0 = 0;
    uint64_t wnb = 0;

    // window offset of stream byte x, when [x, x+k) is held
    __device__ __forceinline__ bool inw(int64_t x, int64_t k, uint64_t &a) const {
        const int64_t sa = (int64_t)gr + x - wa0;
        a = (uint64_t)sa;
        return !PL && ww && sa >= 0 && sa + k <= (int64_t)wnb;
    }
    // 16 window bytes at window offset a (aligned words + byte shifts)
    __device__ __forceinline__ V16 wv16(uint64_t a) const {
        const uint32_t *w = ww + (a >> 2);
        const uint32_t r = (uint32_t)(a & 3);
        const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
        const uint32_t e0 = __builtin_amdgcn_alignbyte(d1, d0, r), e1 = __builtin_amdgcn_alignbyte(d2, d1, r);
        const uint32_t e2 = __builtin_amdgcn_alignbyte(d3, d2, r), e3 = __builtin_amdgcn_alignbyte(d4, d3, r);
        return V16{(uint64_t)e0 | ((uint64_t)e1 << 32), (uint64_t)e2 | ((uint64_t)e3 << 32)};
    }
    __device__ __forceinline__ uint32_t b(int64_t x) const {
        if (PL) return ((const uint8_t *)lw)[lr + (uint64_t)x];
        uint64_t a;
        if (inw(x, 1, a)) return ((const uint8_t *)ww)[a];
        return g[x];
    }
    __device__ __forceinline__ uint32_t u32(int64_t x) const {
        if (PL) return words_u32(lw, lr + (uint64_t)x);
        uint64_t wa;
        if (inw(x, 4, wa)) return words_u32(ww, wa);
        const uint64_t a = gr + (uint64_t)x;
        const uint64_t k = a >> 2;
        const uint32_t w0 = gw[k];
        const uint32_t w1 = gw[k + 1 <= glast ? k + 1 : glast];
        return __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(a & 3));
    }
};

struct OutBuf {
    uint8_t *p;
    int64_t cap;
    int64_t op;
    int err;
};

__device__ __forceinline__ void put_hdr(OutBuf &o, const Hdr &h, int lane) {
    if (o.err) return;
    if (o.op + h.n > o.cap) { o.err = EZ_ENOSPC; return; }
    if (lane < h.n) o.p[o.op + lane] = h.byte(lane);
    o.op += h.n;
}

template <class V>
__device__ __forceinline__ void put_bytes(OutBuf &o, const V &P, int64_t src, int64_t L, int lane) {
    if (o.err) return;
    if (o.op + L > o.cap) { o.err = EZ_ENOSPC; return; }
    uint8_t *d = o.p + o.op;
    if (!V::kLds && L >= 64) {
        // global input (or the LDS window): 16 bytes per lane, 1 KiB per wave step (a fresh
        // stream's trailing literal is the whole Write when nothing matches, C4)
        const uint8_t *q = P.g + src;
        for (int64_t k = 16 * lane; k < L; k += 16 * kWave) {
            uint64_t wa;
            const V16 v = P.inw(src + k, 16, wa) ? P.wv16(wa) : q + k + 16 <= P.hi ? ld16v(q + k) : ld_clamped(q + k, P.lo, P.hi);
            if (k + 16 <= L) st16v(d + k, v);
            else put_small(d + k, v, (uint32_t)(L - k));
        }
    } else {
        for (int64_t k = lane; k < L; k += kWave) d[k] = (uint8_t)P.b(src + k);
    }
    o.op += L;
}

// appendLiteral writer.go:519-522
template <class V>
__device__ __forceinline__ void put_literal(OutBuf &o, const V &P, int64_t st, int64_t end, int lane) {
    Hdr h;
    if (!hdr_tag(h, kLiteral, end - st)) { o.err = EZ_EINVAL; return; }
    put_hdr(o, h, lane);
    put_bytes(o, P, st, end - st, lane);
}

// Wave-cooperative extension: number of consecutive m >= from with ok(m).
template <class T, class F>
__device__ __forceinline__ T coop_count(T from, int lane, F ok) {
    T base = from;
    for (;;) {
        const uint64_t bad = wballot(!ok(base + (T)lane));
        if (bad) return base + (T)ffs64(bad);
        base += kWave;
    }
}

template <bool PL, bool HTL, bool RING, bool MWP>
__device__ void compress_stream(const CompressArgs &A, uint64_t s, uint8_t *smem) {
    // SMALL (fresh single-Write streams shorter than 2 GiB: the launcher's non-multi-Write, non-ring
    // variants): stream positions in 32 bits and start = 0 -- fewer live scalars, 32-bit math
    constexpr bool SMALL = !RING && !MWP;
    typedef typename std::conditional<SMALL, int32_t, int64_t>::type I;
    const int lane = lane_id();
    const uint64_t ib = A.in_off[s];
    // multi-Write streams (A.write_idx; fresh streams, or the handle's stream with RING): Writes k = write_idx[s] ..
    // write_idx[s+1]-1 of one Writer, Write k ending at in[write_end[k]]; each Write's loop runs to
    // its own end (writer.go:213) and the table and the history carry over (writer.go:40-45)
    const bool mw = MWP && A.write_idx != nullptr;  // MWP: a multi-Write variant (fewer live scalars without)
    uint64_t wk = 0, wlast = 0;
    if (mw) {
        wk = A.write_idx[s];
        wlast = A.write_idx[s + 1];
    }
    uint64_t wbeg = ib;  // the current Write's first byte (index into A.in)
    I n = (I)((mw ? (wk < wlast ? A.write_end[wk] : ib) : A.in_off[s + 1]) - ib);
    const int64_t bs = A.bs, mask = bs - 1;
    const I hs = A.hs;
    const unsigned hsh = 32u - (unsigned)(64 - __builtin_clzll((uint64_t)(hs - 1)));
    I start = SMALL ? (I)0 : (I)A.start;  // stream position of the current Write's first byte (fresh single Writes: 0)
    const uint8_t *ring = A.ring;

    // ---- LDS carve (all offsets 16-aligned)
    const uint64_t ht_bytes = HTL ? (uint64_t)hs * 4 : 0;
    // (smem + ht_bytes: kMaskBytes + kHashBytes of scratch, unused since the ballot hash match)
    uint32_t *lw = (uint32_t *)(smem + ht_bytes + kMaskBytes + kHashBytes);
    // FP: beside every table entry, the 16 stream bytes around the position it holds
    // (x-8 .. x+7), so that a candidate is judged without loading its bytes
    constexpr bool FP = HTL && !RING && !PL;
    V16 *fp = (V16 *)(smem + ht_bytes + kMaskBytes + kHashBytes);
    uint32_t *ht;
    if (HTL) ht = (uint32_t *)smem;
    else ht = RING ? A.ht_global : A.ht_global + (uint64_t)blockIdx.x * (uint64_t)hs;

    // ---- input view (+ LDS staging)
    InView<PL> P;
    P.g = A.in + ib;
    P.lo = A.in;
    P.hi = A.in + A.in_off[A.count];
    P.gr = (uint64_t)(uintptr_t)P.g & 3;
    P.gw = (const uint32_t *)(P.g - P.gr);
    P.glast = (P.gr + (uint64_t)n + 3) / 4;
    P.glast = P.glast ? P.glast - 1 : 0;
    P.lw = lw;
    P.lr = (uint32_t)P.gr;
    if (PL) {
        const uint64_t nw = (P.gr + (uint64_t)n + 3) / 4;
        for (uint64_t k = lane; k < nw; k += kWave) lw[k] = P.gw[k];
        if (lane < 4) lw[nw + lane] = 0;
    }
    // K1x resume: the table K1x prepared (spec_mode 1: at its first emitting position; 2: at from)
    const int smode = RING ? 0 : A.spec_mode;
    // long streams: the LDS window (A.win_bytes, after the fingerprints), slid along with the
    // parse; not for spec_mode 1, which takes one action per call
    uint4 *win = (uint4 *)(smem + ht_bytes + kMaskBytes + kHashBytes + (FP ? (uint64_t)hs * 16 : 0));
    const bool wl = !PL && !RING && !mw && A.win_bytes != 0 && smode != 1 && A.in_off[A.count] >= 16;
    bool wend = false;  // the window reaches the stream's (or the batch's) end: no later refill
    // window from stream position base (16-byte aligned addresses, inside the batch)
    auto refill = [&](I base) {
        const uint64_t ga = (uint64_t)(uintptr_t)P.gw;
        int64_t a0 = (int64_t)(((ga + P.gr + (uint64_t)base) & ~15ull) - ga);
        if (ga + (uint64_t)a0 < (uint64_t)(uintptr_t)P.lo) a0 += 16;
        int64_t n16 = (int64_t)(A.win_bytes / 16);
        const int64_t max16 = (int64_t)(((uint64_t)(uintptr_t)P.hi - (ga + (uint64_t)a0)) / 16);
        const int64_t need16 = ((int64_t)P.gr + n + 16 - a0 + 15) / 16;
        if (n16 >= need16 || n16 >= max16) {
            wend = true;
            n16 = need16 < max16 ? need16 : max16;
        }
        __syncthreads();  // the old window's readers are done
        const uint4 *src = (const uint4 *)(ga + (uint64_t)a0);
#pragma unroll 8
        for (I k = lane; k < n16; k += kWave) win[k] = src[k];
        if (lane < 2) win[n16 + lane] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        P.ww = (const uint32_t *)win;
        P.wa0 = a0;
        P.wnb = (uint64_t)n16 * 16;
    };
    // ---- hash table and bucket masks
    if (HTL) {
        if (RING) for (I k = lane; k < hs; k += kWave) ht[k] = A.ht_global[k];
        else if (smode) for (I k = lane; k < hs; k += kWave) ht[k] = A.spec_tab[s * (uint64_t)hs + k];
        else for (I k = lane; k < hs; k += kWave) ht[k] = 0;
    } else if (!RING) {
        for (I k = lane; k < hs; k += kWave) ht[k] = 0;
    }
    __syncthreads();

    OutBuf o;
    o.p = A.out + A.out_off[s];
    o.cap = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    o.op = smode ? (int64_t)A.spec[s].op : 0;
    o.err = 0;

    // ---- header (writer.go:207-209, 495-517; K1x wrote it for the streams it resumes)
    if (A.header && !smode) {
        Hdr h;
        if (A.append_magic) { h.put(0x80); h.put(0x02); h.put('e'); h.put('a'); h.put('z'); h.put('y'); }
        if (A.ver != 0) { h.put(0x80); h.put(0x08); h.put((uint32_t)A.ver); }
        h.put(0x80); h.put(0x10); h.put((uint32_t)__builtin_ctzll((uint64_t)bs));
        put_hdr(o, h, lane);
    }

    // block[y & mask] as seen while w.pos == wpos; a multi-Write stream's earlier
    // Writes are the bytes before P.g in the same batch
    auto ringb = [&](I y, I wpos) -> uint32_t {
        const int64_t q = wpos - bs + ((y - wpos) & mask);
        if (q >= start || (mw && q >= A.start)) return P.b(q - start);
        if (RING) return ring[q & mask];
        return 0u;
    };

    // 8 stream bytes from y (global view; any bytes outside the batch read 0),
    // and the 8 bytes block[(y .. y+7) & mask] when they map to 8 consecutive stream
    // bytes or to the zero history before a fresh stream (false: take the byte loop)
    const uint8_t *in_lo = A.in, *in_hi = A.in + A.in_off[A.count];
    auto s8 = [&](I y) -> uint64_t {
        uint64_t wa;
        if (P.inw(y, 8, wa)) return P.wv16(wa).lo;
        const uint8_t *q = P.g + y;
        if (q >= in_lo && q + 8 <= in_hi) return *(const uint64_t __attribute__((aligned(1))) *)q;
        return (in_hi - in_lo >= 16) ? ld_clamped(q, in_lo, in_hi).lo : 0ull;
    };
    auto ring8 = [&](I y, I wpos, uint64_t &v) -> bool {
        const int64_t r = (y - wpos) & mask;
        if (r + 7 >= bs) return false;  // wraps inside the 8 bytes
        const int64_t q = wpos - bs + r;
        if (q >= start || (mw && q >= A.start)) { v = s8(q - start); return true; }
        if (!RING && q + 8 <= A.start) { v = 0; return true; }
        // the handle's ring: bytes before this call, slot q & mask holds stream byte q (or the zero
        // history); one 8-byte load instead of a dependent byte loop through HBM
        if (RING && q + 8 <= A.start && (q & mask) + 8 <= bs) {
            v = *(const uint64_t __attribute__((aligned(1))) *)(ring + (q & mask));
            return true;
        }
        return false;
    };

    // appendLiteral; in spec_mode 1 the bytes are left to K1x's copy kernel (a literal there can be
    // megabytes, one wave would copy it at 1 KiB per step)
    auto literal = [&](I st, I end) {
        if (smode != 1) { put_literal(o, P, st, end, lane); return; }
        Hdr h;
        if (!hdr_tag(h, kLiteral, end - st)) { o.err = EZ_EINVAL; return; }
        put_hdr(o, h, lane);
        if (o.err) return;
        if (o.op + (end - st) > o.cap) { o.err = EZ_ENOSPC; return; }
        if (lane == 0 && end > st) A.spec_lit[atomicAdd(A.spec_nlit, 1u)] = SpecLit{ib + (uint64_t)st, A.out_off[s] + (uint64_t)o.op, (uint64_t)(end - st)};
        o.op += end - st;
    };
    bool stopped = false;  // spec_mode 1: stopped after one accepted copy
    for (;;) {  // the stream's Writes (one unless mw)
        I done = smode ? (I)A.spec[s].done : 0;
        I i = smode == 1 ? (I)A.spec_first[s] : (smode == 2 ? (I)A.spec[s].from : 0);
        int64_t guard = 0;
        const int64_t guard_max = 16 * n + 4096;
        // global input: the 16 bytes x-8 .. x+7 around each lane's position, and those of
        // the window after this one if nothing is accepted (loaded while this one is judged)
        const bool pf = !PL && in_hi - in_lo >= 16;
        auto around = [&](I y) -> V16 {
            uint64_t wa;
            if (P.inw(y - 8, 16, wa)) return P.wv16(wa);
            const uint8_t *q = P.g + y - 8;
            return q >= in_lo && q + 16 <= in_hi ? ld16v(q) : ld_clamped(q, in_lo, in_hi);
        };
        V16 nxt_w{0, 0};
        I nxt_i = -1;
        const bool usefp = FP && pf && start == 0 && smode != 1;
        if (usefp) {
            if (smode == 2) {  // K1x's table: the bytes around each entry's position
#pragma unroll 4
                for (I k = lane; k < hs; k += kWave) fp[k] = around((I)ht[k]);
            } else {  // the zero entries hold stream position 0
                const V16 z = around(0);
                for (I k = lane; k < hs; k += kWave) fp[k] = z;
            }
            __syncthreads();
        }

#if (EZ_EXP & 64)  // phase timers (debug): cycles per phase, events, iterations; stream 0 prints them
        uint64_t tph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = clock64(), nit = 0, nev = 0;
#define EZ_T(k) do { const uint64_t t_ = clock64(); tph[k] += t_ - tlast; tlast = t_; } while (0)
#else
#define EZ_T(k) do {} while (0)
#endif
        while (i + 4 <= n && !o.err) {
            if (++guard > guard_max) { o.err = EZ_ESTUCK; break; }
#if (EZ_EXP & 64)
            nit++;
#endif
            if (wl) {  // the window holds [i - 64, i + 192) unless it already reaches the end
                const int64_t wlo = P.wa0 - (int64_t)P.gr, whi = wlo + (int64_t)P.wnb;
                if (P.ww == nullptr || (i + 192 > whi && !wend) || (i - 64 < wlo && wlo > 0)) {
                    wend = false;
                    refill(i > 512 ? i - 512 : 0);
                }
            }
            const I wpos = start + done;
            const I rem = n - 3 - i;
            const int nvalid = rem < kWave ? (int)rem : kWave;
            const I x = i + lane;
            const bool valid = lane < nvalid;
            V16 cur{0, 0};  // bytes x-8 .. x+7 (pf)
            if (pf) {
                if (wl) {  // LDS window: no prefetch (an LDS read is short)
                    cur = around(x);
                } else {
                    cur = nxt_i == i ? nxt_w : around(x);
                    nxt_w = around(x + nvalid);
                    nxt_i = i + nvalid;
                }
            }

            EZ_T(0);
            // -- hash + intra-window predecessor / successor with the same hash
            uint32_t h = 0xffffffffu;
            if (valid) h = ((pf ? (uint32_t)cur.hi : P.u32(x)) * kHashMul) >> hsh;
            // the lanes with this lane's hash: one ballot per hash bit (no LDS, no atomics: a zero
            // run puts most lanes of a window on one hash, C4s)
            uint64_t same = wballot(valid);
            for (unsigned bit = 0; bit < 32u - hsh; bit++) {
                const bool v = (h >> bit) & 1u;
                const uint64_t bb = wballot(v);
                same &= v ? bb : ~bb;
            }
            int prev = -1, next = kWave;
            if (valid) {
                const uint64_t below = same & ((1ull << lane) - 1);
                const uint64_t above = lane == 63 ? 0ull : (same & (~0ull << (lane + 1)));
                if (below) prev = 63 - __builtin_clzll(below);
                if (above) next = __builtin_ctzll(above);
            }
            I cand = 0;
            if (valid) cand = prev >= 0 ? (I)(uint32_t)(start + i + prev) : (I)ht[h];
            // the candidate's bytes cand-8 .. cand+7 (usefp): an earlier lane's, or the table's
            V16 cv{0, 0};
            if (usefp) {
                const int src = prev >= 0 ? prev : lane;
                const V16 pv{(uint64_t)__shfl((long long)cur.lo, src, 64), (uint64_t)__shfl((long long)cur.hi, src, 64)};
                if (valid) cv = prev >= 0 ? pv : fp[h];
            }

            EZ_T(1);
            // -- per-lane capped evaluation
            int kind = kReject;
            bool exact = true;
            I v_st = 0, v_ist = 0, v_iend = 0;
            if (valid) {
                const I off = cand - wpos;
                if (-off > bs) {
                    kind = kReject;  // far skip (writer.go:221-224)
                } else if (off >= 0 && x > done + off) {
                    // runlen (writer.go:227-231 -> writeRunlen :441-489)
                    const I st = done + off;
                    v_st = st;
                    if (st + 8 < n && (usefp ? cv.hi == 0 : (P.u32(st) == 0 && P.u32(st + 4) == 0))) {
                        kind = kZero;
                    } else {
                        int f = 0, c = 0;
                        if (!PL && kCap == 8) {  // 8-byte compares (writeRunlen :449-462, capped)
                            const uint64_t df = (usefp ? cv.hi : s8(st)) ^ (pf ? cur.hi : s8(x));
                            const uint64_t db = (usefp ? cv.lo : s8(st - 8)) ^ (pf ? cur.lo : s8(x - 8));
                            f = df ? (int)(__builtin_ctzll(df) >> 3) : 8;
                            if (f > n - x) f = (int)(n - x);
                            c = db ? (int)(__builtin_clzll(db) >> 3) : 8;
                            const I cl = st < x - done ? st : x - done;
                            if (c > cl) c = (int)cl;
                        } else {
                            while (f < kCap && x + f < n && P.b(st + f) == P.b(x + f)) f++;
                            while (c < kCap && st - 1 - c >= 0 && x - 1 - c >= done && P.b(st - 1 - c) == P.b(x - 1 - c)) c++;
                        }
                        const bool capped = f == kCap || c == kCap;
                        if (!capped && f + c < kMinCopyChunk) kind = kReject;
                        else if (x - st >= bs - 8) kind = kCut;
                        else { kind = kRun; exact = !capped; v_ist = x - c; v_iend = x + f; }
                    }
                } else {
                    // window match (writer.go:233-301)
                    I ist = x - 1, st = cand - 1;
                    int c = 0;
                    uint64_t rb = 0, rf = 0;
                    bool vec;
                    if (usefp && cand - 8 >= start && cand + 8 <= wpos && cand - 8 >= wpos - bs) {
                        rb = cv.lo;  // block[y & mask] is stream byte y for wpos - bs <= y < wpos
                        rf = cv.hi;
                        vec = true;
                    } else {
                        vec = !PL && kCap == 8 && ring8(cand - 8, wpos, rb) && ring8(cand, wpos, rf);
                    }
                    if (vec) {  // 8-byte compares against the ring image (writer.go:236-259, capped)
                        const uint64_t db = (pf ? cur.lo : s8(x - 8)) ^ rb;
                        c = db ? (int)(__builtin_clzll(db) >> 3) : 8;
                        if (c > x - done) c = (int)(x - done);
                        ist -= c;
                        st -= c;
                    } else {
                        while (c < kCap && ist >= done && P.b(ist) == ringb(st, wpos)) { ist--; st--; c++; }
                    }
                    ist++; st++;
                    I iend = x, end = cand;
                    int f = 0;
                    if (vec) {
                        const uint64_t df = (pf ? cur.hi : s8(x)) ^ rf;
                        f = df ? (int)(__builtin_ctzll(df) >> 3) : 8;
                        if (f > n - x) f = (int)(n - x);
                        iend += f;
                        end += f;
                    } else {
                        while (f < kCap && iend < n && P.b(iend) == ringb(end, wpos)) { iend++; end++; f++; }
                    }
                    const bool capped = c == kCap || f == kCap;
                    const int64_t blit = wpos - bs;
                    const int64_t bend = blit + (iend - done);
                    int64_t d = bend - st;
                    if (d > 0) { end -= d; iend -= d; }
                    d = (end - bs) - blit;
                    if (d > 0) { end -= d; iend -= d; }
                    if (end - st >= kMinCopyChunk) { kind = kWin; exact = !capped; v_ist = ist; v_iend = iend; }
                    else if (capped) { kind = kWin; exact = false; }
                    else kind = kReject;
                }
            }

            EZ_T(2);
            // -- first lane that accepts (exact resolution, wave-wide)
            uint64_t cm = wballot(valid && kind != kReject);
            const uint64_t exm = wballot(exact);
            int a = -1, ka = kReject;
            I xa = 0, sta = 0, ista = 0, ienda = 0, canda = 0;
            while (cm) {
                const int l = ffs64(cm);
                const int kl = rl32(kind, l);
                const bool ex = (exm >> l) & 1;
                const I xl = i + l;
                if (kl == kWin) {
                    const I cl = rl64(cand, l);
                    I ist, iend;
                    if (ex) {
                        ist = rl64(v_ist, l);
                        iend = rl64(v_iend, l);
                    } else {
                        const I bw = coop_count((I)0, lane, [&](I m) {
                            return xl - 1 - m >= done && P.b(xl - 1 - m) == ringb(cl - 1 - m, wpos);
                        });
                        const I fw = coop_count((I)0, lane, [&](I m) {
                            return xl + m < n && P.b(xl + m) == ringb(cl + m, wpos);
                        });
                        ist = xl - bw;
                        I st = cl - bw;
                        iend = xl + fw;
                        I end = cl + fw;
                        const int64_t blit = wpos - bs;
                        const int64_t bend = blit + (iend - done);
                        int64_t d = bend - st;
                        if (d > 0) { end -= d; iend -= d; }
                        d = (end - bs) - blit;
                        if (d > 0) { end -= d; iend -= d; }
                        if (end - st < kMinCopyChunk) { cm &= cm - 1; continue; }  // maybe -> reject
                    }
                    a = l; ka = kWin; xa = xl; canda = cl; ista = ist; ienda = iend;
                    break;
                }
                a = l; ka = kl; xa = xl; sta = rl64(v_st, l);
                if (kl == kRun) {
                    if (ex) {
                        ista = rl64(v_ist, l);
                        ienda = rl64(v_iend, l);
                    } else {
                        const I jf = coop_count((I)0, lane, [&](I m) {
                            return xl + m < n && P.b(sta + m) == P.b(xl + m);
                        });
                        const I jb = coop_count((I)0, lane, [&](I m) {
                            return sta - 1 - m >= 0 && xl - 1 - m >= done && P.b(sta - 1 - m) == P.b(xl - 1 - m);
                        });
                        ista = xl - jb;
                        ienda = xl + jf;
                    }
                }
                break;
            }

            EZ_T(3);
            // -- hash inserts of the visited lanes 0..last, last writer wins (writer.go:216-217)
            const int last = a < 0 ? nvalid - 1 : a;
            if (valid && lane <= last && next > last) {
                ht[h] = (uint32_t)(start + x);
                if (usefp) fp[h] = cur;
            }
            __syncthreads();

            EZ_T(4);
            if (a < 0) { i += nvalid; continue; }

            // -- lane a's action
            if (ka == kWin) {
                // writer.go:303-321
                if (done < ista) literal(done, ista);
                const I dist = start + xa - canda;  // w.pos - st after the literal
                const I L = ienda - ista;
                if (dist > bs) { o.err = EZ_EINVAL; break; }  // panic("too big offset")
                Hdr hh;
                if (!hdr_tag(hh, kCopy, L) || !hdr_offset(hh, dist, L)) { o.err = EZ_EINVAL; break; }
                put_hdr(o, hh, lane);
                if (xa + 1 + 4 <= n) {
                    const uint32_t h1 = (P.u32(xa + 1) * kHashMul) >> hsh;
                    V16 c1{0, 0};
                    if (usefp) {
                        const int src = a + 1 < kWave ? a + 1 : a;
                        c1 = V16{(uint64_t)__shfl((long long)cur.lo, src, 64), (uint64_t)__shfl((long long)cur.hi, src, 64)};
                        if (a + 1 >= kWave) c1 = around(xa + 1);
                    }
                    if (lane == 0) {
                        ht[h1] = (uint32_t)(start + xa + 1);
                        if (usefp) fp[h1] = c1;
                    }
                    __syncthreads();
                }
                i = ienda;
                done = ienda;
            } else if (ka == kRun) {
                // writer.go:477-488 (the literal is unconditional: SURVEY A.6)
                literal(done, ista);
                Hdr hh;
                if (!hdr_tag(hh, kCopy, ienda - ista) || !hdr_offset(hh, xa - sta, ienda - ista)) { o.err = EZ_EINVAL; break; }
                put_hdr(o, hh, lane);
                i = ienda;
                done = ienda;
            } else if (ka == kCut) {
                // writer.go:464-473
                const I iend = done + xa - sta;
                literal(done, iend);
                i = iend;
                done = iend;
            } else {
                // writeZeros writer.go:407-439, called with i = st
                const I zf = coop_count((I)0, lane, [&](I m) { return sta + m < n && P.b(sta + m) == 0; });
                const I zb = coop_count((I)0, lane, [&](I m) { return sta - 1 - m >= done && P.b(sta - 1 - m) == 0; });
                const I zi = sta - zb, ziend = sta + zf;
                if (ziend - zi < kMinCopyChunk) {
                    i = zi + 1;  // unreachable: >= 8 zeros are guaranteed
                } else {
                    if (done != zi) literal(done, zi);
                    Hdr hh;
                    if (!hdr_tag(hh, kCopy, ziend - zi)) { o.err = EZ_EINVAL; break; }
                    hh.put(kOffLong);
                    hh.put(0);
                    put_hdr(o, hh, lane);
                    i = ziend;
                    done = ziend;
                }
            }
            EZ_T(5);
#if (EZ_EXP & 64)
            nev++;
#endif
            // spec_mode 1: one emitting position resolved; K1x speculates again from here
            if (smode == 1 && i + 4 <= n && !o.err) {
                stopped = true;
                break;
            }
        }
#if (EZ_EXP & 64)
        if (lane == 0 && s == 0)
            printf("K1 phases (cycles): refill+win %llu hash %llu eval %llu resolve %llu insert %llu action %llu; iters %llu events %llu\n",
                   (unsigned long long)tph[0], (unsigned long long)tph[1], (unsigned long long)tph[2], (unsigned long long)tph[3],
                   (unsigned long long)tph[4], (unsigned long long)tph[5], (unsigned long long)nit, (unsigned long long)nev);
#endif
        if (stopped) {  // K1x's state back: the position, the pending literal, the output, the table
            if (lane == 0) A.spec[s] = SpecState{(uint32_t)i, (uint32_t)done, (uint32_t)o.op, 0u};
            if (HTL) for (I k = lane; k < hs; k += kWave) A.spec_tab[s * (uint64_t)hs + k] = ht[k];
            return;
        }
        // trailing literal (writer.go:324-329)
        if (!o.err && done < n) literal(done, n);

        if (mw && A.write_out && lane == 0) A.write_out[wk] = (uint64_t)o.op;  // this Write's output ends here
        if (!mw || ++wk >= wlast || o.err) break;
        // the next Write: its bytes follow this one's in the batch
        start += n;
        wbeg = A.write_end[wk - 1];
        n = (I)(A.write_end[wk] - wbeg);
        P.g = A.in + wbeg;
        P.gr = (uint64_t)(uintptr_t)P.g & 3;
        P.gw = (const uint32_t *)(P.g - P.gr);
        P.glast = (P.gr + (uint64_t)n + 3) / 4;
        P.glast = P.glast ? P.glast - 1 : 0;
    }
    if (RING) {
        // copyData of this call's Writes into the ring (writer.go:529-535): the last bs bytes, the
        // earlier Writes' bytes lying before the last one's in the batch; and the hash table back to HBM
        I k0 = n > bs ? n - bs : 0;
        if (mw) k0 = n - bs > A.start - start ? n - bs : A.start - start;
        for (I k = k0 + lane; k < n; k += kWave) A.ring[(start + k) & mask] = (uint8_t)P.b(k);
        if (HTL) for (I k = lane; k < hs; k += kWave) A.ht_global[k] = ht[k];
    }
    if (lane == 0) {
        A.out_size[s] = (uint64_t)o.op;
        if (A.status) A.status[s] = o.err;
        if (smode) A.spec[s].flags = 1u;  // finished
    }
}

template <bool PL, bool HTL, bool RING, bool MWP>
__global__ __launch_bounds__(64) void k1_compress(CompressArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    for (uint64_t s = blockIdx.x; s < A.count; s += gridDim.x) {
        // K1x resumes: finished streams, and in mode 1 the ones without an emitting position
        if (!RING && A.spec_mode && (A.spec[s].flags != 0 || (A.spec_mode == 1 && A.spec_first[s] == 0xffffffffu))) continue;
        compress_stream<PL, HTL, RING, MWP>(A, s, smem);
        __syncthreads();
    }
}

template <bool PL, bool HTL, bool RING, bool MWP>
hipError_t launch_variant_w(const CompressArgs &a, hipStream_t st, size_t lds, unsigned grid) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_compress<PL, HTL, RING, MWP>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    hipLaunchKernelGGL((k1_compress<PL, HTL, RING, MWP>), dim3(grid), dim3(64), lds, st, a);
    return hipGetLastError();
}
template <bool PL, bool HTL, bool RING>
hipError_t launch_variant(const CompressArgs &a, hipStream_t st, size_t lds, unsigned grid) {
    // PL excludes multi-Write streams (the launcher), so its variants need no multi-Write code
    // (and the 64-bit-position code for fresh Writes of 2 GiB or more: SMALL needs < 2^31)
    if (!PL && (a.write_idx || a.max_len >= (1ull << 31) || a.max_len == 0)) return launch_variant_w<PL, HTL, RING, true>(a, st, lds, grid);
    return launch_variant_w<PL, HTL, RING, false>(a, st, lds, grid);
}

}  // namespace

uint64_t compress_scratch_words(const CompressArgs &a) {
    const char v = compress_variant(a);
    if (v == 's') return split_scratch_words(a);
    if (v == 'x') return (spec_scratch_bytes(a) + 3) / 4;
    if (v == 'l') return (long_scratch_bytes(a) + 3) / 4;
    if (a.hs <= kHtLdsMax) return 0;
    const uint64_t grid = a.count < 2048 ? a.count : 2048;
    return grid * (uint64_t)a.hs;
}

// K1 choice.  Fresh streams with 2n <= block and a table of at most 4096 entries take K1s
// (ez_compress_split.hip: the parse kernel + the token writer); everything else -- writer handles
// (rings), Writes longer than half the window (C4), large tables -- takes the general
// wave-per-stream kernel below, after K1x's rounds (ez_compress_spec.hip) for fresh single-Write
// streams of 64 KiB and more.  EZ_K1=general or ez_select_compress_kernel('w') forces the general
// kernel alone, 'x' K1x for any fresh single-Write batch with a table of at most 4096 entries
// (tests, A/B).
static std::atomic<int> g_forced_variant{-1};  // -1: not read yet; 0: automatic; else the kernel's letter
void select_compress_variant(int v) { g_forced_variant = v; }

static int forced_variant() {
    int forced = g_forced_variant.load();
    if (forced < 0) {
        const char *e = knob_str("EZ_K1");
        const int f = e && std::string(e) == "general" ? 'w' : (e && std::string(e) == "long" ? 'l' : 0);
        (void)g_forced_variant.compare_exchange_strong(forced, f);
        forced = g_forced_variant.load();
    }
    return forced;
}

char compress_variant(const CompressArgs &a) {
    const int forced = forced_variant();
    if (forced == 'w') return 'w';
    if (forced == 'l' && long_applies(a)) return 'l';  // K1L alone (tests, A/B)
    if (split_stride_words(a) != 0 && forced != 'x') return 's';
    return spec_applies(a, forced == 'x') ? 'x' : 'w';
}

bool compress_forced_general() { return forced_variant() == 'w'; }
bool compress_forced_long() { return forced_variant() == 'l'; }

hipError_t launch_compress(const CompressArgs &a, hipStream_t st) {
    if (a.count == 0) return hipSuccess;
    const char v = compress_variant(a);
    if (v == 's') return launch_compress_split(a, a.ht_global, st);
    // long fresh streams: K1x rounds, which call the general kernel to resolve emitting positions
    if (v == 'x') return launch_compress_spec(a, (uint8_t *)a.ht_global, st);
    if (v == 'l') return launch_long(a, (uint8_t *)a.ht_global, st);
    return launch_general(a, st);
}

hipError_t launch_general(const CompressArgs &a, hipStream_t st) {
    const bool htl = a.hs <= kHtLdsMax;
    const bool pl = a.max_len > 0 && (int64_t)a.max_len <= kPLdsMax && !a.write_idx;  // multi-Write: the global view
    const bool ring = a.ring != nullptr;
    size_t lds = (htl ? (size_t)a.hs * 4 : 0) + kMaskBytes + kHashBytes;
    if (pl) lds += ((a.max_len + 3) / 4 + 8) * 4;
    if (htl && !ring && !pl) lds += (size_t)a.hs * 16;  // candidate fingerprints
    lds = (lds + 15) & ~(size_t)15;
    CompressArgs b = a;
    b.win_bytes = 0;
    if (!ring && !pl && !a.write_idx && a.max_len > (uint64_t)kPLdsMax) {  // long streams: the LDS window
        static const uint32_t w = (uint32_t)knob("EZ_K1W_WIN", (int)kWinBytes) & ~15u;
        b.win_bytes = w;
        if (w) lds += w + 32;
    }
    uint64_t grid = a.count;
    if (!htl && !ring) grid = grid < 2048 ? grid : 2048;  // global scratch hash tables
    if (grid > (1u << 30)) grid = 1u << 30;
    const unsigned g = (unsigned)grid;
    if (pl) {
        if (htl) return ring ? launch_variant<true, true, true>(b, st, lds, g) : launch_variant<true, true, false>(b, st, lds, g);
        return ring ? launch_variant<true, false, true>(b, st, lds, g) : launch_variant<true, false, false>(b, st, lds, g);
    }
    if (htl) return ring ? launch_variant<false, true, true>(b, st, lds, g) : launch_variant<false, true, false>(b, st, lds, g);
    return ring ? launch_variant<false, false, true>(b, st, lds, g) : launch_variant<false, false, false>(b, st, lds, g);
}

}  // namespace ez
