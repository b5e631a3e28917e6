// ez_compress_fresh.hip — K1f: batch compression of fresh streams on gfx950.
//
// Same algorithm and bytes as k1_compress (ez_compress.hip: the speculative
// window restatement of Writer.Write, writer.go:206-337), specialised for
// the batch case every BASELINE config uses: a fresh NewWriter per stream
// (zero ring, zero hash table, w.pos = 0) and a Write no longer than the
// window (n <= block).  Then block[y & mask] seen at w.pos == done is simply
// p[y] for 0 <= y < done and 0 otherwise (SURVEY A.8 with start = 0), no
// candidate is ever far-skipped (-off <= done <= n <= block), and every
// position fits 32 bits.
//
// G lanes work on one stream (64/G streams per wave, template G):
//   * a window is G consecutive positions; lane j hashes i+j and takes the
//     latest earlier lane of its group with the same hash (per-group LDS
//     bucket masks + exact check) or ht[hash];
//   * the branch is judged per lane with 8-byte compares (xor + clz/ctz)
//     forward and backward; acceptance is monotone in both lengths, so an
//     8-byte-capped answer is reject / accept / maybe;
//   * the group's first non-reject lane is resolved exactly with 4G-byte
//     cooperative steps (dword compares, ballot, first mismatch);
//   * inserts of lanes <= a (last writer wins), then the action; the group
//     writes its token bytes (literal header, literal, copy header) together.
// Streams are staged in LDS with 8 zero bytes on both sides.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"

namespace ez {
namespace {

constexpr int kNB = 64;  // bucket masks per stream

enum : int { kRej = 0, kWinK = 1, kRunK = 2, kCutK = 3, kZeroK = 4 };

template <int G>
struct GT {
    static constexpr int NG = 64 / G;
    static constexpr uint64_t GM = G == 64 ? ~0ull : ((1ull << G) - 1);
};

template <int G>
__device__ __forceinline__ uint64_t gball(bool p, int g) {
    const uint64_t m = (uint64_t)__ballot(p);
    if constexpr (G == 64) return m;
    else return (m >> (g * G)) & GT<G>::GM;
}

// value of lane a of this lane's group
template <int G>
__device__ __forceinline__ int32_t gbc(int32_t v, int g, int a) {
    if constexpr (G == 64) return __builtin_amdgcn_readlane(v, a);
    else return __shfl(v, g * G + a, 64);
}

// P view: byte y of the stream at LDS byte address pb + y (8 zero bytes on both sides)
struct PV {
    const uint32_t *w;  // LDS words
    uint32_t pb;        // byte address of y = 0 inside w
    __device__ __forceinline__ uint32_t b(int32_t y) const { return ((const uint8_t *)w)[pb + y]; }
    __device__ __forceinline__ uint32_t u32(int32_t y) const { return words_u32(w, (uint32_t)(pb + y)); }
    __device__ __forceinline__ uint64_t u64(int32_t y) const {
        const uint32_t a = pb + y;
        const uint32_t k = a >> 2, sh = a & 3;
        const uint32_t w0 = w[k], w1 = w[k + 1], w2 = w[k + 2];
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
               ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    }
};

// keep the low `k` bytes of x (k in [0, 8])
__device__ __forceinline__ uint64_t low_bytes(uint64_t x, int32_t k) {
    return k >= 8 ? x : (k <= 0 ? 0ull : (x & ((1ull << (8 * k)) - 1)));
}

// 8 ring bytes at y0.. (fresh stream): p[y] for 0 <= y < done, else 0
__device__ __forceinline__ uint64_t ring64(const PV &P, int32_t y0, int32_t done) {
    // y0 >= -8 is guaranteed by the callers (the zero pad covers y in [-8, 0))
    return low_bytes(P.u64(y0), done - y0);
}

__device__ __forceinline__ int32_t ctz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_ctzll(d) >> 3) : 8; }
__device__ __forceinline__ int32_t clz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_clzll(d) >> 3) : 8; }

// Writer writes into a group: bytes [lit header | p[src..src+L) | copy header]
__device__ __forceinline__ uint32_t hbyte(const Hdr &h, int32_t k) { return h.byte(k); }

template <int G>
__device__ __forceinline__ void emit(uint8_t *out, int32_t &op, int32_t cap, int &err, const PV &P, const Hdr &lh,
                                     int32_t src, int32_t L, const Hdr &ch, int lj) {
    const int32_t T = lh.n + L + ch.n;
    if (err) return;
    if (op + T > cap) { err = EZ_ENOSPC; return; }
    uint8_t *d = out + op;
    for (int32_t k = lj; k < T; k += G) {
        uint32_t v;
        if (k < lh.n) v = hbyte(lh, k);
        else if (k < lh.n + L) v = P.b(src + k - lh.n);
        else v = hbyte(ch, k - lh.n - L);
        d[k] = (uint8_t)v;
    }
    op += T;
}

// group-cooperative count of consecutive byte matches, 4G bytes per step.
// fwd: bytes a[k], b[k] for k = from..; bwd: bytes a[-1-k], b[-1-k].
// va / vb produce 4 bytes at a byte offset relative to the anchor; lim caps the count.
template <int G, class FA, class FB>
__device__ __forceinline__ int32_t gcount_fwd(bool active, int g, int lj, int32_t from, int32_t lim, FA va, FB vb) {
    int32_t base = from;
    int32_t res = lim;
    bool run = active && from < lim;
    while (__ballot(run) != 0) {
        int32_t mb = 4;
        if (run) {
            const int32_t k = base + 4 * lj;
            if (k < lim) {
                const uint32_t d = va(k) ^ vb(k);
                mb = d ? (int32_t)(__builtin_ctz(d) >> 3) : 4;
                if (k + mb > lim) mb = lim - k;
                if (mb > 4) mb = 4;
            } else {
                mb = 0;
            }
        }
        const uint64_t bad = gball<G>(run && mb < 4, g);
        const int l = bad ? (int)__builtin_ctzll(bad) : 0;
        const int32_t mbl = gbc<G>(mb, g, l);  // every lane takes part in the broadcast
        if (run) {
            if (bad) {
                res = base + 4 * l + mbl;
                run = false;
            } else {
                base += 4 * G;
            }
        }
    }
    return res < lim ? res : lim;
}

template <int G, class FA, class FB>
__device__ __forceinline__ int32_t gcount_bwd(bool active, int g, int lj, int32_t from, int32_t lim, FA va, FB vb) {
    // va(k) / vb(k): the 4 bytes ending just below offset -k (i.e. bytes -k-4 .. -k-1), high byte = -k-1
    int32_t base = from;
    int32_t res = lim;
    bool run = active && from < lim;
    while (__ballot(run) != 0) {
        int32_t mb = 4;
        if (run) {
            const int32_t k = base + 4 * lj;
            if (k < lim) {
                const uint32_t d = va(k) ^ vb(k);
                mb = d ? (int32_t)(__builtin_clz(d) >> 3) : 4;
                if (k + mb > lim) mb = lim - k;
                if (mb > 4) mb = 4;
            } else {
                mb = 0;
            }
        }
        const uint64_t bad = gball<G>(run && mb < 4, g);
        const int l = bad ? (int)__builtin_ctzll(bad) : 0;
        const int32_t mbl = gbc<G>(mb, g, l);  // every lane takes part in the broadcast
        if (run) {
            if (bad) {
                res = base + 4 * l + mbl;
                run = false;
            } else {
                base += 4 * G;
            }
        }
    }
    return res < lim ? res : lim;
}

template <int G>
__global__ __launch_bounds__(256) void k1_fresh(CompressArgs A, uint32_t stride_words) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NG = GT<G>::NG;
    const int lane = (int)(threadIdx.x & 63);
    const int wave = (int)(threadIdx.x >> 6);
    const int g = lane / G, lj = lane % G;
    const int32_t hs = (int32_t)A.hs;
    const int64_t bs = A.bs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));

    // per-stream LDS region: [ht hs*4][bm kNB*8][H G*4][P words]
    uint32_t *base = (uint32_t *)smem + (uint32_t)(wave * NG + g) * stride_words;
    uint32_t *ht = base;
    uint64_t *bm = (uint64_t *)(base + hs);
    uint32_t *H = base + hs + 2 * kNB;
    uint32_t *pw = base + hs + 2 * kNB + G;

    const uint64_t s = ((uint64_t)blockIdx.x * 4 + wave) * NG + g;
    const bool have = s < A.count;
    int32_t n = 0;
    const uint8_t *gp = A.in;
    if (have) {
        n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        gp = A.in + A.in_off[s];
    }
    // ---- stage p: words aligned like the source, 8 zero bytes before and after
    const uint32_t r = (uint32_t)((uintptr_t)gp & 3);
    const uint32_t *gw = (const uint32_t *)(gp - r);
    const int32_t nw = have ? (int32_t)((r + (uint32_t)n + 3) >> 2) : 0;
    PV P;
    P.w = pw;
    P.pb = 8 + r;
    if (lj < 2) pw[lj] = 0;
    for (int32_t k = lj; k < nw; k += G) {
        uint32_t v = gw[k];
        if (k == 0) v &= ~0u << (8 * r);  // bytes before the stream
        const int32_t y0 = 4 * k - (int32_t)r;  // stream offset of the word's byte 0
        if (y0 + 4 > n) v &= (n - y0) <= 0 ? 0u : (0xffffffffu >> (8 * (4 - (n - y0))));
        pw[2 + k] = v;
    }
    if (lj < 4) pw[2 + nw + lj] = 0;
    for (int32_t k = lj; k < hs; k += G) ht[k] = 0;
    for (int32_t k = lj; k < kNB; k += G) bm[k] = 0;

    uint8_t *out = have ? A.out + A.out_off[s] : A.out;
    const int32_t cap = have ? (int32_t)(A.out_off[s + 1] - A.out_off[s]) : 0;
    int32_t op = 0;
    int err = 0;
    {  // header (writer.go:495-517)
        Hdr h, none;
        if (A.append_magic) { h.put(0x80); h.put(0x02); h.put('e'); h.put('a'); h.put('z'); h.put('y'); }
        h.put(0x80); h.put(0x10); h.put((uint32_t)__builtin_ctzll((uint64_t)bs));
        if (have) emit<G>(out, op, cap, err, P, h, 0, 0, none, lj);
    }

    int32_t i = 0, done = 0;
    bool live = have && n >= 4;
    int32_t guard = 0;
    const int32_t guard_max = 16 * n + 4096;

    while (__ballot(live) != 0) {
        if (live && ++guard > guard_max) { err = EZ_ESTUCK; live = false; }
        const int32_t rem = n - 3 - i;
        const int32_t nvalid = rem < G ? rem : G;
        const int32_t x = i + lj;
        const bool valid = live && lj < nvalid;

        // ---- hash, intra-window predecessor / successor
        uint32_t h = 0;
        if (valid) h = (P.u32(x) * kHashMul) >> hsh;
        const int bk = (int)(h & (kNB - 1));
        if (valid) {
            atomicOr((unsigned long long *)&bm[bk], 1ull << lj);
            H[lj] = h;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        int prev = -1, next = G;
        if (valid) {
            const uint64_t m = bm[bk];
            uint64_t below = m & ((1ull << lj) - 1);
            while (below) {
                const int k = 63 - __builtin_clzll(below);
                if (H[k] == h) { prev = k; break; }
                below &= ~(1ull << k);
            }
            uint64_t above = lj == 63 ? 0ull : (m & (~0ull << (lj + 1)));
            while (above) {
                const int k = __builtin_ctzll(above);
                if (H[k] == h) { next = k; break; }
                above &= above - 1;
            }
        }
        int32_t cand = 0;
        if (valid) cand = prev >= 0 ? i + prev : (int32_t)ht[h];

        // ---- per-lane capped evaluation (8 bytes each way)
        int kind = kRej;
        bool exact = true;
        int32_t v_a = 0, v_b = 0;  // window: ist, iend (after trims); run: c (back), f (fwd)
        if (valid) {
            if (cand >= done && cand < x) {
                // runlen (writer.go:227-231 -> writeRunlen :441-489), st = cand
                const int32_t st = cand;
                if (st + 8 < n && P.u64(st) == 0) {
                    kind = kZeroK;
                } else {
                    const int32_t flim = n - x;
                    int32_t f = ctz_bytes(P.u64(st) ^ P.u64(x));
                    const bool fcap = f >= 8 && flim > 8;
                    if (f > flim) f = flim;
                    const int32_t blim = (x - done) < st ? (x - done) : st;
                    int32_t c = clz_bytes(P.u64(st - 8) ^ P.u64(x - 8));
                    const bool ccap = c >= 8 && blim > 8;
                    if (c > blim) c = blim;
                    const bool capped = fcap || ccap;
                    if (!capped && f + c < kMinCopyChunk) kind = kRej;
                    else if ((int64_t)(x - st) >= bs - 8) kind = kCutK;
                    else { kind = kRunK; exact = !capped; v_a = c; v_b = f; }
                }
            } else {
                // window match (writer.go:233-301)
                const int32_t flim = n - x;
                int32_t f = ctz_bytes(P.u64(x) ^ ring64(P, cand, done));
                const bool fcap = f >= 8 && flim > 8;
                if (f > flim) f = flim;
                const int32_t blim = x - done;
                int32_t c = clz_bytes(P.u64(x - 8) ^ ring64(P, cand - 8, done));
                const bool ccap = c >= 8 && blim > 8;
                if (c > blim) c = blim;
                const bool capped = fcap || ccap;
                int32_t ist = x - c, iend = x + f;
                int64_t st = (int64_t)cand - c, end = (int64_t)cand + f;
                int64_t d = ((int64_t)done - bs + (iend - done)) - st;
                if (d > 0) { end -= d; iend -= (int32_t)d; }
                d = end - done;
                if (d > 0) { end -= d; iend -= (int32_t)d; }
                if (end - st >= kMinCopyChunk) { kind = kWinK; exact = !capped; v_a = ist; v_b = iend; }
                else if (capped) { kind = kWinK; exact = false; }
            }
        }

        // ---- resolve each group's first accepting lane
        uint64_t cm = gball<G>(valid && kind != kRej, g);
        const uint64_t exm = gball<G>(exact, g);
        int a = -1, ka = kRej;
        int32_t xa = 0, ca = 0, r1 = 0, r2 = 0;  // window: ist, iend; run: c, f; zero: zb, zf
        bool pending = live && cm != 0;
        while (__ballot(pending) != 0) {
            int l = 0, kl = kRej;
            bool ex = true;
            int32_t xl = 0, cl = 0, pa = 0, pb2 = 0;
            if (pending) {
                l = (int)__builtin_ctzll(cm);
            }
            // broadcasts (every lane takes part)
            kl = gbc<G>(kind, g, l);
            cl = gbc<G>(cand, g, l);
            pa = gbc<G>(v_a, g, l);
            pb2 = gbc<G>(v_b, g, l);
            ex = (exm >> l) & 1;
            xl = i + l;
            const bool need_win = pending && kl == kWinK && !ex;
            const bool need_run = pending && kl == kRunK && !ex;
            const bool need_zero = pending && kl == kZeroK;
            // window: exact backward / forward extension against the ring
            const int32_t wb = gcount_bwd<G>(need_win, g, lj, 0, xl - done,
                [&](int32_t k) { return P.u32(xl - k - 4); },
                [&](int32_t k) {
                    const int32_t y0 = cl - k - 4;
                    if (y0 + 4 <= 0) return 0u;
                    uint32_t v = y0 >= 0 ? P.u32(y0) : (P.u32(0) << (8 * (-y0)));
                    const int32_t keep = done - y0;  // bytes y < done survive
                    if (keep < 4) v = keep <= 0 ? 0u : (v & (0xffffffffu >> (8 * (4 - keep))));
                    return v;
                });
            const int32_t wf = gcount_fwd<G>(need_win, g, lj, 0, n - xl,
                [&](int32_t k) { return P.u32(xl + k); },
                [&](int32_t k) {
                    const int32_t y0 = cl + k;
                    if (y0 >= done) return 0u;
                    uint32_t v = P.u32(y0);
                    const int32_t keep = done - y0;
                    if (keep < 4) v = keep <= 0 ? 0u : (v & (0xffffffffu >> (8 * (4 - keep))));
                    return v;
                });
            // runlen: exact jf / jb (st = cl)
            const int32_t rbl = (xl - done) < cl ? (xl - done) : cl;
            const int32_t rb = gcount_bwd<G>(need_run, g, lj, 0, rbl,
                [&](int32_t k) { return P.u32(xl - k - 4); }, [&](int32_t k) { return P.u32(cl - k - 4); });
            const int32_t rf = gcount_fwd<G>(need_run, g, lj, 0, n - xl,
                [&](int32_t k) { return P.u32(xl + k); }, [&](int32_t k) { return P.u32(cl + k); });
            // zero run from st = cl: forward zeros, backward zeros down to done
            const int32_t zf = gcount_fwd<G>(need_zero, g, lj, 0, n - cl,
                [&](int32_t k) { return P.u32(cl + k); }, [&](int32_t) { return 0u; });
            const int32_t zb = gcount_bwd<G>(need_zero, g, lj, 0, cl - done,
                [&](int32_t k) { return P.u32(cl - k - 4); }, [&](int32_t) { return 0u; });
            if (pending) {
                bool take = true;
                int32_t t1 = pa, t2 = pb2;
                if (kl == kWinK && !ex) {
                    int32_t ist = xl - wb, iend = xl + wf;
                    int64_t st = (int64_t)cl - wb, end = (int64_t)cl + wf;
                    int64_t d = ((int64_t)done - bs + (iend - done)) - st;
                    if (d > 0) { end -= d; iend -= (int32_t)d; }
                    d = end - done;
                    if (d > 0) { end -= d; iend -= (int32_t)d; }
                    if (end - st >= kMinCopyChunk) { t1 = ist; t2 = iend; }
                    else take = false;  // maybe -> reject
                } else if (kl == kRunK && !ex) {
                    t1 = rb; t2 = rf;
                } else if (kl == kZeroK) {
                    t1 = zb; t2 = zf;
                }
                if (take) {
                    a = l; ka = kl; xa = xl; ca = cl; r1 = t1; r2 = t2;
                    pending = false;
                } else {
                    cm &= cm - 1;
                    pending = cm != 0;
                }
            }
        }

        // ---- inserts of lanes 0..last (writer.go:216-217), last writer wins
        const int last = a < 0 ? nvalid - 1 : a;
        if (valid && lj <= last && next > last) ht[h] = (uint32_t)x;
        if (valid) bm[bk] = 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ---- the group's action
        if (live) {
            if (a < 0) {
                i += nvalid;
            } else {
                Hdr lh, ch;
                int32_t lsrc = done, llen = 0;
                bool lit = false;
                int32_t ni = 0, nd = 0;
                if (ka == kWinK) {
                    // writer.go:303-321
                    const int32_t ist = r1, iend = r2;
                    if (done < ist) { lit = true; llen = ist - done; }
                    const int32_t L = iend - ist;
                    const int32_t dist = xa - ca;  // w.pos - st after the literal
                    if ((int64_t)dist > bs) err = EZ_EINVAL;
                    hdr_tag(ch, kCopy, L);
                    hdr_offset(ch, dist, L);
                    ni = nd = iend;
                } else if (ka == kRunK) {
                    // writer.go:477-488 (the literal is unconditional: SURVEY A.6)
                    const int32_t ist = xa - r1, iend = xa + r2;
                    lit = true;
                    llen = ist - done;
                    hdr_tag(ch, kCopy, iend - ist);
                    hdr_offset(ch, xa - ca, iend - ist);
                    ni = nd = iend;
                } else if (ka == kCutK) {
                    // writer.go:464-473
                    lit = true;
                    llen = xa - ca;
                    ni = nd = done + llen;
                } else {
                    // writeZeros writer.go:407-439, called with i = st = ca
                    const int32_t zi = ca - r1, ziend = ca + r2;
                    if (ziend - zi < kMinCopyChunk) {
                        ni = zi + 1;  // unreachable (>= 8 zeros are guaranteed)
                        nd = done;
                    } else {
                        if (done != zi) { lit = true; llen = zi - done; }
                        hdr_tag(ch, kCopy, ziend - zi);
                        ch.put(kOffLong);
                        ch.put(0);
                        ni = nd = ziend;
                    }
                }
                if (lit) hdr_tag(lh, kLiteral, llen);
                if (!err) emit<G>(out, op, cap, err, P, lh, lsrc, llen, ch, lj);
                // the extra insert of i+1 after a window match (writer.go:315-318)
                if (ka == kWinK && xa + 1 + 4 <= n && lj == 0) {
                    const uint32_t h1 = (P.u32(xa + 1) * kHashMul) >> hsh;
                    ht[h1] = (uint32_t)(xa + 1);
                }
                i = ni;
                done = nd;
            }
            if (err || i + 4 > n) live = false;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    // trailing literal (writer.go:324-329)
    if (have && !err && done < n) {
        Hdr lh, none;
        hdr_tag(lh, kLiteral, n - done);
        emit<G>(out, op, cap, err, P, lh, done, n - done, none, lj);
    }
    if (have && lj == 0) {
        A.out_size[s] = (uint64_t)op;
        if (A.status) A.status[s] = err;
    }
}

}  // namespace

// LDS words per stream for the fresh kernel (0 = the fresh kernel cannot take this launch)
uint32_t fresh_stride_words(const CompressArgs &a, int G) {
    if (a.ring || a.max_len == 0 || (int64_t)a.max_len > a.bs || a.max_len > (1u << 20) || a.hs > 4096) return 0;
    const uint64_t pwords = 2 + (a.max_len + 3) / 4 + 1 + 4;
    uint64_t w = (uint64_t)a.hs + 2 * kNB + G + pwords;
    w = (w + 3) & ~3ull;
    if (w * 4 * (64 / G) * 4 > 160 * 1024) return 0;  // a 4-wave block must fit the CU's LDS
    return (uint32_t)w;
}

hipError_t launch_compress_fresh(const CompressArgs &a, hipStream_t st, int G) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_fresh<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k1_fresh<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k1_fresh<64>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const uint32_t stride = fresh_stride_words(a, G);
    const uint64_t per_block = (uint64_t)(64 / G) * 4;
    const unsigned grid = (unsigned)((a.count + per_block - 1) / per_block);
    const size_t lds = (size_t)stride * 4 * per_block;
    switch (G) {
    case 16: hipLaunchKernelGGL(k1_fresh<16>, dim3(grid), dim3(256), lds, st, a, stride); break;
    case 32: hipLaunchKernelGGL(k1_fresh<32>, dim3(grid), dim3(256), lds, st, a, stride); break;
    default: hipLaunchKernelGGL(k1_fresh<64>, dim3(grid), dim3(256), lds, st, a, stride); break;
    }
    return hipGetLastError();
}

}  // namespace ez
