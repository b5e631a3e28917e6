// ez_compress_fresh.hip — K1f: batch compression of fresh streams on gfx950.
//
// Same algorithm and bytes as k1_compress (ez_compress.hip: the speculative
// window restatement of Writer.Write, writer.go:206-337), specialised for
// the batch case every BASELINE config uses: a fresh NewWriter per stream
// (zero ring, zero hash table, w.pos = 0) and a Write no longer than the
// window (2n <= block), staged in LDS.  Then block[y & mask] seen at
// w.pos == done is simply p[y] for 0 <= y < done and 0 otherwise
// (SURVEY A.8 with start = 0), no candidate is ever far-skipped
// (-off <= done <= n <= block), and positions fit 16 bits (n < 65536), so
// the hash table is u16 — half the LDS a u32 table needs.
//
// One wave per stream, scalar (SGPR) control:
//   * a window is up to 64 consecutive positions i..i+63, one per lane;
//   * duplicate hashes inside a window: lane j's candidate is the latest
//     earlier lane of the window with the same hash, else ht[hash]; found
//     with 128 per-stream bucket masks (LDS atomic or) checked against the
//     lanes' u16 hashes;
//   * each lane judges its position with 8-byte compares forward and
//     backward (xor + ctz/clz); acceptance is monotone in both lengths, so
//     a capped answer is reject / accept / maybe;
//   * the first lane that can accept is resolved exactly with 256-byte
//     wave-wide steps; inserts of the lanes up to it, then its action.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"

namespace ez {
namespace {

enum : int { kRej = 0, kWinK = 1, kRunK = 2, kCutK = 3, kZeroK = 4 };

// P view: byte y of the stream at LDS byte address pb + y (>= 8 zero bytes on both sides)
struct PV {
    const uint32_t *w;  // LDS words
    uint32_t pb;        // byte address of y = 0 inside w
    __device__ __forceinline__ uint32_t b(int32_t y) const { return ((const uint8_t *)w)[pb + y]; }
    __device__ __forceinline__ uint32_t u32(int32_t y) const { return words_u32(w, (uint32_t)(pb + y)); }
    // 16 bytes y-8 .. y+7 as (before, from)
    __device__ __forceinline__ void around(int32_t y, uint64_t &before, uint64_t &from) const {
        const uint32_t a = pb + y - 8;
        const uint32_t k = a >> 2, sh = a & 3;
        const uint32_t w0 = w[k], w1 = w[k + 1], w2 = w[k + 2], w3 = w[k + 3], w4 = w[k + 4];
        before = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
        from = (uint64_t)__builtin_amdgcn_alignbyte(w3, w2, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w4, w3, sh) << 32);
    }
};

// keep the low `k` bytes of x (k may be outside [0, 8])
__device__ __forceinline__ uint64_t low_bytes(uint64_t x, int32_t k) {
    return k >= 8 ? x : (k <= 0 ? 0ull : (x & ((1ull << (8 * k)) - 1)));
}
__device__ __forceinline__ uint32_t low_bytes32(uint32_t x, int32_t k) {
    return k >= 4 ? x : (k <= 0 ? 0u : (x & (0xffffffffu >> (8 * (4 - k)))));
}
__device__ __forceinline__ int32_t ctz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_ctzll(d) >> 3) : 8; }
__device__ __forceinline__ int32_t clz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_clzll(d) >> 3) : 8; }

// wave-wide count of matching bytes, 256 per step, starting at `from` (< lim)
template <class FA, class FB>
__device__ __forceinline__ int32_t wcount_fwd(int lane, int32_t from, int32_t lim, FA va, FB vb) {
    for (int32_t base = from; base < lim; base += 256) {
        const int32_t k = base + 4 * lane;
        int32_t mb = 4;
        if (k < lim) {
            const uint32_t d = va(k) ^ vb(k);
            if (d) mb = (int32_t)(__builtin_ctz(d) >> 3);
            if (mb > lim - k) mb = lim - k;
        } else {
            mb = 0;
        }
        const uint64_t bad = wballot(mb < 4);
        if (bad) {
            const int l = ffs64(bad);
            const int32_t r = base + 4 * l + rl32(mb, l);
            return r < lim ? r : lim;
        }
    }
    return lim;
}

// backward: va(k) / vb(k) give the 4 bytes -k-4 .. -k-1 (the high byte is compared first)
template <class FA, class FB>
__device__ __forceinline__ int32_t wcount_bwd(int lane, int32_t from, int32_t lim, FA va, FB vb) {
    for (int32_t base = from; base < lim; base += 256) {
        const int32_t k = base + 4 * lane;
        int32_t mb = 4;
        if (k < lim) {
            const uint32_t d = va(k) ^ vb(k);
            if (d) mb = (int32_t)(__builtin_clz(d) >> 3);
            if (mb > lim - k) mb = lim - k;
        } else {
            mb = 0;
        }
        const uint64_t bad = wballot(mb < 4);
        if (bad) {
            const int l = ffs64(bad);
            const int32_t r = base + 4 * l + rl32(mb, l);
            return r < lim ? r : lim;
        }
    }
    return lim;
}

// writes [lit header | p[src..src+L) | copy header] at out+op
__device__ __forceinline__ void emit(uint8_t *out, int32_t &op, int32_t cap, int &err, const PV &P, const Hdr &lh,
                                     int32_t src, int32_t L, const Hdr &ch, int lane) {
    const int32_t T = lh.n + L + ch.n;
    if (op + T > cap) { err = EZ_ENOSPC; return; }
    uint8_t *d = out + op;
    const int32_t e1 = lh.n, e2 = lh.n + L;
    for (int32_t k = lane; k < T; k += kWave) {
        uint32_t v;
        if (k < e1) v = lh.byte(k);
        else if (k < e2) v = P.b(src + k - e1);
        else v = ch.byte(k - e2);
        d[k] = (uint8_t)v;
    }
    op += T;
}

__global__ __launch_bounds__(256) void k1_fresh(CompressArgs A, uint32_t stride_words, uint32_t ht_words) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int wave = (int)(threadIdx.x >> 6);
    const uint64_t s = (uint64_t)blockIdx.x * 4 + wave;
    if (s >= A.count) return;  // wave-uniform; the kernel uses no block barrier
    const int32_t hs = (int32_t)A.hs;
    const int64_t bs = A.bs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));

    // LDS: [ht u16 x hs][bucket masks u64 x 128][lane hashes u16 x 64][p words]
    uint32_t *base = (uint32_t *)smem + (uint32_t)wave * stride_words;
    uint16_t *ht = (uint16_t *)base;
    // volatile: lanes read what OTHER lanes stored (no store->load forwarding)
    volatile uint64_t *bm = (volatile uint64_t *)(base + ht_words);
    volatile uint16_t *H = (volatile uint16_t *)(base + ht_words + 256);
    uint32_t *pw = base + ht_words + 256 + 32;

    const int32_t n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint8_t *gp = A.in + A.in_off[s];
    // ---- stage p: words aligned like the source, 8 zero bytes before, >= 16 after
    const uint32_t r = (uint32_t)((uintptr_t)gp & 3);
    const uint32_t *gw = (const uint32_t *)(gp - r);
    const int32_t nw = (int32_t)((r + (uint32_t)n + 3) >> 2);
    PV P;
    P.w = pw;
    P.pb = 8 + r;
    if (lane < 2) pw[lane] = 0;
    for (int32_t k = lane; k < nw; k += kWave) {
        uint32_t v = gw[k];
        if (k == 0) v &= ~0u << (8 * r);        // bytes before the stream
        const int32_t y0 = 4 * k - (int32_t)r;  // stream offset of the word's byte 0
        v = low_bytes32(v, n - y0);             // bytes after the stream
        pw[2 + k] = v;
    }
    if (lane < 5) pw[2 + nw + lane] = 0;
    for (int32_t k = lane; k < (int32_t)ht_words; k += kWave) ((uint32_t *)ht)[k] = 0;
    for (int32_t k = lane; k < 128; k += kWave) bm[k] = 0;

    uint8_t *out = A.out + A.out_off[s];
    const int32_t cap = (int32_t)(A.out_off[s + 1] - A.out_off[s]);
    int32_t op = 0;
    int err = 0;
    {  // header (writer.go:495-517)
        Hdr h, none;
        if (A.append_magic) { h.put(0x80); h.put(0x02); h.put('e'); h.put('a'); h.put('z'); h.put('y'); }
        h.put(0x80); h.put(0x10); h.put((uint32_t)__builtin_ctzll((uint64_t)bs));
        emit(out, op, cap, err, P, h, 0, 0, none, lane);
    }

    int32_t i = 0, done = 0;
    int32_t guard = 16 * n + 4096;
    while (i + 4 <= n && !err) {
        if (--guard < 0) { err = EZ_ESTUCK; break; }
        int32_t nvalid = n - 3 - i;
        if (nvalid > kWave) nvalid = kWave;
        const int32_t x = i + lane;
        bool valid = lane < nvalid;

        // ---- hash (writer.go:491-493); the latest earlier lane with the same hash
        uint64_t pxb, pxf;
        P.around(x, pxb, pxf);
        const uint32_t h = ((uint32_t)pxf * kHashMul) >> hsh;
        const uint32_t bk = h & 127;
        if (valid) {
            atomicOr((unsigned long long *)&bm[bk], 1ull << lane);
            H[lane] = (uint16_t)h;
        }
        int prev = -1, next = kWave;
        if (valid) {
            const uint64_t m = bm[bk];
            uint64_t below = m & ((1ull << lane) - 1);
            while (below) {
                const int k = 63 - __builtin_clzll(below);
                if (H[k] == (uint16_t)h) { prev = k; break; }
                below &= ~(1ull << k);
            }
            uint64_t above = lane == 63 ? 0ull : (m & (~0ull << (lane + 1)));
            while (above) {
                const int k = __builtin_ctzll(above);
                if (H[k] == (uint16_t)h) { next = k; break; }
                above &= above - 1;
            }
        }
        const int32_t cand = valid ? (prev >= 0 ? i + prev : (int32_t)ht[h]) : 0;

        // ---- per-lane capped evaluation (8 bytes each way)
        int kind = kRej;
        bool exact = true;
        int32_t va = 0, vb = 0;  // window: ist, iend after trims; run: c (back), f (fwd)
        if (valid) {
            uint64_t pcb, pcf;
            P.around(cand, pcb, pcf);
            const bool run = cand >= done && cand < x;  // writer.go:227 with off = cand - done
            const int32_t flim = n - x;
            const int32_t fr = ctz_bytes(pxf ^ (run ? pcf : low_bytes(pcf, done - cand)));
            const int32_t f = fr < flim ? fr : flim;
            const int32_t blim = run ? ((x - done) < cand ? (x - done) : cand) : (x - done);
            const int32_t cr = clz_bytes(pxb ^ (run ? pcb : low_bytes(pcb, done - cand + 8)));
            const int32_t c = cr < blim ? cr : blim;
            const bool capped = (fr >= 8 && flim > 8) || (cr >= 8 && blim > 8);
            if (run) {
                // writeRunlen writer.go:441-489 (st = cand)
                if (cand + 8 < n && pcf == 0) kind = kZeroK;
                else if (!capped && f + c < kMinCopyChunk) kind = kRej;
                else if ((int64_t)(x - cand) >= bs - 8) kind = kCutK;
                else { kind = kRunK; exact = !capped; va = c; vb = f; }
            } else {
                // window match writer.go:233-301
                int32_t ist = x - c, iend = x + f;
                int64_t st = (int64_t)cand - c, end = (int64_t)cand + f;
                int64_t dd = ((int64_t)done - bs + (iend - done)) - st;
                if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
                dd = end - done;
                if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
                if (end - st >= kMinCopyChunk) { kind = kWinK; exact = !capped; va = ist; vb = iend; }
                else if (capped) { kind = kWinK; exact = false; }
            }
        }

        // ---- the first lane that accepts (exact resolution)
        uint64_t cm = wballot(kind != kRej);
        const uint64_t exm = wballot(exact);
        int a = -1, ka = kRej;
        int32_t xa = 0, ca = 0, r1 = 0, r2 = 0;
        while (cm) {
            const int l = ffs64(cm);
            const int kl = rl32(kind, l);
            const int32_t cl = rl32(cand, l);
            const int32_t xl = i + l;
            const bool ex = (exm >> l) & 1;
            int32_t t1 = rl32(va, l), t2 = rl32(vb, l);
            if (kl == kWinK && !ex) {
                const int32_t bw = wcount_bwd(lane, 0, xl - done,
                    [&](int32_t k) { return P.u32(xl - k - 4); },
                    [&](int32_t k) {
                        const int32_t y0 = cl - k - 4;  // ring bytes y0 .. y0+3: p[y] for 0 <= y < done
                        if (y0 + 4 <= 0 || y0 >= done) return 0u;
                        const uint32_t v = y0 >= 0 ? P.u32(y0) : (P.u32(0) << (8 * (-y0)));
                        return low_bytes32(v, done - y0);
                    });
                const int32_t fw = wcount_fwd(lane, 0, n - xl,
                    [&](int32_t k) { return P.u32(xl + k); },
                    [&](int32_t k) {
                        const int32_t y0 = cl + k;
                        if (y0 >= done) return 0u;
                        return low_bytes32(P.u32(y0), done - y0);
                    });
                int32_t ist = xl - bw, iend = xl + fw;
                int64_t st = (int64_t)cl - bw, end = (int64_t)cl + fw;
                int64_t dd = ((int64_t)done - bs + (iend - done)) - st;
                if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
                dd = end - done;
                if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
                if (end - st < kMinCopyChunk) { cm &= cm - 1; continue; }  // maybe -> reject
                t1 = ist;
                t2 = iend;
            } else if (kl == kRunK && !ex) {
                const int32_t rbl = (xl - done) < cl ? (xl - done) : cl;
                t1 = wcount_bwd(lane, 0, rbl, [&](int32_t k) { return P.u32(xl - k - 4); },
                                [&](int32_t k) { return P.u32(cl - k - 4); });
                t2 = wcount_fwd(lane, 0, n - xl, [&](int32_t k) { return P.u32(xl + k); },
                                [&](int32_t k) { return P.u32(cl + k); });
            } else if (kl == kZeroK) {
                t1 = wcount_bwd(lane, 0, cl - done, [&](int32_t k) { return P.u32(cl - k - 4); },
                                [&](int32_t) { return 0u; });
                t2 = wcount_fwd(lane, 8, n - cl, [&](int32_t k) { return P.u32(cl + k); },
                                [&](int32_t) { return 0u; });
            }
            a = l; ka = kl; xa = xl; ca = cl; r1 = t1; r2 = t2;
            break;
        }

        // ---- inserts of lanes 0..last (writer.go:216-217), last writer wins
        const int last = a < 0 ? nvalid - 1 : a;
        if (valid && lane <= last && next > last) ht[h] = (uint16_t)x;
        if (valid) bm[bk] = 0;
        if (a < 0) {
            i += nvalid;
            continue;
        }

        // ---- lane a's action
        Hdr lh, ch;
        int32_t llen = 0;
        bool lit = false;
        int32_t ni, nd;
        if (ka == kWinK) {
            // writer.go:303-321
            const int32_t ist = r1, iend = r2;
            if (done < ist) { lit = true; llen = ist - done; }
            const int32_t L = iend - ist;
            const int32_t dist = xa - ca;  // w.pos - st after the literal
            if ((int64_t)dist > bs) { err = EZ_EINVAL; break; }
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
        emit(out, op, cap, err, P, lh, done, llen, ch, lane);
        // the extra insert of i+1 after a window match (writer.go:315-318)
        if (ka == kWinK && xa + 1 + 4 <= n) {
            const uint32_t h1 = (P.u32(xa + 1) * kHashMul) >> hsh;
            if (lane == 0) ht[h1] = (uint16_t)(xa + 1);
        }
        i = ni;
        done = nd;
    }
    // trailing literal (writer.go:324-329)
    if (!err && done < n) {
        Hdr lh, none;
        hdr_tag(lh, kLiteral, n - done);
        emit(out, op, cap, err, P, lh, done, n - done, none, lane);
    }
    if (lane == 0) {
        A.out_size[s] = (uint64_t)op;
        if (A.status) A.status[s] = err;
    }
}

}  // namespace

// LDS words per stream for the fresh kernel (0 = the fresh kernel cannot take this launch)
uint32_t fresh_stride_words(const CompressArgs &a, int /*G*/) {
    // ring bytes are read up to 2n past the window start: 2n <= block keeps them in the fresh image
    if (a.ring || a.max_len == 0 || 2 * (int64_t)a.max_len > a.bs || a.max_len > 16384 || a.hs > 4096) return 0;
    const uint64_t ht_words = ((uint64_t)a.hs * 2 + 15) / 16 * 4;
    const uint64_t pwords = 2 + (a.max_len + 3) / 4 + 1 + 5;
    uint64_t w = ht_words + 256 + 32 + pwords;
    w = (w + 3) & ~3ull;
    return (uint32_t)w;
}

hipError_t launch_compress_fresh(const CompressArgs &a, hipStream_t st, int G) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_fresh, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const uint32_t stride = fresh_stride_words(a, G);
    const uint32_t ht_words = (uint32_t)(((uint64_t)a.hs * 2 + 15) / 16 * 4);
    const unsigned grid = (unsigned)((a.count + 3) / 4);
    const size_t lds = (size_t)stride * 4 * 4;
    hipLaunchKernelGGL(k1_fresh, dim3(grid), dim3(256), lds, st, a, stride, ht_words);
    return hipGetLastError();
}

}  // namespace ez
