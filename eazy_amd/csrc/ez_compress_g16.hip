// ez_compress_g16.hip — K1g: batch compression of fresh streams, 4 streams per wave.
//
// The algorithm of k1_fresh (ez_compress_fresh.hip: the speculative window
// restatement of Writer.Write, writer.go:206-337, for fresh streams with
// 2n <= block) with 16 lanes per stream, so one wave advances 4 streams
// per window step and every instruction serves 4 streams.  Control is per
// 16-lane group (VGPR-resident stream state, group ballots, ds_bpermute
// broadcasts); token headers are built branch-free.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"

namespace ez {
namespace {

constexpr int G = 16;
constexpr int NG = 4;  // streams per wave
constexpr int kNB = 128;

enum : int { kRej = 0, kWinK = 1, kRunK = 2, kCutK = 3, kZeroK = 4 };

__device__ __forceinline__ uint32_t gball(bool p, int g) { return (uint32_t)(((uint64_t)__ballot(p) >> (16 * g)) & 0xffff); }
__device__ __forceinline__ int32_t gbc(int32_t v, int src_lane) { return __shfl(v, src_lane, 64); }

struct PV {
    const uint32_t *w;
    uint32_t pb;
    __device__ __forceinline__ uint32_t b(int32_t y) const { return ((const uint8_t *)w)[pb + y]; }
    __device__ __forceinline__ uint32_t u32(int32_t y) const { return words_u32(w, (uint32_t)(pb + y)); }
    __device__ __forceinline__ void around(int32_t y, uint64_t &before, uint64_t &from) const {
        const uint32_t a = pb + y - 8;
        const uint32_t k = a >> 2, sh = a & 3;
        const uint32_t w0 = w[k], w1 = w[k + 1], w2 = w[k + 2], w3 = w[k + 3], w4 = w[k + 4];
        before = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
        from = (uint64_t)__builtin_amdgcn_alignbyte(w3, w2, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w4, w3, sh) << 32);
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

// group-cooperative match count, 64 bytes per step (4 per lane)
template <bool FWD, class FA, class FB>
__device__ __forceinline__ int32_t gcount(bool active, int g, int lj, int32_t lim, FA va, FB vb) {
    int32_t base = 0, res = lim;
    bool run = active && lim > 0;
    if (active && lim <= 0) res = 0;
    while (__ballot(run) != 0) {
        int32_t mb = 4;
        if (run) {
            const int32_t k = base + 4 * lj;
            if (k < lim) {
                const uint32_t d = va(k) ^ vb(k);
                if (d) mb = FWD ? (int32_t)(__builtin_ctz(d) >> 3) : (int32_t)(__builtin_clz(d) >> 3);
                if (mb > lim - k) mb = lim - k;
            } else {
                mb = 0;
            }
        }
        const uint32_t bad = gball(run && mb < 4, g);
        const int l = bad ? __builtin_ctz(bad) : 0;
        const int32_t mbl = gbc(mb, 16 * g + l);
        if (run) {
            if (bad) {
                res = base + 4 * l + mbl;
                if (res > lim) res = lim;
                run = false;
            } else {
                base += 4 * G;
                if (base >= lim) run = false;
            }
        }
    }
    return res;
}

__global__ __launch_bounds__(64) void k1_g16(CompressArgs A, uint32_t stride_words, uint32_t ht_words) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int wave = 0;  // one wave per block: finer LDS granularity per CU
    const int g = lane >> 4, lj = lane & 15;
    const int32_t hs = (int32_t)A.hs;
    const int64_t bs = A.bs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));

    // per-stream LDS: [ht u16 x hs][bucket masks u32 x 128][lane hashes u16 x 16][p words]
    uint32_t *base = (uint32_t *)smem + (uint32_t)(wave * NG + g) * stride_words;
    uint16_t *ht = (uint16_t *)base;
    volatile uint32_t *bm = (volatile uint32_t *)(base + ht_words);
    volatile uint16_t *H = (volatile uint16_t *)(base + ht_words + kNB);
    uint32_t *pw = base + ht_words + kNB + 8;

    const uint64_t s = ((uint64_t)blockIdx.x + wave) * NG + g;
    const bool have = s < A.count;
    int32_t n = 0;
    const uint8_t *gp = A.in;
    if (have) {
        n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        gp = A.in + A.in_off[s];
    }
    const uint32_t r = (uint32_t)((uintptr_t)gp & 3);
    const uint32_t *gw = (const uint32_t *)(gp - r);
    const int32_t nw = have ? (int32_t)((r + (uint32_t)n + 3) >> 2) : 0;
    PV P;
    P.w = pw;
    P.pb = 8 + r;
    if (lj < 2) pw[lj] = 0;
    for (int32_t k = lj; k < nw; k += G) {
        uint32_t v = gw[k];
        if (k == 0) v &= ~0u << (8 * r);
        v = low_bytes32(v, n - (4 * k - (int32_t)r));
        pw[2 + k] = v;
    }
    if (lj < 5) pw[2 + nw + lj] = 0;
    for (int32_t k = lj; k < (int32_t)ht_words; k += G) ((uint32_t *)ht)[k] = 0;
    for (int32_t k = lj; k < kNB; k += G) bm[k] = 0;

    uint8_t *out = have ? A.out + A.out_off[s] : A.out;
    const int32_t cap = have ? (int32_t)(A.out_off[s + 1] - A.out_off[s]) : 0;
    int err = 0;
    // header (writer.go:495-517): magic + reset, or reset alone
    int32_t op = A.append_magic ? 9 : 3;
    if (have) {
        if (op > cap) err = EZ_ENOSPC;
        else if (lj < op) {
            const uint64_t hm = 0x141080797a616502ull;  // 02 e a z y 80 10 14 (after the leading 80), little-endian
            uint32_t v;
            const int32_t bsl = (int32_t)__builtin_ctzll((uint64_t)bs);
            if (A.append_magic) v = lj == 0 ? 0x80 : (lj == 8 ? (uint32_t)bsl : (uint32_t)((hm >> (8 * (lj - 1))) & 0xff));
            else v = lj == 0 ? 0x80 : (lj == 1 ? 0x10 : (uint32_t)bsl);
            out[lj] = (uint8_t)v;
        }
    }

    int32_t i = 0, done = 0;
    bool live = have && n >= 4 && !err;
    int32_t guard = 16 * n + 4096;

    while (__ballot(live) != 0) {
        if (live && --guard < 0) { err = EZ_ESTUCK; live = false; }
        int32_t nvalid = n - 3 - i;
        if (nvalid > G) nvalid = G;
        const int32_t x = i + lj;
        const bool valid = live && lj < nvalid;

        uint64_t pxb = 0, pxf = 0;
        uint32_t h = 0, bk = 0;
        int prev = -1, next = G;
        if (valid) {
            P.around(x, pxb, pxf);
            h = ((uint32_t)pxf * kHashMul) >> hsh;
            bk = h & (kNB - 1);
            atomicOr((unsigned int *)&bm[bk], 1u << lj);
            H[lj] = (uint16_t)h;
        }
        if (valid) {
            const uint32_t m = bm[bk];
            uint32_t below = m & ((1u << lj) - 1);
            while (below) {
                const int k = 31 - __builtin_clz(below);
                if (H[k] == (uint16_t)h) { prev = k; break; }
                below &= ~(1u << k);
            }
            uint32_t above = m & (~0u << (lj + 1));
            while (above) {
                const int k = __builtin_ctz(above);
                if (H[k] == (uint16_t)h) { next = k; break; }
                above &= above - 1;
            }
        }
        int32_t cand = 0;
        if (valid) cand = prev >= 0 ? i + prev : (int32_t)ht[h];

        // ---- per-lane capped evaluation
        int kind = kRej;
        bool exact = true;
        int32_t va = 0, vb = 0;
        if (valid) {
            uint64_t pcb, pcf;
            P.around(cand, pcb, pcf);
            const bool run = cand >= done && cand < x;
            const int32_t flim = n - x;
            const int32_t fr = ctz_bytes(pxf ^ (run ? pcf : low_bytes(pcf, done - cand)));
            const int32_t f = fr < flim ? fr : flim;
            const int32_t blim = run ? ((x - done) < cand ? (x - done) : cand) : (x - done);
            const int32_t cr = clz_bytes(pxb ^ (run ? pcb : low_bytes(pcb, done - cand + 8)));
            const int32_t c = cr < blim ? cr : blim;
            const bool capped = (fr >= 8 && flim > 8) || (cr >= 8 && blim > 8);
            int32_t ist = x - c, iend = x + f;
            int64_t st = (int64_t)cand - c, end = (int64_t)cand + f;
            int64_t dd = ((int64_t)done - bs + (iend - done)) - st;
            if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
            dd = end - done;
            if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
            const bool wacc = end - st >= kMinCopyChunk;
            const bool zero = cand + 8 < n && pcf == 0;
            const bool racc = capped || f + c >= kMinCopyChunk;
            const bool cut = (int64_t)(x - cand) >= bs - 8;
            kind = run ? (zero ? kZeroK : (!racc ? kRej : (cut ? kCutK : kRunK)))
                       : ((wacc || capped) ? kWinK : kRej);
            exact = !capped;
            va = run ? c : ist;
            vb = run ? f : iend;
            if (!run && !wacc) exact = false;  // capped maybe
        }

        // ---- first accepting lane per group
        uint32_t cm = gball(valid && kind != kRej, g);
        const uint32_t exm = gball(exact, g);
        int a = -1, ka = kRej;
        int32_t xa = 0, ca = 0, r1 = 0, r2 = 0;
        bool pending = live && cm != 0;
        while (__ballot(pending) != 0) {
            const int l = pending ? __builtin_ctz(cm) : 0;
            const int src = 16 * g + l;
            const int kl = gbc(kind, src);
            const int32_t cl = gbc(cand, src);
            const int32_t t1 = gbc(va, src), t2 = gbc(vb, src);
            const bool ex = (exm >> l) & 1;
            const int32_t xl = i + l;
            const bool need_win = pending && kl == kWinK && !ex;
            const bool need_run = pending && kl == kRunK && !ex;
            const bool need_zero = pending && kl == kZeroK;
            int32_t e1 = t1, e2 = t2;
            if (__ballot(need_win) != 0) {
                const int32_t bw = gcount<false>(need_win, g, lj, xl - done,
                    [&](int32_t k) { return P.u32(xl - k - 4); },
                    [&](int32_t k) {
                        const int32_t y0 = cl - k - 4;
                        if (y0 + 4 <= 0 || y0 >= done) return 0u;
                        const uint32_t v = y0 >= 0 ? P.u32(y0) : (P.u32(0) << (8 * (-y0)));
                        return low_bytes32(v, done - y0);
                    });
                const int32_t fw = gcount<true>(need_win, g, lj, n - xl,
                    [&](int32_t k) { return P.u32(xl + k); },
                    [&](int32_t k) {
                        const int32_t y0 = cl + k;
                        if (y0 >= done) return 0u;
                        return low_bytes32(P.u32(y0), done - y0);
                    });
                if (need_win) {
                    int32_t ist = xl - bw, iend = xl + fw;
                    int64_t st = (int64_t)cl - bw, end = (int64_t)cl + fw;
                    int64_t dd = ((int64_t)done - bs + (iend - done)) - st;
                    if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
                    dd = end - done;
                    if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
                    e1 = ist;
                    e2 = iend;
                    if (end - st < kMinCopyChunk) e1 = -1;  // maybe -> reject
                }
            }
            if (__ballot(need_run) != 0) {
                const int32_t rbl = (xl - done) < cl ? (xl - done) : cl;
                const int32_t jb = gcount<false>(need_run, g, lj, rbl, [&](int32_t k) { return P.u32(xl - k - 4); },
                                                 [&](int32_t k) { return P.u32(cl - k - 4); });
                const int32_t jf = gcount<true>(need_run, g, lj, n - xl, [&](int32_t k) { return P.u32(xl + k); },
                                                [&](int32_t k) { return P.u32(cl + k); });
                if (need_run) { e1 = jb; e2 = jf; }
            }
            if (__ballot(need_zero) != 0) {
                const int32_t zb = gcount<false>(need_zero, g, lj, cl - done, [&](int32_t k) { return P.u32(cl - k - 4); },
                                                 [](int32_t) { return 0u; });
                const int32_t zf = gcount<true>(need_zero, g, lj, n - cl, [&](int32_t k) { return P.u32(cl + k); },
                                                [](int32_t) { return 0u; });
                if (need_zero) { e1 = zb; e2 = zf; }
            }
            if (pending) {
                if (need_win && e1 < 0) {
                    cm &= cm - 1;
                    pending = cm != 0;
                } else {
                    a = l; ka = kl; xa = xl; ca = cl; r1 = e1; r2 = e2;
                    pending = false;
                }
            }
        }

        // ---- inserts (writer.go:216-217), last writer wins
        const int last = a < 0 ? nvalid - 1 : a;
        if (valid && lj <= last && next > last) ht[h] = (uint16_t)x;
        if (valid) bm[bk] = 0;

        // ---- the group's action, branch-free headers
        if (live) {
            if (a < 0) {
                i += nvalid;
            } else {
                const bool win = ka == kWinK, rn = ka == kRunK, ct = ka == kCutK, zr = ka == kZeroK;
                // literal [done, lend) and copy (clen, dist) of the action
                const int32_t zi = ca - r1, ziend = ca + r2;
                int32_t lend = win ? r1 : (rn ? xa - r1 : (ct ? done + xa - ca : zi));
                int32_t nxt = win ? r2 : (rn ? xa + r2 : (ct ? lend : ziend));
                const int32_t clen = win ? r2 - r1 : (rn ? r2 + r1 : ziend - zi);
                const int32_t dist = win ? xa - ca : (rn ? xa - ca : 0);
                const bool lit = rn || ct || lend > done;  // runlen's literal is unconditional
                if (win && (int64_t)dist > bs) err = EZ_EINVAL;
                const int32_t L = lend - done;
                int32_t ln = 0;
                const uint64_t lb = tag_bytes(0x00, L, &ln);
                if (!lit) ln = 0;
                // copy header = tag (<= 5 bytes) + offset (<= 6 bytes): 128 bits (cb, ch2)
                uint64_t cb = 0, ch2 = 0;
                int32_t cn = 0;
                if (!ct) {
                    int32_t tn, on;
                    const uint64_t tb = tag_bytes(0x80, clen, &tn);
                    uint64_t ob;
                    if (zr) { ob = 0x00ffull; on = 2; }  // OffLong, 0: zero region
                    else ob = off_bytes(dist, clen, &on);
                    cb = tb | (ob << (8 * tn));
                    ch2 = ob >> (64 - 8 * tn);
                    cn = tn + on;
                }
                const int32_t T = ln + (lit ? L : 0) + cn;
                if (zr && ziend - zi < kMinCopyChunk) {
                    // unreachable: >= 8 zeros are guaranteed
                    i = zi + 1;
                } else if (!err) {
                    if (op + T > cap) {
                        err = EZ_ENOSPC;
                    } else {
                        uint8_t *d = out + op;
                        const int32_t e1 = ln, e2 = ln + (lit ? L : 0);
                        for (int32_t k = lj; k < T; k += G) {
                            uint32_t v;
                            if (k < e1) v = (uint32_t)(lb >> (8 * k));
                            else if (k < e2) v = P.b(done + k - e1);
                            else {
                                const int32_t q = k - e2;
                                v = (uint32_t)(q < 8 ? (cb >> (8 * q)) : (ch2 >> (8 * (q - 8))));
                            }
                            d[k] = (uint8_t)v;
                        }
                        op += T;
                    }
                    i = nxt;
                    done = nxt;
                }
                // the extra insert of i+1 after a window match (writer.go:315-318)
                if (win && xa + 1 + 4 <= n && lj == 0) {
                    const uint32_t h1 = (P.u32(xa + 1) * kHashMul) >> hsh;
                    ht[h1] = (uint16_t)(xa + 1);
                }
            }
            if (err || i + 4 > n) live = false;
        }
    }
    // trailing literal (writer.go:324-329)
    if (have && !err && done < n) {
        int32_t ln;
        const uint64_t lb = tag_bytes(0x00, n - done, &ln);
        const int32_t T = ln + n - done;
        if (op + T > cap) {
            err = EZ_ENOSPC;
        } else {
            uint8_t *d = out + op;
            for (int32_t k = lj; k < T; k += G) d[k] = (uint8_t)(k < ln ? (uint32_t)(lb >> (8 * k)) : P.b(done + k - ln));
            op += T;
        }
    }
    if (have && lj == 0) {
        A.out_size[s] = (uint64_t)op;
        if (A.status) A.status[s] = err;
    }
}

}  // namespace

uint32_t g16_stride_words(const CompressArgs &a) {
    if (a.ring || a.max_len == 0 || 2 * (int64_t)a.max_len > a.bs || a.max_len > 16384 || a.hs > 4096) return 0;
    const uint64_t ht_words = ((uint64_t)a.hs * 2 + 15) / 16 * 4;
    const uint64_t pwords = 2 + (a.max_len + 3) / 4 + 1 + 5;
    uint64_t w = ht_words + kNB + 8 + pwords;
    w = (w + 3) & ~3ull;
    if (w * 4 * NG > 160 * 1024) return 0;
    return (uint32_t)w;
}

hipError_t launch_compress_g16(const CompressArgs &a, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_g16, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const uint32_t stride = g16_stride_words(a);
    const uint32_t ht_words = (uint32_t)(((uint64_t)a.hs * 2 + 15) / 16 * 4);
    const uint64_t per_block = (uint64_t)NG;
    const unsigned grid = (unsigned)((a.count + per_block - 1) / per_block);
    const size_t lds = (size_t)stride * 4 * per_block;
    hipLaunchKernelGGL(k1_g16, dim3(grid), dim3(64), lds, st, a, stride, ht_words);
    return hipGetLastError();
}

}  // namespace ez
