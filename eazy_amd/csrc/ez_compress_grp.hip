// ez_compress_grp.hip — K1grp: batch compression of fresh streams, G lanes per
// stream, 64/G streams per wave, table and input staged in LDS.
//
// Writer.Write (writer.go:206-337) for a fresh stream (SURVEY §8 unit of work,
// 2n <= block so the ring is the linear history with zeros from `done` on,
// no far skip, no cut, no trim 1), as speculative windows of G positions:
//   1. every lane hashes its position (writer.go:491-493), finds the latest
//      earlier position of the window with the same hash (LDS bucket masks,
//      hashes verified) or else reads the table (the window's visited
//      positions shadow the table: inserts are monotone in position);
//   2. every lane judges its candidate with 8-byte capped match lengths —
//      exact, because the acceptance threshold (minCopyChunk = 6,
//      writer.go:119) is below the cap — for the run-length branch
//      (writeRunlen :441-489, writeZeros :407-439) or the window branch
//      (:233-301, trim 2 :292-296);
//   3. the group takes its first accepting lane (group ballot), inserts the
//      visited positions (last writer per hash), extends that match exactly
//      with one cooperative compare of 4*G bytes per step, and writes the
//      literal + copy tokens cooperatively (Encoder.Tag/Offset :537-597).
// All lanes of a wave run one instruction stream: per-group differences are
// data (selects), loops run only while a group still has bytes to compare.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_k1_common.h"

namespace ez {
namespace {
using namespace k1;

constexpr int kNBg = 64;  // bucket masks per stream (hash & 63), verified against the lanes' hashes

template <int G>
__global__ __launch_bounds__(64) void k1_grp(CompressArgs A, uint32_t stride_words, uint32_t ht_words) {
    constexpr int S = 64 / G;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / G, lj = lane % G;
    const int32_t hs = (int32_t)A.hs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));

    // per-stream LDS: [ht u16 x hs][bucket masks u32 x kNBg][lane hashes u16 x G][input words]
    uint32_t *base = (uint32_t *)smem + (uint32_t)g * stride_words;
    uint16_t *ht = (uint16_t *)base;
    volatile uint32_t *bm = (volatile uint32_t *)(base + ht_words);
    volatile uint16_t *H = (volatile uint16_t *)(base + ht_words + kNBg);
    uint32_t *pw = base + ht_words + kNBg + (G + 1) / 2;

    const uint64_t s = (uint64_t)blockIdx.x * S + g;
    const bool have = s < A.count;
    int32_t n = 0;
    const uint8_t *gp = A.in;
    if (have) {
        n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        gp = A.in + A.in_off[s];
    }
    // stage the input: words of the aligned span, 2 zero words in front and 5 behind
    const uint32_t r = (uint32_t)((uintptr_t)gp & 3);
    const uint32_t *gw = (const uint32_t *)(gp - r);
    const int32_t nw = have ? (int32_t)((r + (uint32_t)n + 3) >> 2) : 0;
    PW P;
    P.w = pw;
    P.pb = 8 + r;
    if (lj < 2) pw[lj] = 0;
    for (int32_t k = lj; k < nw; k += G) {
        uint32_t v = gw[k];
        if (k == 0) v &= ~0u << (8 * r);
        v = low_bytes32(v, n - (4 * k - (int32_t)r));
        pw[2 + k] = v;
    }
    for (int32_t k = lj; k < 5; k += G) pw[2 + nw + k] = 0;
    for (int32_t k = lj; k < (int32_t)ht_words; k += G) ((uint32_t *)ht)[k] = 0;
    for (int32_t k = lj; k < kNBg; k += G) bm[k] = 0;

    uint8_t *out = have ? A.out + A.out_off[s] : A.out;
    const int32_t cap = have ? (int32_t)(A.out_off[s + 1] - A.out_off[s]) : 0;
    int err = 0;
    // header (writer.go:495-517): magic + reset, or reset alone
    int32_t op = A.append_magic ? 9 : 3;
    if (have) {
        if (op > cap) err = EZ_ENOSPC;
        else {
            const uint64_t hm = 0x141080797a616502ull;  // 02 e a z y 80 10 14 (after the leading 80)
            const int32_t bsl = (int32_t)__builtin_ctzll((uint64_t)A.bs);
            for (int32_t k = lj; k < op; k += G) {
                uint32_t v;
                if (A.append_magic) v = k == 0 ? 0x80 : (k == 8 ? (uint32_t)bsl : (uint32_t)((hm >> (8 * (k - 1))) & 0xff));
                else v = k == 0 ? 0x80 : (k == 1 ? 0x10 : (uint32_t)bsl);
                out[k] = (uint8_t)v;
            }
        }
    }

    int32_t i = 0, done = 0;
    bool live = have && n >= 4 && !err;
    int32_t guard = 2 * n + 64;
    while (__ballot(live) != 0) {
        if (live && --guard < 0) { err = EZ_ESTUCK; live = false; }
        const int32_t nvalid = n - 3 - i < G ? n - 3 - i : G;
        const int32_t x = i + lj;
        const bool valid = live && lj < nvalid;

        // ---- 1. hash, same-hash lanes of the window, candidate
        uint64_t pxb = 0, pxf = 0;
        uint32_t h = 0, bk = 0;
        int prev = -1, next = G;
        if (valid) {
            P.around(x, pxb, pxf);
            h = ((uint32_t)pxf * kHashMul) >> hsh;
            bk = h & (kNBg - 1);
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
            uint32_t above = lj + 1 < 32 ? m & (~0u << (lj + 1)) : 0u;
            while (above) {
                const int k = __builtin_ctz(above);
                if (H[k] == (uint16_t)h) { next = k; break; }
                above &= above - 1;
            }
        }
        int32_t cand = 0;
        if (valid) cand = prev >= 0 ? i + prev : (int32_t)ht[h];

        // ---- 2. capped judgement (exact decision)
        bool acc = false;
        uint64_t pcb = 0, pcf = 0;
        int32_t known = 0;  // capped counts already exact below 8: forward | backward << 8
        if (valid) {
            P.around(cand, pcb, pcf);
            const bool rl = cand >= done && cand < x;
            const bool zr = rl && cand + 8 < n && pcf == 0;
            const int32_t bl = rl ? ((x - done) < cand ? (x - done) : cand) : x - done;
            int32_t jb = clz_bytes(pxb ^ pcb);
            jb = jb < bl ? jb : bl;
            int32_t jf = ctz_bytes(pxf ^ (rl ? pcf : low_bytes(pcf, done - cand)));
            jf = jf < n - x ? jf : n - x;
            acc = rl ? (zr || jf + jb >= kMinCopyChunk) : ((jf < done - cand ? jf : done - cand) + jb >= kMinCopyChunk);
            // zeros: 8 known zero bytes from the candidate, and the zero bytes before it (>= done)
            int32_t zb = clz_bytes(pcb);
            zb = zb < cand - done ? zb : cand - done;
            known = zr ? (8 | (zb << 8)) : (jf | (jb << 8));
        }
        const uint32_t am = gball<G>(acc, g);
        const int a = am ? __builtin_ctz(am) : -1;  // the group's first accepting lane

        // ---- 3. inserts of the visited positions (writer.go:216-217), last writer per hash
        const int last = a < 0 ? nvalid - 1 : a;
        if (valid && lj <= last && next > last) ht[h] = (uint16_t)x;
        if (valid) bm[bk] = 0;

        // ---- 4. the accepted match: exact lengths, tokens
        const int src = G * g + (a < 0 ? 0 : a);
        const int32_t ca = bcast(cand, src);
        const uint32_t pcf_lo = (uint32_t)bcast((int32_t)(uint32_t)pcf, src), pcf_hi = (uint32_t)bcast((int32_t)(uint32_t)(pcf >> 32), src);
        const uint64_t cf_a = (uint64_t)pcf_lo | ((uint64_t)pcf_hi << 32);
        const bool act = live && a >= 0;
        const int32_t xa = i + a;
        const bool rl = ca >= done && ca < xa;
        const bool zr = rl && ca + 8 < n && cf_a == 0;
        const int mode = zr ? 0 : (rl ? 1 : 2);
        // forward from fa (zeros: from the candidate, 8 known zero bytes)
        const int32_t fa = zr ? ca : xa;
        const int32_t kn = bcast(known, src), fk = kn & 0xff, bk8 = kn >> 8;
        // only a saturated capped count (8) needs the cooperative extension
        const int32_t fx = gcount<G, true>(P, act && fk == 8, g, lj, fa, ca, mode, done, 8, n - fa);
        const int32_t f = fk == 8 ? fx : fk;
        // backward before fa; window: the candidate side is below done
        const int32_t blim = zr ? ca - done : (rl ? ((xa - done) < ca ? (xa - done) : ca) : xa - done);
        const int32_t cx = gcount<G, false>(P, act && bk8 == 8, g, lj, fa, ca, mode, done, 8, blim);
        const int32_t c = bk8 == 8 ? cx : bk8;
        if (act) {
            int32_t lit_end, nxt, clen;
            if (zr) {
                lit_end = ca - c;
                nxt = ca + f;
                clen = nxt - lit_end;
            } else if (rl) {
                lit_end = xa - c;
                nxt = xa + f;
                clen = f + c;
            } else {
                const int32_t over = ca + f - done;  // trim 2 (writer.go:292-296)
                lit_end = xa - c;
                nxt = xa + f - (over > 0 ? over : 0);
                clen = nxt - lit_end;
            }
            const bool lit = (rl && !zr) || lit_end > done;  // run-length: unconditional
            const int32_t L = lit_end - done;
            int32_t ln = 0;
            const uint64_t lb = tag_bytes(0x00, L, &ln);
            if (!lit) ln = 0;
            int32_t tn, on;
            const uint64_t tb = tag_bytes(0x80, clen, &tn);
            uint64_t ob;
            if (zr) { ob = 0x00ffull; on = 2; }  // OffLong, 0: zero region
            else ob = off_bytes(xa - ca, clen, &on);
            const uint64_t cb = tb | (ob << (8 * tn)), ch2 = ob >> (64 - 8 * tn);
            const int32_t cn = tn + on;
            const int32_t e1 = ln, e2 = ln + (lit ? L : 0);
            const int32_t T = e2 + cn;
            if (op + T > cap) {
                err = EZ_ENOSPC;
            } else {
                uint8_t *d = out + op;
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
            // the extra insert of i+1 after a window match (writer.go:315-318)
            if (!rl && xa + 1 + 4 <= n && lj == 0) {
                const uint32_t h1 = (P.u32(xa + 1) * kHashMul) >> hsh;
                ht[h1] = (uint16_t)(xa + 1);
            }
            i = done = nxt;
        } else if (live) {
            i += nvalid;
        }
        if (live && (err || i + 4 > n)) live = false;
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

template <int G>
uint32_t grp_stride(const CompressArgs &a) {
    if (a.ring || a.max_len == 0 || 2 * (int64_t)a.max_len > a.bs || a.max_len > 16384 || a.hs > 4096) return 0;
    const uint64_t ht_words = ((uint64_t)a.hs * 2 + 15) / 16 * 4;
    const uint64_t pwords = 2 + (a.max_len + 3) / 4 + 1 + 5;
    uint64_t w = ht_words + kNBg + (G + 1) / 2 + pwords;
    w = (w + 3) & ~3ull;
    if (w * 4 * (64 / G) > 160 * 1024) return 0;
    return (uint32_t)w;
}

template <int G>
hipError_t launch_grp(const CompressArgs &a, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_grp<G>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    constexpr int S = 64 / G;
    const uint32_t stride = grp_stride<G>(a);
    const uint32_t ht_words = (uint32_t)(((uint64_t)a.hs * 2 + 15) / 16 * 4);
    const unsigned grid = (unsigned)((a.count + S - 1) / S);
    hipLaunchKernelGGL(k1_grp<G>, dim3(grid), dim3(64), (size_t)stride * 4 * S, st, a, stride, ht_words);
    return hipGetLastError();
}

}  // namespace

static int grp_lanes() {
    static const int g = getenv("EZ_K1_G") ? atoi(getenv("EZ_K1_G")) : 16;
    return g == 8 || g == 16 || g == 32 ? g : 16;
}

uint32_t grp_stride_words(const CompressArgs &a) {
    const int G = grp_lanes();
    return G == 8 ? grp_stride<8>(a) : (G == 32 ? grp_stride<32>(a) : grp_stride<16>(a));
}

hipError_t launch_compress_grp(const CompressArgs &a, hipStream_t st) {
    const int G = grp_lanes();
    return G == 8 ? launch_grp<8>(a, st) : (G == 32 ? launch_grp<32>(a, st) : launch_grp<16>(a, st));
}

}  // namespace ez
