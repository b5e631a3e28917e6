// ez_decompress_group.hip — K2g: batch decompression of small streams, G lanes
// per stream, the stream's compressed bytes and its decoded history in LDS.
//
// Restates Reader.Read to EOF for NewReaderBytes (reader.go:116-216 read,
// readTag :218-270, continueMetaTag :272-325, reset :327-344, Decoder
// :346-514) for the common case: header metas (magic, version 0, a MetaReset
// before any output), padding, breaks (skipped), literal and copy tokens.
// Anything else — an error of any kind, a mid-stream MetaReset, an unsupported
// or wide meta, a length over BlockSizeLimit, a full slot, a stream that does
// not fit the LDS region — is handed to the lane-per-stream decoder (k2_fast,
// over a list) and from there, if need be, to the exact decoder.
//
// Why.  A lane-per-stream decoder (k2_fast) reads every back-reference from
// HBM/L2 output it wrote a few tokens earlier, and its 64 lanes touch 64
// unrelated streams per instruction: one dependent global round trip per
// token.  Here a group of G lanes owns one stream:
//   * the compressed stream is staged at the top of an LDS region with
//     coalesced loads, the output grows from the region's bottom;
//   * batches of up to G tokens are parsed serially (every lane of the group
//     runs the same parse on the same LDS bytes) and lane t keeps token t:
//     its output position, length and source;
//   * the batch executes in parallel: a token whose source is already final
//     (a literal, a zero region, or a copy whose source ends before the first
//     unfinished token of the batch) copies its bytes with 8-byte LDS moves
//     (unaligned LDS access, exact-length tails), short tokens one lane each
//     in order, long tokens by the whole group; overlapping runs (the
//     reference's doubling copy, reader.go:180-201) take a period-D pattern
//     for D < 8 and steps of D rounded down to 8 otherwise; rounds repeat
//     until the batch is done (the first unfinished token is always ready);
//   * the decoded bytes leave LDS with 16-byte stores at the end.
// Sources before the stream start read zeros (the fresh ring).
// The output may not overwrite compressed bytes not yet parsed: a batch ends
// before a token whose output would reach the first unparsed byte.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"

#ifndef EZ_EXP
#define EZ_EXP 0  // diagnostic builds only: bit 2 = cycle profile (parse / execute / store)
#endif

namespace ez {
namespace {

constexpr int kG = 16;          // lanes per stream
constexpr int kS = 64 / kG;     // streams per wave (one wave per block)
constexpr int32_t kLong = 48;   // tokens longer than this are copied by the whole group

// 16 bytes from byte q of a dword-aligned LDS area (5 aligned dword reads)
__device__ __forceinline__ V16 lds16(const uint8_t *reg, int32_t q) {
    const uint32_t *w = (const uint32_t *)reg + (q >> 2);
    const uint32_t sh = (uint32_t)q & 3;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    const uint32_t a0 = __builtin_amdgcn_alignbyte(w1, w0, sh), a1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    const uint32_t a2 = __builtin_amdgcn_alignbyte(w3, w2, sh), a3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
    return V16{(uint64_t)a0 | ((uint64_t)a1 << 32), (uint64_t)a2 | ((uint64_t)a3 << 32)};
}

typedef uint64_t __attribute__((aligned(1))) u64_ua;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef uint16_t __attribute__((aligned(1))) u16_ua;

// 8 region bytes from q; bytes before the region start (q < 0: history before
// the stream start) read 0
__device__ __forceinline__ uint64_t ld8r(const uint8_t *reg, int32_t q) {
    if (q >= 0) return *(const u64_ua *)(reg + q);
    return q <= -8 ? 0ull : (*(const u64_ua *)reg) << (8 * -q);
}
// the low k bytes of v to p (k >= 8: all 8)
__device__ __forceinline__ void st8n(uint8_t *p, uint64_t v, int32_t k) {
    if (k >= 8) {
        *(u64_ua *)p = v;
        return;
    }
    int32_t o = 0;
    if (k & 4) { *(u32_ua *)p = (uint32_t)v; v >>= 32; o = 4; }
    if (k & 2) { *(u16_ua *)(p + o) = (uint16_t)v; v >>= 16; o += 2; }
    if (k & 1) p[o] = (uint8_t)v;
}
// the 8 output bytes at offset k of a token: literal (kind 1) from the staged
// input at src, copy (kind 2) from src = dst - D (D == 0: zero region;
// 0 < D < 8: the period-D pattern P of the D bytes before dst)
__device__ __forceinline__ uint64_t chunk8(const uint8_t *reg, int kind, int32_t src, int32_t D, int32_t k, V16 P) {
    if (kind == 2 && D == 0) return 0ull;
    if (kind == 2 && D < 8) return shr16(P, (uint32_t)(k % D)).lo;
    return ld8r(reg, src + k);
}
__device__ __forceinline__ V16 pattern8(const uint8_t *reg, int kind, int32_t src, int32_t D) {
    if (kind != 2 || D == 0 || D >= 8) return V16{0, 0};
    return run_pattern(V16{ld8r(reg, src), 0}, (uint32_t)D);
}

// the LDS region: [output grows up ... | compressed words | 16 zero bytes];
// returns the region byte of compressed byte 0 (< 0: does not fit)
__device__ __forceinline__ int32_t group_ib(uint32_t R, uint32_t r, int32_t nb) {
    const int32_t nw = (int32_t)((r + (uint32_t)nb + 3) >> 2);
    const int32_t wb = (int32_t)(R >> 2) - 4 - nw;
    return wb < 0 ? -1 : 4 * wb + (int32_t)r;
}

__global__ __launch_bounds__(64) void k2_group(DecompressArgs A, uint32_t R) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / kG, lj = lane % kG;
    const uint64_t s = (uint64_t)blockIdx.x * kS + g;
    const bool have = s < A.count;
    uint8_t *reg = smem + (uint32_t)g * R;
    const uint8_t *in_end = A.in + A.in_off[A.count];
    const uint8_t *b = have ? A.in + A.in_off[s] : A.in;
    const int64_t nb64 = have ? (int64_t)(A.in_off[s + 1] - A.in_off[s]) : 0;
    const int64_t cap64 = have ? (int64_t)(A.out_off[s + 1] - A.out_off[s]) : 0;
    const int64_t limit = A.block_size_limit;
    const int32_t nb = nb64 > (int64_t)R ? (int32_t)R + 1 : (int32_t)nb64;
    const int32_t cap = cap64 > (1ll << 30) ? (1 << 30) : (int32_t)cap64;
    const uint32_t r = (uint32_t)((uintptr_t)b & 3);
    const int32_t ib = group_ib(R, r, nb);
    bool slow = have && ib < 0;
    bool run = have && !slow;

    // stage the compressed words at the region's top (bytes outside the batch read 0), then 16 zero bytes
    if (run) {
        const int32_t nw = (int32_t)((r + (uint32_t)nb + 3) >> 2);
        const uint8_t *gb = b - r;
        uint32_t *lw = (uint32_t *)(reg + (ib - (int32_t)r));
        for (int32_t k = lj; k < nw + 4; k += kG) {
            uint32_t v = 0;
            if (k < nw) {
                const uint8_t *q = gb + 4 * k;
                if (q >= A.in && q + 4 <= in_end) {
                    v = *(const uint32_t *)q;
                } else {
                    for (int t = 0; t < 4; t++)
                        if (q + t >= A.in && q + t < in_end) v |= (uint32_t)q[t] << (8 * t);
                }
            }
            lw[k] = v;
        }
    }
    __syncthreads();

    int32_t i = 0, pos = 0, bsl = -1;  // bsl: log2 of the window after MetaReset (-1: none yet)
    bool fin = !run;
#if (EZ_EXP & 4)
    uint64_t pf[4] = {0, 0, 0, 0}, pt = __builtin_amdgcn_s_memtime(), nbat = 0, nrnd = 0;
#define EZ_PM(k) do { __builtin_amdgcn_s_waitcnt(0); const uint64_t t_ = __builtin_amdgcn_s_memtime(); pf[k] += t_ - pt; pt = t_; } while (0)
#else
#define EZ_PM(k) do {} while (0)
#endif
    EZ_PM(3);
    while (__ballot(!fin) != 0) {
#if (EZ_EXP & 4)
        nbat++;
#endif
        // ---- parse up to kG tokens (the same work in every lane of the group)
        int32_t myL = 0, mydst = 0, mysrc = 0, myD = 0;
        int kind = 0;  // 0 none, 1 literal, 2 copy
        int32_t t = 0;
        const int32_t ifirst = ib + i;  // nothing at or above this region byte may be overwritten by this batch
        bool more = !fin;
        for (int guard = 0; more && guard < 4 * kG; guard++) {
            if (i >= nb) { fin = true; more = false; break; }
            const V16 h = lds16(reg, ib + i);
            const uint64_t lo = h.lo;
            const uint32_t w0 = (uint32_t)lo, w1 = (uint32_t)(lo >> 32);
            const uint32_t t0 = w0 & 0xff, l7 = t0 & 0x7f;
            if (t0 == 0) {  // padding (reader.go:221-224): the zero bytes of the window at once
                i += lo ? (int32_t)(__builtin_ctzll(lo) >> 3) : (h.hi ? 8 + (int32_t)(__builtin_ctzll(h.hi) >> 3) : 16);
                continue;
            }
            if (t0 == 0x80) {  // meta (continueMetaTag reader.go:272-325): header metas and breaks only
                const uint32_t mb = (w0 >> 8) & 0xff, mt = mb & 0xf8, ml = mb & 7;
                const int32_t mln = ml == 7 ? 0 : (1 << ml);
                const uint32_t marg = (w0 >> 16) & 0xff;
                const bool m_brk = mt == kMetaBreak && mln == 0;
                const bool m_rst = mt == kMetaReset && mln == 1 && marg <= 32 && pos == 0 && (limit == 0 || (1ll << marg) <= limit);
                const bool m_ver = mt == kMetaVer && mln == 1 && marg == 0;
                const bool m_mag = mt == kMetaMagic && mln == 4 && ((w0 >> 16) | (w1 << 16)) == 0x797a6165u;
                if (ml == 6 || i + 2 + mln > nb || !(m_brk || m_rst || m_ver || m_mag)) { slow = true; fin = true; more = false; break; }
                if (m_rst) bsl = (int32_t)marg;
                i += 2 + mln;
                continue;
            }
            // Decoder.Tag reader.go:346-392, Decoder.Offset :394-420 (1-3 byte forms here)
            const uint32_t lx = (w0 >> 8) | (w1 << 24);
            const int32_t L = l7 < 124 ? (int32_t)l7 : (l7 == 124 ? 124 + (int32_t)(lx & 0xff) : 380 + (int32_t)(lx & 0xffff));
            const uint32_t j = l7 < 124 ? 1 : (l7 == 124 ? 2 : 3);
            const bool cp = (t0 & 0x80) != 0;
            const uint32_t x = (uint32_t)(lo >> (8 * j));
            const bool lng = (x & 0xff) == 0xff;
            const uint32_t y = lng ? (uint32_t)(lo >> (8 * j + 8)) : x;
            const uint32_t o = y & 0xff, ox = y >> 8;
            const int32_t D0 = o < 252 ? (int32_t)o : (o == 252 ? 252 + (int32_t)(ox & 0xff) : 508 + (int32_t)(ox & 0xffff));
            const int32_t D = lng ? D0 : D0 + L;
            const int32_t adv = cp ? (int32_t)(j + (lng ? 1 : 0) + (o < 252 ? 1 : (o == 252 ? 2 : 3))) : (int32_t)j + L;
            const int64_t bs = bsl < 0 ? 0 : (1ll << bsl);
            // 5-byte forms, LenAlt/OffAlt, BlockSizeLimit, missed meta, truncation, the slot, distance > window
            const bool bad = l7 >= 126 || (cp && o >= 254) || (limit != 0 && L > limit) || bs == 0 || pos + L > cap ||
                             i + adv > nb || (cp && D > bs);
            if (bad) { slow = true; fin = true; more = false; break; }
            if (pos + L > ifirst) {  // the output would reach unparsed bytes: end the batch here
                if (t == 0) { slow = true; fin = true; }
                more = false;
                break;
            }
            if (lj == t) {
                myL = L;
                mydst = pos;
                kind = cp ? 2 : 1;
                myD = D;
                mysrc = cp ? pos - D : ib + i + (int32_t)j;
            }
            pos += L;
            i += adv;
            if (++t == kG) more = false;
        }
        if (slow) kind = 0;
        EZ_PM(0);

        // ---- execute the batch: rounds of the tokens whose sources are final
        bool pend = kind != 0;
        while (__ballot(pend) != 0) {
            const uint32_t pm = (uint32_t)(((uint64_t)__ballot(pend) >> (kG * g)) & 0xffffu);
            const int first = pm ? __builtin_ctz(pm) : 0;
            const int32_t fdst = __shfl(mydst, kG * g + first, 64);
            const int32_t complete = pm ? fdst : pos;  // every byte below it is final
            const bool ready = pend && (kind == 1 || myD == 0 || (myD >= myL ? mysrc + myL <= complete : mydst <= complete));
            // short tokens: one lane each, 8 bytes per step in order (a copy's
            // source bytes from dst on are written by its earlier steps, D >= 8)
            const bool sh = ready && myL <= kLong;
            const V16 P = pattern8(reg, kind, mysrc, myD);
            for (int32_t k = 0; __ballot(sh && k < myL) != 0; k += 8) {
                if (sh && k < myL) st8n(reg + mydst + k, chunk8(reg, kind, mysrc, myD, k, P), myL - k);
            }
            // long tokens: the whole group, one token at a time in stream order,
            // 8 bytes per lane; a run with 8 <= D < 8G advances D rounded down to 8
            const bool lg = ready && myL > kLong;
            uint32_t lm = (uint32_t)(((uint64_t)__ballot(lg) >> (kG * g)) & 0xffffu);
            while (__ballot(lm != 0) != 0) {
                const int tl = lm ? __builtin_ctz(lm) : 0;
                const int src = kG * g + tl;
                const int32_t L = __shfl(myL, src, 64), dst = __shfl(mydst, src, 64), sp = __shfl(mysrc, src, 64),
                              D = __shfl(myD, src, 64);
                const int kd = __shfl(kind, src, 64);
                if (lm) {
                    const V16 PL = pattern8(reg, kd, sp, D);
                    const int32_t step = (kd == 2 && D >= 8 && D < L && (D & ~7) < 8 * kG) ? (D & ~7) : 8 * kG;
                    for (int32_t base = 0; base < L; base += step) {
                        const int32_t k = base + 8 * lj;
                        if (8 * lj < step && k < L) st8n(reg + dst + k, chunk8(reg, kd, sp, D, k, PL), L - k);
                    }
                    lm &= lm - 1;
                }
            }
            pend = pend && !ready;
#if (EZ_EXP & 4)
            nrnd++;
#endif
        }
        EZ_PM(1);
    }

    // ---- the decoded bytes to the slot, or the stream to the next decoder
    if (have && slow) {
        if (lj == 0) {
            const uint32_t at = atomicAdd(&A.slow[0], 1u);
            A.slow[1 + at] = (uint32_t)s;
        }
    } else if (have) {
        uint8_t *out = A.out + A.out_off[s];
        for (int32_t k = 16 * lj; k < pos; k += 16 * kG) {
            const uint4 v = *(const uint4 *)(reg + k);
            const V16 x{(uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z | ((uint64_t)v.w << 32)};
            if (k + 16 <= pos) st16v(out + k, x);
            else put_small(out + k, x, (uint32_t)(pos - k));
        }
        if (lj == 0) {
            A.out_size[s] = (uint64_t)pos;
            if (A.status) A.status[s] = EZ_OK;
        }
    }
    EZ_PM(2);
#if (EZ_EXP & 4)
    if (blockIdx.x < 4 && lane == 0)
        printf("k2g blk %u batches %llu rounds %llu: stage %llu parse %llu exec %llu store %llu\n", blockIdx.x, (unsigned long long)nbat,
               (unsigned long long)nrnd, (unsigned long long)pf[3], (unsigned long long)pf[0], (unsigned long long)pf[1],
               (unsigned long long)pf[2]);
#endif
}

}  // namespace

// LDS region per stream for a batch whose largest output slot is max_out (0 = not usable)
uint32_t group_decode_region(uint64_t max_out) {
    if (max_out == 0 || max_out > 32768) return 0;
    const uint64_t R = (max_out + 512 + 15) & ~15ull;
    if (R * kS > 160 * 1024) return 0;
    return (uint32_t)R;
}

hipError_t launch_decompress_group(const DecompressArgs &a, uint32_t R, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k2_group, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const uint64_t grid = (a.count + kS - 1) / kS;
    hipLaunchKernelGGL(k2_group, dim3((unsigned)grid), dim3(64), (size_t)R * kS, st, a, R);
    return hipGetLastError();
}

}  // namespace ez
