// ez_decompress_wave.hip — K2w: batch decompression of long streams, one wave
// per stream, the parse uniform (scalar) and every token's bytes produced by
// the 64 lanes, 16 bytes each, with the stream's input and recent output in LDS.
//
// Restates Reader.Read to EOF for NewReaderBytes (reader.go:116-216 read,
// readTag :218-270, continueMetaTag :272-325, Decoder :346-514) for the common
// case through k2_parse (ez_k2_parse.h), as K2r does; anything else hands the
// stream to the exact decoder (ez_decompress.hip).
//
// Why.  With streams of 64 KiB and more (C2: 4,096 x 256 KiB) there are too few
// streams to give every lane one (K2r), and the exact wave decoder pays a global
// round trip for every header byte it parses and every byte it copies.  Here a
// token costs one LDS read of its header (the input is staged 512 bytes at a
// time, one chunk ahead of the parse, in a 1 KiB input ring), a scalar parse,
// and one LDS read + write per 16 output bytes per lane: copies read the last
// 8 KiB of output from an LDS ring, farther ones the output already in HBM.
// Output leaves the ring 1 KiB at a time (64 lanes x 16 bytes, whole lines).
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"
#include "ez_k2_parse.h"
#include "ez_k2_ring.h"

namespace ez {
namespace {

constexpr int32_t kWR = 8192;      // output ring bytes per stream (power of two)
constexpr int32_t kWIn = 1024;     // input ring bytes per stream (power of two)
constexpr int32_t kWStage = 512;   // input staged this many bytes at a time (32 lanes x 16)
constexpr int32_t kWChunk = 1024;  // output leaves the ring this many bytes at a time
constexpr size_t kWLds = 16 + (size_t)kWR + 32 + kWIn + 16 + 12 * kDefSlots;  // rings, deferred literals
// Long literals (C4: a whole fp32 bucket is one literal) are not moved through the ring by the
// stream's one wave (1 KiB per pass, one HBM round trip each): their tag is parsed, the ring gets
// their last 8 KiB, and kd_copy moves their bytes with the whole chip afterwards.  A far copy
// reading from such a literal before kd_copy has run reads its bytes from the input instead.

__device__ __forceinline__ V16 ld_in(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    return y + 16 <= hi ? ld16v(y) : ld_clamped(y, lo, hi);
}

// stream s by the whole wave; false = hand it over
__device__ bool wave_one(const DecompressArgs &A, const uint64_t s, uint8_t *ring, uint8_t *inb, int32_t *defs, const int lane) {
    const uint8_t *b = A.in + A.in_off[s];
    const int64_t nb64 = (int64_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint8_t *in_end = A.in + A.in_off[A.count];
    uint8_t *out = A.out + A.out_off[s];
    const int64_t cap64 = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;
    if (in_end - A.in < 16 || nb64 >= (1ll << 30) || cap64 >= (1ll << 30) || cap64 < 16) return false;
    const int32_t nb = (int32_t)nb64, cap = (int32_t)cap64;
    // zero ring = the fresh window's zero history
    for (int32_t k = 16 * lane - 16; k < kWR + 32; k += 1024) {
        *(u64_ua *)(ring + k) = 0;
        *(u64_ua *)(ring + k + 8) = 0;
    }
    // input ring: bytes [in_hi - kWIn, in_hi) staged; pend = the next chunk, in flight
    auto put_in = [&](int32_t x, V16 v) {
        if (lane < kWStage / 16) {
            const int32_t r = (x + 16 * lane) & (kWIn - 1);
            *(u64_ua *)(inb + r) = v.lo;
            *(u64_ua *)(inb + r + 8) = v.hi;
            if (r == 0) {
                *(u64_ua *)(inb + kWIn) = v.lo;
                *(u64_ua *)(inb + kWIn + 8) = v.hi;
            }
        }
    };
    auto get_in = [&](int32_t x) { return lane < kWStage / 16 ? ld_in(b + x + 16 * lane, A.in, in_end) : V16{0, 0}; };
    int32_t in_hi = 0;
    for (; in_hi < kWIn; in_hi += kWStage) put_in(in_hi, get_in(in_hi));
    V16 pend = get_in(in_hi);

    int32_t i = 0, pos = 0, bsl = -1, fl = 0;  // fl: output below it is in HBM (or deferred)
    int nd = 0;                                 // deferred literals of this stream (defs: theirs, in LDS)
    // A group: tokens whose sources lie before the group's first output byte gpos
    // (literals staged in the input ring, copies with D >= L from the output ring),
    // cut into pieces of <= 16 bytes, one per lane: one LDS read and one exact write
    // for all of them.  Lane l's piece: gn bytes to output position gd from gs (input
    // ring if gi, else output ring).
    int32_t used = 0, gpos = 0, gd = 0, gs = 0;
    uint32_t gn = 0;
    bool gi = false;
    auto run_group = [&]() {
        if (used > 0) {
            if (lane < used) {
                const uint8_t *a = gi ? inb + (gs & (kWIn - 1)) : ring + (gs & (kWR - 1));
                rput<kWR>(ring, gd, V16{*(const u64_ua *)a, *(const u64_ua *)(a + 8)}, gn);
            }
            while (pos >= fl + kWChunk) {
                st16v(out + fl + 16 * lane, rld<kWR>(ring, fl + 16 * lane));
                fl += kWChunk;
            }
            used = 0;
        }
        gpos = pos;
    };
    while (i < nb) {
        if (i + 96 > in_hi) {  // the scan below reads input bytes i .. i+79
            if (i + 96 > in_hi + kWStage) {  // past a long literal: stage afresh
                in_hi = i & ~(kWStage - 1);
                for (int32_t e = in_hi + kWIn; in_hi < e; in_hi += kWStage) put_in(in_hi, get_in(in_hi));
            } else {
                put_in(in_hi, pend);
                in_hi += kWStage;
            }
            pend = get_in(in_hi);
        }
        // every lane scans the step that would start at input byte i + lane; the steps
        // then run in order from i, each reading its scan from its start's lane
        K2Tok c;
        c.adv = 1;
        const int rs = k2_scan(rld<kWIn>(inb, i + lane), i + lane, nb, lim32, limit, c);
        // Fast path: the steps from i (walked on the scalar unit: M = their starts) are
        // tokens, paddings and header metas, and no copy reads output of this batch.  Then
        // every token is produced by its start's lane at once, 16 bytes per round.
        {
            const int32_t advl = rs == kParseHandOver ? 64 : c.adv;
            uint64_t M = 0;
            int32_t pe = 0;
            while (pe < 64 && i + pe < nb) {
                M |= 1ull << pe;
                pe += __builtin_amdgcn_readlane(advl, pe);
            }
            const bool st = (M >> lane) & 1;
            const bool tok = st && rs == kParseToken;
            const int32_t Ll = tok ? c.L : 0;
            int32_t incl = Ll;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int32_t v = __shfl_up(incl, d, 64);
                if (lane >= d) incl += v;
            }
            const int32_t total = __builtin_amdgcn_readlane(incl, 63);
            const int32_t dst = pos + incl - Ll;
            const int32_t cs = dst - (int32_t)c.D;  // a copy's source
            bool ok = !(st && (rs == kParseHandOver || rs == kScanReset));
            if (tok) {
                ok = ok && c.L <= 256 && bsl >= 0;
                // the source: before this batch's output, and in ring slots none of its writes reach
                if (c.cp) ok = ok && (c.D == 0 || (cs + c.L <= pos && cs >= pos + total + 16 - kWR)) && (bsl >= 30 || c.D <= (1u << bsl));
                else ok = ok && i + lane + c.j + c.L <= in_hi;
            }
            // the steps before the first one that cannot go (a copy reading this batch's
            // output, say) run now; the next batch starts at that one
            const uint64_t bad = __ballot(st && !ok);
            const int32_t pf = bad ? (int32_t)__builtin_ctzll(bad) : pe;
            // (a short prefix costs a whole scan per few steps: then step by step instead)
            const int nrun = pf >= 64 ? 64 : __builtin_popcountll(M & ((1ull << pf) - 1));
            if ((pf == pe || nrun >= 4) && (uint32_t)pos + (uint32_t)total <= (uint32_t)cap) {
                const bool run = tok && lane < pf;
                for (int32_t k = 0; __ballot(run && 16 * k < c.L) != 0; k++) {
                    if (run && 16 * k < c.L) {
                        V16 v{0, 0};  // a zero region's
                        if (!c.cp) v = rld<kWIn>(inb, i + lane + c.j + 16 * k);
                        else if (c.D != 0) v = rld<kWR>(ring, cs + 16 * k);
                        rput<kWR>(ring, dst + 16 * k, v, (uint32_t)(c.L - 16 * k < 16 ? c.L - 16 * k : 16));
                    }
                }
                // output of the steps before pf: the exclusive prefix at lane pf
                pos = pf < 64 ? __builtin_amdgcn_readlane(dst, pf) : pos + total;
                i += pf;
                while (pos >= fl + kWChunk) {
                    st16v(out + fl + 16 * lane, rld<kWR>(ring, fl + 16 * lane));
                    fl += kWChunk;
                }
                gpos = pos;
                continue;
            }
        }
        // otherwise step by step
        uint32_t w0, w1, w2;
        {
            const uint32_t adv_small = rs == kParseToken && !c.cp ? 0u : (uint32_t)c.adv;  // <= 34 unless a literal
            w0 = (uint32_t)c.L;
            w1 = c.D;
            w2 = (uint32_t)(rs + 1) | ((uint32_t)c.cp << 2) | ((uint32_t)c.j << 3) | (adv_small << 6) | (c.marg << 16);
        }
        int32_t p = 0;
        while (p < 64 && i + p < nb) {
            const uint32_t x2 = (uint32_t)__builtin_amdgcn_readlane((int)w2, p);
            K2Tok t;
            t.cp = (x2 >> 2) & 1;
            t.j = (int32_t)((x2 >> 3) & 7);
            t.marg = (x2 >> 16) & 63;
            t.L = __builtin_amdgcn_readlane((int)w0, p);
            t.D = (uint32_t)__builtin_amdgcn_readlane((int)w1, p);
            int r = (int)(x2 & 3) - 1;
            t.adv = r == kParseToken && !t.cp ? t.j + t.L : (int32_t)((x2 >> 6) & 1023);
            r = k2_check(r, t, pos, cap, bsl);
            if (r == kParseHandOver) return false;
            const int32_t L = t.L, np = (L + 15) >> 4;
            const int32_t src = i + p + t.j;  // literal
            // a piece of a group: a literal whose bytes are staged, a copy with D >= L whose
            // source is still in the ring
            const bool piece = r == kParseToken && np <= 64 &&
                               (t.cp ? (t.D >= (uint32_t)L && pos - (int32_t)t.D >= pos + 16 - kWR) : src + L <= in_hi);
            if (piece) {
                if (used + np > 64 || (t.cp && pos - (int32_t)t.D + L > gpos)) run_group();
                const uint32_t k = (uint32_t)(lane - used);
                if (k < (uint32_t)np) {
                    gd = pos + 16 * (int32_t)k;
                    gs = (t.cp ? pos - (int32_t)t.D : src) + 16 * (int32_t)k;
                    gi = !t.cp;
                    gn = (uint32_t)(L - 16 * (int32_t)k < 16 ? L - 16 * (int32_t)k : 16);
                }
                used += np;
                pos += L;
            } else if (r == kParseToken && !t.cp && L >= kDeferMin && nd < kDefSlots && A.defer) {
                // a long literal: the bytes before it leave the ring exactly, the ring gets its last
                // kWR bytes, kd_copy moves it (the record's slot from the batch-wide counter)
                run_group();
                for (int32_t q = fl + 16 * lane; q < pos; q += 1024) {
                    const V16 v = rld<kWR>(ring, q);
                    if (q + 16 <= pos) st16v(out + q, v);
                    else put_small(out + q, v, (uint32_t)(pos - q));
                }
                const int32_t tail = L - kWR;  // >= 0: kDeferMin > kWR
#pragma unroll
                for (int32_t k = 0; k < kWR / 1024; k++) {
                    const int32_t q = tail + 1024 * k + 16 * lane;
                    rst<kWR>(ring, pos + q, ld_in(b + src + q, A.in, in_end));
                }
                if (lane == 0) {
                    const uint32_t at = atomicAdd(&A.defer[0], 1u);
                    if (at < A.defer_cap) ((DeferLit *)(A.defer + 4))[at] = DeferLit{A.in_off[s] + (uint64_t)src, A.out_off[s] + (uint64_t)pos, (uint64_t)L};
                }
                if (lane == 0) {
                    defs[3 * nd] = pos;
                    defs[3 * nd + 1] = src;
                    defs[3 * nd + 2] = L;
                }
                nd++;
                pos += L;
                fl = pos;
                gpos = pos;
            } else if (r == kParseToken) {
                run_group();
                const int32_t D = (int32_t)t.D;
                // lane's bytes of the token: [q, q + 16) for q = done + lane * step
                int32_t step = 16, W = 16 * 64;
                V16 pv{0, 0};
                if (t.cp && D < 16) {
                    if (D > 0) {  // a short-period run: its 16-byte pattern every `step` bytes
                        const uint32_t per = (uint32_t)D;
                        pv = run_pattern(shr16(rld<kWR>(ring, pos - 16), 16 - per), per);
                        step = (int32_t)(per * (16 / per));
                    }
                    W = 64 * step;
                } else if (t.cp) {
                    W = D & ~15;  // reads stay below the bytes this pass writes
                    W = W < 1024 ? W : 1024;
                }
                const bool staged = !t.cp && src + L <= in_hi;         // its bytes in the input ring
                for (int32_t done = 0; done < L; done += W) {
                    const int32_t q = done + step * lane;
                    const bool act = step * lane < W && q < L;
                    // ring slots of positions >= rlo are intact; below it the output is in HBM
                    const int32_t sq = pos + q - D, rlo = pos + done + 16 - kWR;
                    if (act) {
                        V16 v = pv;
                        if (!t.cp) v = staged ? rld<kWIn>(inb, src + q) : ld_in(b + src + q, A.in, in_end);
                        else if (D >= 16) v = sq >= rlo ? rld<kWR>(ring, sq) : far16(out, cap, b, sq, nd, defs);
                        rst<kWR>(ring, pos + q, v);
                    }
                    const int32_t fin = pos + (done + W < L ? done + W : L);  // final bytes end here
                    while (fin >= fl + kWChunk) {
                        st16v(out + fl + 16 * lane, rld<kWR>(ring, fl + 16 * lane));
                        fl += kWChunk;
                    }
                }
                pos += L;
                gpos = pos;
            }
            p += t.adv;
        }
        run_group();  // before the input ring moves on
        i += p;
    }
    for (int32_t q = fl + 16 * lane; q < pos; q += 1024) {  // the last partial chunk, exact bytes
        const V16 v = rld<kWR>(ring, q);
        if (q + 16 <= pos) st16v(out + q, v);
        else put_small(out + q, v, (uint32_t)(pos - q));
    }
    if (lane == 0) {
        A.out_size[s] = (uint64_t)pos;
        if (A.status) A.status[s] = EZ_OK;
    }
    return true;
}

__global__ __launch_bounds__(64) void k2_wave(DecompressArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *ring = smem + 16, *inb = smem + 16 + kWR + 32;
    int32_t *defs = (int32_t *)(smem + 16 + kWR + 32 + kWIn + 16);
    const int lane = (int)threadIdx.x;
    for (uint64_t s = blockIdx.x; s < A.count; s += gridDim.x)
        if (!wave_one(A, s, ring, inb, defs, lane) && lane == 0) {
            const uint32_t at = atomicAdd(&A.slow[0], 1u);
            A.slow[1 + at] = (uint32_t)s;
        }
}

// every deferred literal's bytes, 64 KiB pieces per block step
__global__ __launch_bounds__(256) void kd_copy(DecompressArgs A, uint64_t kp) {
    const uint64_t nl = A.defer[0] < A.defer_cap ? A.defer[0] : A.defer_cap;
    const DeferLit *rec = (const DeferLit *)(A.defer + 4);
    const uint8_t *lo = A.in, *hi = A.in + A.in_off[A.count];
    for (uint64_t q = blockIdx.x; q < nl * kp; q += gridDim.x) {
        const DeferLit L = rec[q / kp];
        // kp is a hint (the caller's largest slot): a longer literal's block takes every kp-th piece
        for (uint64_t b = (q % kp) * 65536; b < L.len; b += kp * 65536) {
            const uint64_t e = b + 65536 < L.len ? b + 65536 : L.len;
            for (uint64_t k = b + 16 * threadIdx.x; k < e; k += 16 * 256) {
                const uint8_t *y = A.in + L.src + k;
                const V16 v = y + 16 <= hi ? ld16v(y) : ld_clamped(y, lo, hi);
                if (k + 16 <= e) st16v(A.out + L.dst + k, v);
                else put_small(A.out + L.dst + k, v, (uint32_t)(e - k));
            }
        }
    }
}

}  // namespace

hipError_t launch_defer_copy(const DecompressArgs &a, hipStream_t st) {
    // pieces per record: the largest output slot bounds a literal (max_out 0: unknown, take 1 GiB)
    const uint64_t mo = a.max_out ? a.max_out : (1ull << 30);
    hipLaunchKernelGGL(kd_copy, dim3(2048), dim3(256), 0, st, a, (mo + 65535) / 65536);
    return hipGetLastError();
}

hipError_t launch_decompress_wave(const DecompressArgs &a, hipStream_t st) {
    const uint64_t grid = a.count < (1u << 30) ? a.count : (1u << 30);
    hipLaunchKernelGGL(k2_wave, dim3((unsigned)grid), dim3(64), kWLds, st, a);
    return hipGetLastError();
}

}  // namespace ez
