// ez_decompress_ring.hip — K2r: batch decompression, one lane per stream, the
// last 512 decoded bytes of every stream in an LDS ring.
//
// Restates Reader.Read to EOF for NewReaderBytes (reader.go:116-216 read,
// readTag :218-270, continueMetaTag :272-325, reset :327-344, Decoder
// :346-514) for the common case — header metas, padding, breaks, literal and
// copy tokens; anything else hands the stream to the exact decoder.
//
// Why the ring.  A lane decoder without it (k2_fast, round 1; removed) read every
// back-reference from the output it wrote to HBM a
// few tokens earlier; 64 lanes of a wave touch 64 unrelated streams, and at
// C1 the 8,192 streams in flight per XCD keep ~5 MB of recently written lines
// live against a 4 MB L2 (PMC: 43 % L2 misses).  Most distances are short
// (median 365 bytes on the C1 logs), so each lane keeps its stream's last 512
// output bytes in LDS (ring[p & 511] = output byte p, plus a 16-byte mirror of
// the ring's first bytes after its end so that any 16-byte read is one
// contiguous LDS access): copies with distance <= 496 read the ring, farther
// ones read HBM as before.  The ring starts zeroed, which is the fresh
// window's zero history: a position before the stream start
// maps to a ring slot that has not been written yet.  The output reaches HBM
// from the ring in whole 128-byte lines once they are final, instead of one
// 16-byte partial-line store per move (the stores cost half of k2_fast's time:
// 1.37 -> 0.69 ms with them removed).  One block of 256 lanes per CU (4
// waves, one per SIMD) holds 256 rings of 528 bytes.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"
#include "ez_k2_parse.h"

namespace ez {
namespace {

constexpr int32_t kRing = 512;           // ring bytes per stream (power of two)
// per lane: a 16-byte front guard, the ring, the mirror of bytes 0..15, a 16-byte back guard
constexpr int32_t kRingStride = 16 + kRing + 16 + 16;
constexpr int32_t kNear = kRing - 16;    // copies this close read the ring
constexpr int kRingBlock = 256;          // lanes per block (one wave per SIMD of a CU)
constexpr int32_t kChunk = 128;          // output leaves the ring in whole 128-byte lines
// a step moves <= 16 bytes, plus a paired short literal's <= 15 (below): the unflushed output stays
// below kChunk + 31 * (fper + 1) + 16 <= kRing for fper <= 8
constexpr uint32_t kMaxFlushPer = 8;

typedef uint64_t __attribute__((aligned(1))) u64_ua;

// the compiler's scheduler does not move instructions across this point (device code)
__host__ __device__ __forceinline__ void sched_fence() {
#ifdef __HIP_DEVICE_COMPILE__
    __builtin_amdgcn_sched_barrier(0);
#endif
}

// whether c holds on any lane of the wave (the host emulation runs one lane)
__host__ __device__ __forceinline__ bool any_lane(bool c) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_ballot_w64(c) != 0;
#else
    return c;
#endif
}

// bytes a run of period per (1..15) advances per 16-byte pattern store: the largest
// multiple of per <= 16 (per 0, the zero region: 16), from a nibble table
__host__ __device__ constexpr uint64_t run_steps() {
    uint64_t k = 0;
    for (uint32_t per = 0; per < 16; per++) k |= (uint64_t)((per ? per * (16 / per) : 16) - 1) << (4 * per);
    return k;
}
__host__ __device__ __forceinline__ int32_t run_step(uint32_t per) { return (int32_t)((run_steps() >> (4 * per)) & 15) + 1; }

// 16 bytes at y of the batch [lo, hi) (bytes from hi on read as 0)
__host__ __device__ __forceinline__ V16 ld_in(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    return y + 16 <= hi ? ld16v(y) : ld_clamped16(y, lo, hi);  // (the batch holds >= 16 bytes: checked)
}
__host__ __device__ __forceinline__ V16 ring_ld(const uint8_t *ring, int32_t p) {
    const uint8_t *q = ring + (p & (kRing - 1));
    return V16{*(const u64_ua *)q, *(const u64_ua *)(q + 8)};
}
// 16 bytes of output position p into the ring, keeping the mirror equal to bytes 0..15,
// branch-free: the same 16 bytes are written a second time at r - kRing when they wrap
// (their head lands in the front guard, their tail at the ring's start) or at r + kRing
// when they start in the first 16 bytes (their head lands in the mirror, their tail in
// the back guard), else again at r
__host__ __device__ __forceinline__ void ring_st(uint8_t *ring, int32_t p, V16 v) {
    const int32_t r = p & (kRing - 1);
    const int32_t r2 = r + 16 > kRing ? r - kRing : (r < 16 ? r + kRing : r);
    *(u64_ua *)(ring + r) = v.lo;
    *(u64_ua *)(ring + r + 8) = v.hi;
    *(u64_ua *)(ring + r2) = v.lo;
    *(u64_ua *)(ring + r2 + 8) = v.hi;
}

// bytes o .. o+15 (0 <= o <= 16) of the 32 bytes (a, b)
__host__ __device__ __forceinline__ V16 win16(V16 a, V16 b, uint32_t o) {
    const uint32_t q = o >> 3, r = o & 7;
    const uint64_t w0 = q == 0 ? a.lo : (q == 1 ? a.hi : b.lo);
    const uint64_t w1 = q == 0 ? a.hi : (q == 1 ? b.lo : b.hi);
    const uint64_t w2 = q == 0 ? b.lo : b.hi;  // (q == 2: o == 16, r == 0: w2 unused)
    return V16{fun8(w0, w1, r), fun8(w1, w2, r)};
}

#ifndef __HIP_DEVICE_COMPILE__
inline uint64_t g_ring_iters = 0, g_ring_stat[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // (host emulation statistics)
#endif

// decodes stream s with `ring` (kRing + 16 bytes, with 16-byte guards on both sides) as its history; false = hand
// the stream over (host-compilable: tools/ring_emu.hip runs it on the CPU)
// fper: iterations between flushes (a power of two <= kMaxFlushPer)
// HW (A/B only): the headers from a 32-byte window of 16-byte-aligned input loads, reloaded only when
// the next header leaves it (one aligned pair per ~3 tokens at C1), instead of one byte-unaligned
// 16-byte load per token: measured slower at C1 (0.544 against 0.462 ms): the loads are not what
// binds K2r, and the window's selects and the reload branch add to the per-token chain
template <bool HW>
__host__ __device__ __forceinline__ bool ring_one(const DecompressArgs &A, const uint64_t s, uint8_t *ring, uint32_t fper = 8) {
    const uint8_t *b = A.in + A.in_off[s];
    const int64_t nb64 = (int64_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint8_t *in_end = A.in + A.in_off[A.count];  // loads never pass the last stream's end
    uint8_t *out = A.out + A.out_off[s];
    const int64_t cap64 = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;  // 0: no limit
    // 32-bit positions; clamped loads need >= 16 input bytes in the batch and a 16-byte slot
    bool slow = in_end - A.in < 16 || nb64 >= (1ll << 30) || cap64 >= (1ll << 30) || cap64 < 16;
    const int32_t nb = slow ? 0 : (int32_t)nb64, cap = (int32_t)cap64;
    // the batch's last 16-byte load position, relative to b (capped: a batch may pass 2 GiB)
    const int64_t lh64 = (int64_t)(in_end - b) - 16;
    const int32_t lit_hi = lh64 > 0x7fffffff ? 0x7fffffff : (int32_t)lh64;
    for (int32_t k = 0; k < kRing + 16; k += 16) {
        *(u64_ua *)(ring + k) = 0;
        *(u64_ua *)(ring + k + 8) = 0;
    }
    int32_t i = 0, pos = 0, bsl = -1;  // bsl: log2 of the window after MetaReset (-1: none yet)
    int32_t win = 0;                   // the window's size once bsl is set (copies farther hand over)
    V16 h{0, 0};                       // 16 bytes at b + i (the next header)
    int32_t hd = 0;  // a header loaded from the batch's last 16 bytes: its shift, applied after the wait
    // HW: the input [wb, wb + 32) (wb 16-byte aligned) in hw0, hw1; the next header at wb + hd
    const uint8_t *wb = (const uint8_t *)((uintptr_t)b & ~(uintptr_t)15);
    V16 hw0{0, 0}, hw1{0, 0};
    if (!slow) {
        if (HW) {
            hw0 = ld_clamped16(wb, A.in, in_end);
            hw1 = ld_clamped16(wb + 16, A.in, in_end);
            hd = (int32_t)(b - wb);
        } else {
            h = ld_in(b, A.in, in_end);
        }
    }
    // the token being written: rem bytes at dst from sb + so (input / HBM output; 32-bit offsets,
    // loads clamped to [sb, sb + shi + 16)) or from the ring
    int32_t rem = 0, dst = 0, step = 16, rp = 0, fl = 0;  // fl: output below it is in HBM
    uint32_t it = 0;
    const uint8_t *sb = b;
    int32_t so = 0, shi = lit_hi;
    int32_t src = 0;  // the move's bytes: 0 from HBM (a far copy, a long literal), 1 the pattern pv, 2 the ring
    bool live = !slow;
    V16 pv{0, 0};
    // (a load after the first header, as every iteration ends with one after the next header:
    // the loop's entry then matches its back edge and the header wait counts past it; the
    // offset table holds >= 16 bytes)
    V16 graw = ld16v((const uint8_t *)A.in_off);
    int32_t gd = 0;
    // The lanes of a wave iterate together; every step is written for all of them with selects,
    // and the rare work (the full parse, runs, HBM moves, clamped loads) sits behind wave-uniform
    // tests.  An iteration issues the loads of the current token's move, parses the next token
    // (for the lanes whose current token ends with this move) and loads the header after it
    // while those loads are in flight, then stores the move and takes the next token's state: the
    // parse no longer waits behind the move's HBM read, nor the move behind the parse.
    // (every lane loads in every iteration; lanes are live only if the batch holds >= 16 bytes)
    for (bool go = any_lane(live); go; go = any_lane(live)) {
        if (HW) {
            h = win16(hw0, hw1, (uint32_t)hd);
        } else if (any_lane(hd != 0)) {
            if (hd != 0) h = shr16(h, (uint32_t)hd);  // bytes past the batch read 0
        }
        // ---- move, part 1: this iteration's bytes of the current token (rem == 0: nothing);
        // a far copy's or long literal's 16 bytes (graw) were loaded one iteration ago
        V16 v = ring_ld(ring, rp);
        const bool hb = rem > 0 && src == 0;  // a far copy or a long literal: from HBM
        const int32_t kk = rem < step ? rem : step;
        // ---- parse: the lanes whose current token ends with this move take the next one
        bool np = live && rem == kk;
        const bool fin = np && i >= nb;  // the input is done: this move is the lane's last
        np = np && !fin;
        // the common forms branch-free; anything else (padding, metas, long tags and
        // offsets, a check that fails) takes the full parse, which may hand over
        int32_t L, adv, j = 1;
        uint32_t D;
        bool cp;
        const int32_t ft = fast_tok(h.lo, L, adv, D, cp);
        const bool f = (ft | bsl | (nb - i - adv) | (cap - pos - L) | (lim32 - L) | (cp ? win - (int32_t)D : 0)) >= 0;
        V16 hv{(h.lo >> 8) | (h.hi << 56), h.hi >> 8};  // the header after a 1-byte tag
        bool ho = false;                                // hand the stream over
        if (any_lane(np && !f)) {
            if (np && !f) {
                K2Tok t;
                const int r = k2_parse(h, i, nb, pos, cap, lim32, limit, bsl, t);
                if (r == kParseHandOver) {
                    ho = true;
                } else {
                    L = t.L;
                    adv = t.adv;
                    j = t.j;
                    D = t.D;
                    cp = t.cp;
                    win = bsl < 0 ? 0 : (bsl >= 30 ? 0x7fffffff : 1 << bsl);  // (D < 2^17 on the fast path)
                    hv = shr16(h, (uint32_t)j);
                }
            }
        }
        np = np && !ho;
        const int32_t i0 = i;
        i = np ? i + adv : i;
        // ---- a short literal and the copy after it in one step (!HW): the literal's
        // bytes are in the header already (src 1), so when the copy's header lies in the same 16
        // bytes the literal is stored right after this step's move and the copy becomes the lane's
        // next token -- one iteration per literal-copy pair instead of two (C1's logs: 462 -> ~343
        // iterations per stream)
        bool pair = false;
        int32_t L1 = 0;
#if (EZ_EXP & (1 << 27))  // (timing builds: one token per step, A/B)
        if (false) {
#else
        if (!HW) {
#endif
            const uint32_t o2 = 1u + (uint32_t)L;  // (the fast path's 1-byte tag; o2 <= 11 below)
            const uint64_t h2 = o2 < 8 ? (h.lo >> (8 * o2)) | (h.hi << (64 - 8 * o2)) : h.hi >> (8 * (o2 & 7));
            int32_t L2, adv2;
            uint32_t D2;
            bool cp2;
            const int32_t ft2 = fast_tok(h2, L2, adv2, D2, cp2);
            pair = np && f && !cp && cp2 && o2 <= 11 &&
                   (ft2 | (16 - (int32_t)o2 - adv2) | (nb - i - adv2) | (cap - pos - L - L2) | (lim32 - L2) | (win - (int32_t)D2)) >= 0;
            if (pair) {
                L1 = L;
                L = L2;
                D = D2;
                cp = true;
                i += adv2;
            }
        }
        // the next header (lanes not parsing reload theirs), one load for every lane: near the
        // batch's end from its last 16 bytes, shifted after the wait at the next iteration's top
        if (HW) {
            const uint8_t *y = b + i;
            const bool rl = y > wb + 16;  // (the header leaves the window; i never moves back)
            if (any_lane(rl)) {
                if (rl) {
                    wb = (const uint8_t *)((uintptr_t)y & ~(uintptr_t)15);
                    if (wb >= A.in && wb + 32 <= in_end) {
                        hw0 = ld16v(wb);
                        hw1 = ld16v(wb + 16);
                    } else {  // the batch's end: bytes past it read 0
                        hw0 = ld_clamped16(wb, A.in, in_end);
                        hw1 = ld_clamped16(wb + 16, A.in, in_end);
                    }
                }
            }
            hd = (int32_t)(y - wb);
        } else {
            const int32_t ic = i < lit_hi ? i : lit_hi;  // (the batch's last 16 bytes)
            h = ld16v(b + ic);
            hd = i - ic;
        }
        // ---- move, part 2
        V16 g = graw;
        if (any_lane(hb && gd != 0)) {  // bytes outside the batch or before the slot read 0
            if (hb && gd != 0) g = gd > 0 ? shr16(graw, (uint32_t)gd) : shl16(graw, (uint32_t)-gd);
        }
        v.lo = hb ? g.lo : v.lo;  // (field by field: a select of the struct went through scratch)
        v.hi = hb ? g.hi : v.hi;
        v.lo = src == 1 ? pv.lo : v.lo;
        v.hi = src == 1 ? pv.hi : v.hi;
        ring_st(ring, dst, v);
        dst += kk;
        so += kk;
        rp += kk;
        rem -= kk;
        if (pair) ring_st(ring, dst, hv);  // the paired literal at the output position (dst == pos)
#ifndef __HIP_DEVICE_COMPILE__
        if (live) {
            g_ring_stat[0]++;
            if (!np) g_ring_stat[src == 0 ? 1 : (src == 1 ? 2 : 3)]++;  // a long token's inner move: HBM / pattern / ring
            if (np && pair) g_ring_stat[4]++;
            if (np && !pair && !cp) g_ring_stat[5]++;  // a literal parsed alone
            if (np && !pair && cp) g_ring_stat[6]++;   // a copy parsed alone
        }
#endif
        dst = pair ? dst + L1 : dst;
        pos = pair ? pos + L1 : pos;
        // ---- the next token's state (a padding or meta step has L = 0: no move)
        const bool run = cp && D < 16;
        rem = np ? L : rem;
        rp = np ? pos - (int32_t)D : rp;
        so = np ? (cp ? pos - (int32_t)D : i0 + j) : so;
        sb = np ? (cp ? (const uint8_t *)out : b) : sb;
        shi = np ? (cp ? cap - 16 : lit_hi) : shi;
        // zero region (D == 0, reader.go:176-179) or a short-period run: one 16-byte pattern
        // stored every `step` bytes; a short literal is in the header's 16 bytes already
        src = np ? (run || (!cp && j + L <= 16) ? 1 : (cp && D <= kNear ? 2 : 0)) : src;
        step = np ? (run ? run_step(D) : 16) : step;
        pv.lo = np ? hv.lo : pv.lo;
        pv.hi = np ? hv.hi : pv.hi;
        if (any_lane(np && run)) {  // (after the store: the pattern's source may be this move's bytes)
            if (np && run) pv = run_pattern(shr16(ring_ld(ring, pos - 16), 16 - D), D);  // D == 0: zeros
        }
        pos = np ? pos + L : pos;
        // finished 128-byte chunks of output leave the ring as whole lines, every fper-th
        // iteration: one wave-wide block every fper iterations with many lanes active, not
        // one nearly every iteration for the few lanes that just finished a chunk (16-byte
        // pieces stored every iteration, and the fixed store count that lets the waits count
        // past them, measured slower: 0.75 against 0.57 ms at C1)
        // (unflushed output stays below kChunk + 31 * (fper + 1) <= kRing - 16 bytes)
        if ((++it & (fper - 1)) == 0) {
#if (EZ_EXP & (1 << 26))  // timing builds: no flush (wrong bytes)
            if (it) {} else
#endif
            while (any_lane(dst >= fl + kChunk)) {
                if (dst >= fl + kChunk) {
#pragma unroll
                    for (int32_t t = 0; t < kChunk; t += 16) st16v(out + fl + t, ring_ld(ring, fl + t));
                    fl += kChunk;
                }
            }
        }
        slow = slow || ho;
        rem = ho ? 0 : rem;
        live = live && !fin && !ho;
        // the HBM source of the next iteration's move, loaded now (every lane one load: the
        // clamped address for a source at the batch's or the slot's edge, fixed up after the
        // wait; A.in for the others, the batch holds >= 16 bytes when any lane is live), so the
        // next iteration's parse and header load run while it is in flight
        {
            const bool hn = rem > 0 && src == 0;
            int32_t sc = so > 0 ? so : 0;
            sc = sc < shi ? sc : shi;  // (a copy before the slot's start, a literal at the batch's end)
            // (the others all load the batch's first line: one line per wave instead of a gather)
            const uint8_t *gc = hn ? sb + sc : A.in;
#if (EZ_EXP & (1 << 25))  // timing builds: far copies read a line at the slot's start (wrong bytes; C1 only)
            gc = hn && sb == out ? out + ((uint32_t)so & 63) : gc;
#endif
            graw = ld16v(gc);
            gd = so - sc;  // (hn lanes: the clamp's shift)
            sched_fence();            // (issued here, not sunk to the next iteration's parse)
        }
    }
#ifndef __HIP_DEVICE_COMPILE__
    g_ring_iters += it;  // (the host emulation counts the iterations: tools/ring_emu)
#endif
    if (!slow) {  // the last partial chunk, exact bytes
        int32_t q = fl;
        for (; q + 16 <= pos; q += 16) st16v(out + q, ring_ld(ring, q));
        if (q < pos) put_small(out + q, ring_ld(ring, q), (uint32_t)(pos - q));
    }
    if (!slow) {
        A.out_size[s] = (uint64_t)pos;
        if (A.status) A.status[s] = EZ_OK;
    }
    return !slow;
}

// spw: streams per wave (lanes spw..63 idle): fewer streams per wave put more
// waves on each SIMD within the same LDS
template <bool HW>
__global__ __launch_bounds__(kRingBlock) void k2_ring(DecompressArgs A, uint32_t spw, uint32_t fper) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (l >= spw) return;
    uint8_t *ring = smem + (w * spw + l) * kRingStride + 16;
    const uint64_t per_block = (uint64_t)(kRingBlock / 64) * spw;
    for (uint64_t s = (uint64_t)blockIdx.x * per_block + w * spw + l; s < A.count; s += (uint64_t)gridDim.x * per_block)
        if (!ring_one<HW>(A, s, ring, fper)) {
            const uint32_t at = atomicAdd(&A.slow[0], 1u);
            A.slow[1 + at] = (uint32_t)s;
        }
}

}  // namespace

hipError_t launch_decompress_ring(const DecompressArgs &a, hipStream_t st) {
    static const uint32_t spw = (uint32_t)knob("EZ_K2R_SPW", 64);
    static bool attr_done = false;
    const size_t lds = (size_t)(kRingBlock / 64) * spw * kRingStride;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k2_ring<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k2_ring<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    static const bool hw = knob("EZ_K2R_HW", 0) != 0;  // A/B (experiment builds): the aligned header window
    const uint64_t per_block = (uint64_t)(kRingBlock / 64) * spw;
    const uint64_t grid = (a.count + per_block - 1) / per_block;
    // EZ_K2R_FLUSH (A/B): iterations between ring flushes, a power of two <= kMaxFlushPer
    static const uint32_t fper = [] {
        const uint32_t v = (uint32_t)knob("EZ_K2R_FLUSH", 8);
        return v >= 1 && v <= kMaxFlushPer && (v & (v - 1)) == 0 ? v : 8u;
    }();
    if (hw) hipLaunchKernelGGL(k2_ring<true>, dim3((unsigned)grid), dim3(kRingBlock), lds, st, a, spw, fper);
    else hipLaunchKernelGGL(k2_ring<false>, dim3((unsigned)grid), dim3(kRingBlock), lds, st, a, spw, fper);
    return hipGetLastError();
}

}  // namespace ez
