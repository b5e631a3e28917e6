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
constexpr uint32_t kMaxFlushPer = 16;    // kChunk + 16 * (16 + 1) < kRing

typedef uint64_t __attribute__((aligned(1))) u64_ua;

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

// The common token forms from the header's first 8 bytes, in 32-bit arithmetic without
// branches: a 1-byte tag (length 1..123; not padding, not a meta) and, for a copy, a 1..3-byte
// offset (plain, Off1 or Off2, reader.go:422-472) after an optional long prefix (:394-420).
// false: another form (k2_parse decides).  D is the copy distance, adv the input bytes taken.
__host__ __device__ __forceinline__ bool fast_tok(uint64_t lo, int32_t &L, int32_t &adv, uint32_t &D, bool &cp) {
    const uint32_t w0 = (uint32_t)lo;
    const uint32_t l7 = w0 & 0x7f;
    cp = (w0 & 0x80) != 0;
    L = (int32_t)l7;
    const bool lng = (w0 & 0xff00) == 0xff00;
    const uint32_t y = (uint32_t)(lo >> (lng ? 16 : 8));  // the offset's bytes
    const uint32_t o = y & 0xff;
    const uint32_t D0 = o < 252 ? o : (o == 252 ? 252 + ((y >> 8) & 0xff) : 508 + ((y >> 8) & 0xffff));
    D = lng ? D0 : D0 + l7;
    adv = cp ? 2 + (int32_t)lng + (o < 252 ? 0 : (int32_t)o - 251) : 1 + L;
    return l7 != 0 && l7 < 124 && (!cp || o < 254);
}

// decodes stream s with `ring` (kRing + 16 bytes, with 16-byte guards on both sides) as its history; false = hand
// the stream over (host-compilable: tools/ring_emu.hip runs it on the CPU)
// fper: iterations between flushes (a power of two <= kMaxFlushPer)
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
    for (int32_t k = 0; k < kRing + 16; k += 16) {
        *(u64_ua *)(ring + k) = 0;
        *(u64_ua *)(ring + k + 8) = 0;
    }
    int32_t i = 0, pos = 0, bsl = -1;  // bsl: log2 of the window after MetaReset (-1: none yet)
    uint32_t win = 0;                  // the window's size once bsl is set (copies farther hand over)
    V16 h{0, 0};                       // 16 bytes at b + i (the next header)
    if (!slow) h = ld_in(b, A.in, in_end);
    // the token being written: rem bytes at dst from sp (input / HBM output) or from the ring
    int32_t rem = 0, dst = 0, step = 16, rp = 0, fl = 0;  // fl: output below it is in HBM
    uint32_t it = 0;
    const uint8_t *sp = b;
    bool from_in = false, patt = false, near = false;
    V16 pv{0, 0};
    for (;;) {
        if (rem == 0) {
            if (i >= nb) break;
            // the common forms branch-free; anything else (padding, metas, long tags and
            // offsets, a check that fails) takes the full parse, which may hand over
            int32_t L, adv, j = 1;
            uint32_t D;
            bool cp;
            const bool f = fast_tok(h.lo, L, adv, D, cp) && bsl >= 0 && i + adv <= nb && pos + L <= cap && L <= lim32 && (!cp || D <= win);
            V16 hv{(h.lo >> 8) | (h.hi << 56), h.hi >> 8};  // the header after a 1-byte tag
            if (!f) {
                K2Tok t;
                const int r = k2_parse(h, i, nb, pos, cap, lim32, limit, bsl, t);
                if (r == kParseHandOver) { slow = true; break; }  // the exact decoder takes the stream
                L = t.L;
                adv = t.adv;
                j = t.j;
                D = t.D;
                cp = t.cp;
                win = bsl < 0 ? 0u : (bsl >= 30 ? 0xffffffffu : 1u << bsl);
                hv = shr16(h, (uint32_t)j);
            }
            {  // the token's state, set by every step (a padding or meta step has L = 0: no move)
                dst = pos;
                rem = L;
                pos += L;
                from_in = !cp;
                near = cp && D <= kNear;
                rp = dst - (int32_t)D;
                sp = cp ? out + rp : b + (i + j);
                // zero region (D == 0, reader.go:176-179) or a short-period run: one 16-byte
                // pattern stored every `step` bytes; a short literal is in the header's 16
                // bytes already
                const bool run = cp && D < 16;
                patt = run || (!cp && j + L <= 16);
                step = run ? run_step(D) : 16;
                pv = hv;
                if (run) pv = run_pattern(shr16(ring_ld(ring, dst - 16), 16 - D), D);  // D == 0: zeros
            }
            i += adv;
            // the next header, loaded beside this token's first move
            if (i < nb) h = ld_in(b + i, A.in, in_end);
        }
        if (rem > 0) {
            // the ring read is taken by every lane (one LDS read, no branch level); only far
            // copies and long literals load from HBM
            V16 v = patt ? pv : ring_ld(ring, rp);
            if (!patt && !near) {
                if (from_in ? sp + 16 > in_end : sp < out) v = from_in ? ld_clamped16(sp, A.in, in_end) : ld_clamped16(sp, out, out + cap);
                else v = ld16v(sp);
            }
            ring_st(ring, dst, v);
            const int32_t kk = rem < step ? rem : step;
            dst += kk;
            sp += kk;
            rp += kk;
            rem -= kk;
        }
        // finished 128-byte chunks of output leave the ring as whole lines, every fper-th
        // iteration: the lanes of a wave iterate together, so the flush is one wave-wide
        // block every fper iterations with many lanes active, not one nearly every
        // iteration for the few lanes that just finished a chunk (unflushed output stays
        // below kChunk + 16 * (fper + 1) <= kRing bytes)
        if ((++it & (fper - 1)) == 0) {
            while (dst >= fl + kChunk) {
#pragma unroll
                for (int32_t t = 0; t < kChunk; t += 16) st16v(out + fl + t, ring_ld(ring, fl + t));
                fl += kChunk;
            }
        }
    }
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
__global__ __launch_bounds__(kRingBlock) void k2_ring(DecompressArgs A, uint32_t spw, uint32_t fper) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (l >= spw) return;
    uint8_t *ring = smem + (w * spw + l) * kRingStride + 16;
    const uint64_t per_block = (uint64_t)(kRingBlock / 64) * spw;
    for (uint64_t s = (uint64_t)blockIdx.x * per_block + w * spw + l; s < A.count; s += (uint64_t)gridDim.x * per_block)
        if (!ring_one(A, s, ring, fper)) {
            const uint32_t at = atomicAdd(&A.slow[0], 1u);
            A.slow[1 + at] = (uint32_t)s;
        }
}

}  // namespace

hipError_t launch_decompress_ring(const DecompressArgs &a, hipStream_t st) {
    static const uint32_t spw = getenv("EZ_K2R_SPW") ? (uint32_t)atoi(getenv("EZ_K2R_SPW")) : 64u;
    static bool attr_done = false;
    const size_t lds = (size_t)(kRingBlock / 64) * spw * kRingStride;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k2_ring, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const uint64_t per_block = (uint64_t)(kRingBlock / 64) * spw;
    const uint64_t grid = (a.count + per_block - 1) / per_block;
    // EZ_K2R_FLUSH (A/B): iterations between ring flushes, a power of two <= kMaxFlushPer
    static const uint32_t fper = [] {
        const uint32_t v = getenv("EZ_K2R_FLUSH") ? (uint32_t)atoi(getenv("EZ_K2R_FLUSH")) : 8u;
        return v >= 1 && v <= kMaxFlushPer && (v & (v - 1)) == 0 ? v : 8u;
    }();
    hipLaunchKernelGGL(k2_ring, dim3((unsigned)grid), dim3(kRingBlock), lds, st, a, spw, fper);
    return hipGetLastError();
}

}  // namespace ez
