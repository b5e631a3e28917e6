// ez_decompress_small.hip — K2s: batch decompression of small streams (output slots of at most
// 4 KiB: the C1 / C3 configurations) in two kernels, a parse and a move.
//
// Restates Reader.Read to EOF for NewReaderBytes (reader.go:116-216 read, readTag :218-270,
// continueMetaTag :272-325, reset :327-344, Decoder :346-514) for the common case through the
// token parse K2r uses (ez_k2_parse.h); anything else hands the stream to the exact decoder
// (ez_decompress.hip).
//
// Why two kernels.  K2r (a lane per stream, ez_decompress_ring.hip) runs Reader.read's token chain
// with every header and every far copy source a 64-address gather on the chain: at C1 the chip
// holds one such wave per SIMD and waits on those loads in every iteration.  Here the chain is
// split from the bytes:
//
//  K2p (k2_pre), a lane per stream: only the token walk — every step the parse of K2r (fast_tok,
//    k2_parse for padding, metas and long forms, every check: window, slot room, block size
//    limit) — from an LDS ring of the lane's input, refilled 128 bytes at a time one step ahead
//    (the loads of step k+1 are in flight while step k parses), so no global load sits on the
//    chain.  It writes one bit per input byte: the token starts (literal and copy tokens only),
//    in a per-stream region of the workspace, and the token count (or "hand over").
//  K2q (k2_small), 16 lanes per stream, 4 streams per wave: the whole output of a stream in LDS;
//    the bitmap becomes a list of token starts (popcount prefix sum), then rounds of 16 tokens,
//    one per lane: each lane parses its token from the 32 input bytes at its start (loaded one
//    round ahead), a prefix sum over the 16 lanes (DPP) gives every token's output position,
//    the literals are written at once, the copies in batches (every copy up to the first one
//    whose source reaches into the batch's own output; copies whose source is final at the
//    round's start run in any batch), and the finished output leaves LDS in 256-byte pieces.
//    No copy ever reads HBM: a 4 KiB stream's history is all in LDS.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"
#include "ez_k2_parse.h"

namespace ez {

namespace {

typedef uint64_t __attribute__((aligned(1))) u64_ua;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef uint16_t __attribute__((aligned(1))) u16_ua;

constexpr uint32_t kSHandOver = 0xffffffffu;

// whether c holds on any lane of the wave
__device__ __forceinline__ bool any_lane(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0; }

__device__ __forceinline__ V16 lds16(const uint8_t *p) { return V16{*(const u64_ua *)p, *(const u64_ua *)(p + 8)}; }

// 16 bytes at y of the batch [lo, hi) (hi - lo >= 16; bytes from hi on read as 0)
__device__ __forceinline__ V16 ld_batch(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    return y + 16 <= hi ? ld16v(y) : ld_clamped16(y, lo, hi);
}

// ---------------------------------------------------------------------------------------------
// K2p: the token walk, a lane per stream
// ---------------------------------------------------------------------------------------------
constexpr int kPBlock = 256;
constexpr int32_t kPRing = 256;                // input ring bytes per lane
constexpr int32_t kPStride = kPRing + 16;      // + a mirror of its first 16 bytes
constexpr int32_t kPRefill = 128;              // bytes a lane's refill brings
constexpr int kPStep = 8;                      // tokens parsed per refill step (<= 16 bytes each)

// the refill of one lane: 128 bytes of the stream from input position at
struct Refill {
    V16 v[kPRefill / 16];
};

__device__ __forceinline__ void refill_issue(Refill &r, const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    // (loads past the batch's last 16 bytes clamp and shift; only the batch's last stream reaches them)
    const bool edge = y + kPRefill > hi;
    if (any_lane(edge)) {
#pragma unroll
        for (int k = 0; k < kPRefill / 16; k++) r.v[k] = ld_batch(y + 16 * k, lo, hi);
    } else {
#pragma unroll
        for (int k = 0; k < kPRefill / 16; k++) r.v[k] = ld16v(y + 16 * k);
    }
}

__device__ __forceinline__ void refill_commit(const Refill &r, uint8_t *ring, int32_t at) {
#pragma unroll
    for (int k = 0; k < kPRefill / 16; k++) {
        const int32_t slot = (at + 16 * k) & (kPRing - 1);
        *(u64_ua *)(ring + slot) = r.v[k].lo;
        *(u64_ua *)(ring + slot + 8) = r.v[k].hi;
        if (slot == 0) {  // the mirror: a 16-byte read at any slot is one contiguous access
            *(u64_ua *)(ring + kPRing) = r.v[k].lo;
            *(u64_ua *)(ring + kPRing + 8) = r.v[k].hi;
        }
    }
}

// the token walk of stream s (valid: s < count) with `ring` (kPStride bytes of LDS) as its input
// window; writes its region of the bitmap workspace (kSmallRegion words: [0] the token count or
// kSHandOver, then one bit per input byte set at every literal or copy token's first byte)
__device__ __forceinline__ void pre_one(const DecompressArgs &A, const uint64_t s, const bool valid, uint8_t *ring, uint32_t *bm) {
    const uint64_t sc = valid ? s : 0;
    const uint8_t *b = A.in + A.in_off[sc];
    const int64_t nb64 = (int64_t)(A.in_off[sc + 1] - A.in_off[sc]);
    const uint8_t *in_end = A.in + A.in_off[A.count];
    const int64_t cap64 = (int64_t)(A.out_off[sc + 1] - A.out_off[sc]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;  // 0: no limit
    uint32_t *reg = bm + sc * (uint64_t)kSmallRegion;
    // what K2s takes: slots of <= 4 KiB, streams of <= kSmallIn bytes, batches of >= 16 bytes
    const bool fits = in_end - A.in >= 16 && nb64 <= kSmallIn && cap64 <= kSmallOut;
    bool live = valid && fits, ho = valid && !fits;
    const int32_t nb = live ? (int32_t)nb64 : 0, cap = (int32_t)cap64;
    int32_t i = 0, pos = 0, bsl = -1, win = 0, ntok = 0;
    int32_t F = 0;       // the ring holds input [F - kPRing, F) (what has been committed)
    int32_t cw = 0;      // bitmap word being built
    uint32_t acc = 0;
    live = live && nb > 0;
    Refill r;
    // prologue: the first 128 bytes, waited for
    if (any_lane(live)) {
        refill_issue(r, b, A.in, in_end);
        if (live) refill_commit(r, ring, 0);
        F = live ? kPRefill : 0;
    }
    while (any_lane(live)) {
        // a lane whose next header lies past its window restarts it there; a lane with at most
        // 128 bytes ahead (the oldest half of its ring is behind it) refills the next 128
        if (live && i >= F) F = i & ~15;
        const bool rf = live && F - i <= kPRing - kPRefill && F < nb + 16;
        if (any_lane(rf)) {
            if (rf) refill_issue(r, b + F, A.in, in_end);
        }
        // up to kPStep tokens from the ring while the refill is in flight
#pragma unroll 1
        for (int st = 0; st < kPStep; st++) {
            const bool rd = live && i + 16 <= F;
            if (!any_lane(rd)) break;
            const V16 h = lds16(ring + (i & (kPRing - 1)));
            int32_t L, adv;
            uint32_t D;
            bool cp;
            const int32_t ft = fast_tok(h.lo, L, adv, D, cp);
            const bool f = (ft | bsl | (nb - i - adv) | (cap - pos - L) | (lim32 - L) | (cp ? win - (int32_t)D : 0)) >= 0;
            bool tok = true, bad = false;
            if (any_lane(rd && !f)) {
                if (rd && !f) {
                    K2Tok t;
                    const int rr = k2_parse(h, i, nb, pos, cap, lim32, limit, bsl, t);
                    if (rr == kParseHandOver) {
                        bad = true;
                    } else {
                        L = t.L;
                        adv = t.adv;
                        tok = rr == kParseToken;
                        win = bsl < 0 ? 0 : (bsl >= 30 ? 0x7fffffff : 1 << bsl);
                    }
                }
            }
            const bool go = rd && !bad;
            const bool mark = go && tok;
            // the bitmap: a word is stored when the walk leaves it (the words it jumps over are 0)
            const int32_t wi = i >> 5;
            const bool nw = mark && wi != cw;
            if (any_lane(nw)) {
                if (nw) {
                    reg[1 + cw] = acc;
#pragma unroll 1
                    for (int32_t x = cw + 1; x < wi; x++) reg[1 + x] = 0;
                    cw = wi;
                    acc = 0;
                }
            }
            acc = mark ? acc | (1u << (i & 31)) : acc;
            ntok += mark ? 1 : 0;
            pos = go ? pos + (tok ? L : 0) : pos;
            i = go ? i + adv : i;
            ho = ho || (rd && bad);
            live = live && !(rd && bad) && i < nb;
        }
        if (any_lane(rf)) {
            if (rf) refill_commit(r, ring, F);
        }
        F = rf ? F + kPRefill : F;
    }
    if (valid && !ho) {  // the last word, the words after it, the count
        const int32_t nw = (nb + 31) >> 5;
        if (nw > 0) reg[1 + cw] = acc;
        for (int32_t x = cw + 1; x < nw; x++) reg[1 + x] = 0;
        reg[0] = (uint32_t)ntok;
    }
    if (ho) {
        reg[0] = kSHandOver;
        const uint32_t at = atomicAdd(&A.slow[0], 1u);
        A.slow[1 + at] = (uint32_t)s;
    }
}

__global__ __launch_bounds__(kPBlock) void k2_pre(DecompressArgs A, uint32_t *bm) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *ring = smem + threadIdx.x * kPStride;
    for (uint64_t s0 = (uint64_t)blockIdx.x * kPBlock; s0 < A.count; s0 += (uint64_t)gridDim.x * kPBlock) {
        const uint64_t s = s0 + threadIdx.x;
        pre_one(A, s, s < A.count, ring, bm);
    }
}

// ---------------------------------------------------------------------------------------------
// K2q: the moves, 16 lanes per stream (one DPP row), the stream's whole output in LDS
// ---------------------------------------------------------------------------------------------
constexpr int kQBlock = 256;
constexpr int kQG = 16;                        // lanes per stream: one DPP row
constexpr int kQPer = kQBlock / kQG;           // streams per block
constexpr int32_t kQList = 256;                // token starts per 512-position chunk at most (tokens take >= 2 bytes)
// per stream: [16 zero bytes: the history before the stream][output][token list u16][trash 8 B per lane]
constexpr int32_t kQOut = 16, kQListAt = kQOut + kSmallOut, kQTrash = kQListAt + 2 * kQList;
constexpr int32_t kQStride = kQTrash + 8 * kQG;
static_assert(kQStride % 16 == 0, "16-byte aligned groups");

// DPP within a row of 16 lanes
__device__ __forceinline__ int32_t row_shr(int32_t v, int n) {  // lane k gets lane k - n's value, 0 below the row
    switch (n) {
        case 1: return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
        case 2: return __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
        case 4: return __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
        default: return __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
    }
}
__device__ __forceinline__ int32_t row_ror(int32_t v, int n) {  // rotate within the row
    switch (n) {
        case 1: return __builtin_amdgcn_update_dpp(v, v, 0x121, 0xf, 0xf, false);
        case 2: return __builtin_amdgcn_update_dpp(v, v, 0x122, 0xf, 0xf, false);
        case 4: return __builtin_amdgcn_update_dpp(v, v, 0x124, 0xf, 0xf, false);
        default: return __builtin_amdgcn_update_dpp(v, v, 0x128, 0xf, 0xf, false);
    }
}
__device__ __forceinline__ int32_t row_incl_sum(int32_t v) {
    v += row_shr(v, 1);
    v += row_shr(v, 2);
    v += row_shr(v, 4);
    v += row_shr(v, 8);
    return v;
}
__device__ __forceinline__ int32_t row_last(int32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x15F, 0xf, 0xf, false); }  // row_newbcast:15
__device__ __forceinline__ int32_t row_min(int32_t v) {
    v = min(v, row_ror(v, 1));
    v = min(v, row_ror(v, 2));
    v = min(v, row_ror(v, 4));
    v = min(v, row_ror(v, 8));
    return v;
}

// the first n bytes (0..16) of v at d, without branches: the absent pieces go to trash (8 bytes)
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

// bytes j .. j+15 of the 32 bytes (a, b), 0 <= j <= 16
__device__ __forceinline__ V16 at32(V16 a, V16 b, uint32_t j) {
    const V16 x = shr16(a, j), y = shl16(b, 16 - j);
    return V16{x.lo | y.lo, x.hi | y.hi};
}

// 16 output bytes at position x (x >= -16 reads the zero history before the stream from the guard)
__device__ __forceinline__ V16 out16(const uint8_t *ob, int32_t x) {
    const V16 v = lds16(ob + (x < -16 ? -16 : x));
    return x < -16 ? V16{0, 0} : v;
}

__device__ __forceinline__ int32_t run_step_of(int32_t per) { return per * (16 / per); }

// streams s .. s+3 of a wave (s = base + row); ob: the row's LDS output, list, trash
__device__ __forceinline__ void small_one(const DecompressArgs &A, const uint32_t *bm, const uint64_t s, const int k, uint8_t *ob,
                                          uint16_t *list, uint8_t *trash) {
    const bool v0 = s < A.count;
    const uint64_t sc = v0 ? s : 0;
    const uint32_t *reg = bm + sc * (uint64_t)kSmallRegion;
    const bool valid = v0 && reg[0] != kSHandOver;
    const uint8_t *b = A.in + A.in_off[sc];
    const uint8_t *in_end = A.in + A.in_off[A.count];
    const int32_t nb = valid ? (int32_t)(A.in_off[sc + 1] - A.in_off[sc]) : 0;
    const int32_t nwd = (nb + 31) >> 5;  // bitmap words
    int32_t pos = 0;
    uint32_t wnext = k < nwd ? reg[1 + k] : 0;
#pragma unroll 1
    for (int32_t w0 = 0; any_lane(w0 < nwd); w0 += kQG) {
        // ---- the chunk's token starts (512 input positions): a row prefix sum of the popcounts
        uint32_t word = wnext;
        wnext = w0 + kQG + k < nwd ? reg[1 + w0 + kQG + k] : 0;  // (the next chunk's words, in flight)
        const int32_t c = __builtin_popcount(word);
        const int32_t ci = row_incl_sum(c);
        const int32_t nt = row_last(ci);
        int32_t e = ci - c;
        const int32_t wbase = (w0 + k) << 5;
        while (any_lane(word != 0)) {
            if (word != 0) {
                list[e++] = (uint16_t)(wbase + (int32_t)__builtin_ctz(word));
                word &= word - 1;
            }
        }
        // ---- rounds of 16 tokens, one per lane; the next round's headers load during this one
        V16 n0{0, 0}, n1{0, 0};
        {
            const int32_t q = k < nt ? (int32_t)list[k] : 0;
            n0 = ld_batch(b + q, A.in, in_end);
            n1 = ld_batch(b + q + 16, A.in, in_end);
        }
#pragma unroll 1
        for (int32_t t0 = 0; any_lane(t0 < nt); t0 += kQG) {
            const bool has = t0 + k < nt;
            const int32_t q = has ? (int32_t)list[t0 + k] : 0;
            const V16 a0 = n0, a1 = n1;
            {
                const int32_t qn = t0 + kQG + k < nt ? (int32_t)list[t0 + kQG + k] : 0;
                n0 = ld_batch(b + qn, A.in, in_end);
                n1 = ld_batch(b + qn + 16, A.in, in_end);
            }
            // ---- the token (K2p checked every one: the common forms branch-free, the long ones by k2_scan)
            int32_t L, fadv, j = 1;
            uint32_t Du;
            bool cp;
            const int32_t ft = fast_tok(a0.lo, L, fadv, Du, cp);
            if (any_lane(has && ft < 0)) {
                if (has && ft < 0) {
                    K2Tok t;
                    (void)k2_scan(a0, q, nb, 0x7fffffff, 0, t);
                    L = t.L;
                    j = t.j;
                    Du = t.D;
                    cp = t.cp;
                }
            }
            L = has ? L : 0;
            cp = has && cp;
            const int32_t D = cp ? (int32_t)Du : 0;
            const int32_t incl = row_incl_sum(L);
            const int32_t total = row_last(incl);
            const int32_t dst = pos + incl - L;
            // ---- literals: their bytes from the 32 loaded at the token's start, or the input
            const bool lit = has && !cp;
            put_exact(lit ? ob + dst : trash, at32(a0, a1, (uint32_t)j), lit ? (uint32_t)(L < 16 ? L : 16) : 0u, trash);
#pragma unroll 1
            for (int32_t p = 16; any_lane(lit && p < L); p += 16) {
                const bool act = lit && p < L;
                V16 v = shr16(a1, (uint32_t)j);  // bytes j+16 .. 31: enough when L <= 32 - j
                const bool ld = act && (p > 16 || L > 32 - j);
                if (any_lane(ld)) {
                    if (ld) v = ld_batch(b + q + j + p, A.in, in_end);
                }
                put_exact(act ? ob + dst + p : trash, v, act ? (uint32_t)(L - p < 16 ? L - p : 16) : 0u, trash);
            }
            // ---- copies in batches: a batch runs from the first pending copy up to the first one
            // whose source reaches past that copy's output position (the output before it is final);
            // a copy whose source ends before the round's first byte (or a zero region) is final now
            const int32_t cs = dst - D;
            const int32_t need = cs + (D < L ? D : L);
            const bool fre = cp && (D == 0 || need <= pos);
            bool pend = cp;
            const uint32_t rsh = (uint32_t)(threadIdx.x & 48);
#pragma unroll 1
            while (any_lane(pend)) {
                const int32_t oa = row_min(pend ? dst : 0x7fffffff);
                const bool br = pend && !fre && dst > oa && need > oa;
                const uint32_t bb = (uint32_t)(__builtin_amdgcn_ballot_w64(br) >> rsh) & 0xffffu;
                const int32_t bnd = (int32_t)__builtin_ctz(bb | 0x10000u);
                const bool ex = pend && (fre || k < bnd);
                pend = pend && !ex;
                // the common copy: D >= 16, at most 16 bytes: one read, one write
                int32_t stp = 16;
                V16 pv{0, 0};
                const bool run = ex && D > 0 && D < 16;
                if (any_lane(run)) {
                    if (run) {
                        pv = run_pattern(shr16(out16(ob, dst - 16), (uint32_t)(16 - D)), (uint32_t)D);
                        stp = run_step_of(D);
                    }
                }
                int32_t o = 0;
                while (any_lane(ex && o < L)) {
                    const bool act = ex && o < L;
                    const V16 v = D >= 16 ? out16(ob, cs + o) : pv;  // (D == 0: zeros)
                    put_exact(act ? ob + dst + o : trash, v, act ? (uint32_t)(L - o < 16 ? L - o : 16) : 0u, trash);
                    o += stp;
                }
            }
            pos += total;
        }
    }
    // ---- the output to its slot, 256 bytes per row and step
    if (valid) {
        uint8_t *out = A.out + A.out_off[sc];
        for (int32_t x = 16 * k; x < pos; x += 16 * kQG) {
            const V16 v = lds16(ob + x);
            if (x + 16 <= pos) st16v(out + x, v);
            else put_small(out + x, v, (uint32_t)(pos - x));
        }
        if (k == 0) {
            A.out_size[sc] = (uint64_t)pos;
            if (A.status) A.status[sc] = EZ_OK;
        }
    }
}

__global__ __launch_bounds__(kQBlock) void k2_small(DecompressArgs A, const uint32_t *bm) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int row = (int)(threadIdx.x >> 4), k = (int)(threadIdx.x & 15);
    uint8_t *g = smem + row * kQStride;
    if (k == 0) {  // the zero history before every stream
        *(u64_ua *)g = 0;
        *(u64_ua *)(g + 8) = 0;
    }
    for (uint64_t base = (uint64_t)blockIdx.x * kQPer; base < A.count; base += (uint64_t)gridDim.x * kQPer)
        small_one(A, bm, base + row, k, g + kQOut, (uint16_t *)(g + kQListAt), g + kQTrash + 8 * k);
}

}  // namespace

hipError_t launch_decompress_small(const DecompressArgs &a, uint32_t *bm, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k2_pre, hipFuncAttributeMaxDynamicSharedMemorySize, kPBlock * kPStride);
        (void)hipFuncSetAttribute((const void *)k2_small, hipFuncAttributeMaxDynamicSharedMemorySize, kQPer * kQStride);
        attr_done = true;
    }
    const uint64_t gp = (a.count + kPBlock - 1) / kPBlock;
    hipLaunchKernelGGL(k2_pre, dim3((unsigned)(gp < (1u << 30) ? gp : (1u << 30))), dim3(kPBlock), kPBlock * kPStride, st, a, bm);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint64_t gq = (a.count + kQPer - 1) / kQPer;
    hipLaunchKernelGGL(k2_small, dim3((unsigned)(gq < (1u << 30) ? gq : (1u << 30))), dim3(kQBlock), kQPer * kQStride, st, a, bm);
    return hipGetLastError();
}

}  // namespace ez
