// ez_decompress_jump.hip — K2j: the decode of a few long streams with the whole chip.
//
// Reader.read (reader.go:143-216) is a chain twice over: every token starts where the previous one
// ends (readTag :218-270), and every copied byte reads output written before it (:173-201).  K2t
// runs both chains on one wave per stream, which leaves a batch of a few long streams (a Reader
// handle's one stream, C4's 64 buckets, 1 MiB streams) to a handful of waves on a 1,024-SIMD chip.
// K2j cuts both chains into data-parallel steps:
//
//  1. token starts (kj_spec, kj_verify, kj_fix): the compressed stream is cut into 1 KiB chunks; a
//     lane per chunk parses speculatively from kJWarm bytes before the chunk and records the
//     positions it visits inside it (a bitmap) and where it leaves it.  A wrong start parses
//     garbage, but its chain meets the true one within a few tokens (median ~110 bytes on the log
//     streams; 99 % within 1 KiB), after which both are the same chain, so the warm-up has usually
//     met it before the chunk starts.  kj_verify (a lane per chunk, all in parallel) takes chunk j's
//     entry to be chunk j-1's speculative exit and walks the true chain from it until it meets a
//     recorded position (the chunk's exit is then the speculative one) or leaves the chunk.
//     kj_fix (a wave per stream) finds, 64 chunks per step, the first chunk whose assumed entry
//     differs from its predecessor's true exit and re-walks only that chunk (rare); an entry past a
//     chunk (inside a long token) skips to the chunk it lies in.
//  2. tokens (kj_tok, kj_scan, kj_place): a lane per chunk walks the true chain from its entry
//     once, checks every form (k2_scan, ez_k2_parse.h) and writes a chunk-local record per token
//     (output position from the chunk's start, length, distance or input position), its token and
//     output counts, the longest distance and its Breaks; a wave per stream scans the chunks'
//     counts into token and output positions and validates the stream as K2t does (one MetaReset
//     before any output, the window set before the first token, every distance within the window,
//     the output within the slot); kj_place moves each chunk's records into the stream's array.
//  3. bytes (kj_expand): a thread per 16 output bytes finds its tokens (a binary search over the
//     stream's records), writes literal bytes and zero regions, and for every copied byte p a
//     pointer ptr[p] = p - D (a marker for bytes before the stream start: the fresh window's zeros,
//     SURVEY A.12; a Reader's continuation points into the history placed before out_off[0]);
//     literal, zero and history bytes point at themselves.
//  4. copies (kj_jump): pointer jumping, ptr[p] = ptr[ptr[p]] over all bytes, until every pointer
//     names a literal byte, a zero byte or the zero marker: ceil(log2(chain depth)) passes, each a
//     sequential read and a gather that stays mostly local (copy distances are short).  Passes
//     after the one that changed nothing return at once (the launcher queues a fixed number, so
//     nothing waits on the host).
//  5. kj_gather writes every copied byte from its resolved source; kj_final reports each stream
//     (out_size, status, Break positions, a Reader's end state) or hands it to the exact decoder.
//
// Continuation (DecompressArgs.c_on, a NewReader's read-ahead, ez_capi.hip stream_ahead): one stream
// whose history (c_hist bytes) sits before out_off[0]; the chain stops before a token the input ends
// inside of, a literal whose body runs past the input is output as far as it goes, and the end state
// says where the input was left.
//
// Streams K2j cannot take as a whole (an error, a form k2_scan hands over, a MetaReset after output,
// a slot too small) go to the exact decoder (ez_decompress.hip), which recomputes them from the start.
#include <hip/hip_runtime.h>

#include "ez_bytes.h"
#include "ez_cache.h"
#include "ez_internal.h"
#include "ez_k2_parse.h"

namespace ez {
namespace {

constexpr int32_t kJC = 1024;                        // compressed bytes per chunk at most (JWork.jc: 1,024 or 256)
constexpr int32_t kJW = kJC / 32;                    // bitmap words per chunk
constexpr uint32_t kJGap = 0xffffffffu;              // ptr: not a byte of any stream's output
constexpr uint32_t kJZero = 0xfffffffeu;             // ptr: a zero byte of the history before the stream
constexpr uint32_t kJCopy = 0x80000000u;             // JTok.kd: a copy (distance in the low bits; 0: zero region)
constexpr int kJPasses = 34;                         // pointer-jumping passes at most (chains up to 2^34)
constexpr uint32_t kJRec = kJC / 2 + 2;              // token records of a chunk at most (a token takes >= 2 bytes)

struct JHead {
    uint32_t chunk0, nchunk;  // the stream's chunks
    uint32_t state;           // 0: K2j decodes it; 1: handed over
    int32_t bsl;              // log2 of the window (MetaReset)
    uint64_t total;           // output bytes
    uint64_t ntok;            // token records
    uint64_t tok0;            // its first record
    // (c_on) where the chain stops: the input consumed by whole tokens, and a literal starting there
    // whose body runs past the input (its header length, its length; 0: none)
    int32_t tstop, tj;
    int64_t tL;
};

// the ptr array's first byte: out_off[0] less the continuation's history, rounded down to 16 bytes
__device__ __forceinline__ uint64_t jg0(const DecompressArgs &A) {
    return (A.out_off[0] - (A.c_on ? A.c_hist : 0)) & ~15ull;
}

struct JTok {
    uint32_t dst, L, kd, src;  // output position, length, kJCopy | distance (or 0: literal), literal's input position
};

struct JWork {
    JHead *head;
    uint32_t *cbase;    // count+1: first chunk of each stream (and the total)
    uint32_t *entry, *sexit, *bits;
    uint32_t *cnt;      // tokens of a chunk's true chain
    uint64_t *cout;     // output bytes of a chunk
    uint32_t *cflag;    // kJF* bits, bits 8-15: the chunk's last MetaReset
    uint64_t *ctbase, *cobase;
    JTok *tok;
    uint64_t tok_cap;
    JTok *ltok;         // kj_tok's records, chunk-local (kJRec per chunk, dst from the chunk's output start)
    uint32_t *cmaxd;    // the longest copy distance of a chunk
    uint32_t *ptr;
    uint32_t *pass;     // [kJPasses]: the pass changed something; [kJPasses]: token records allocated
    int32_t jc;         // compressed bytes per chunk (jchunk)
};

// Chunks of 256 bytes for batches of at most 96 KiB of input (a Reader's refill of ~64 KiB: four
// times the lanes, each walk a quarter as long -- one wave of 1 KiB chunks was the refill's critical
// path: 0.60 -> 0.51 ms; C++ NewReader over 64 KiB pieces 143 -> 200 - 208 MiB/s), 1 KiB above (at
// 122 / 244 KiB, 256-byte chunks measured 0.85 / 1.03 against 0.82 / 0.66 ms: the per-stream scan and
// fix over four times the chunks outweigh the shorter walks)
inline int32_t jchunk(uint64_t in_total) { return in_total <= (96ull << 10) ? 256 : kJC; }

enum : uint32_t { kJFBad = 1, kJFReset = 2, kJFOutFirst = 4, kJFResetLate = 8, kJFBreak = 16 };

// the stream of chunk c (binary search over cbase)
__device__ __forceinline__ uint32_t chunk_stream(const uint32_t *cbase, uint32_t count, uint32_t c) {
    uint32_t lo = 0, hi = count;  // cbase[lo] <= c < cbase[hi]
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (cbase[m] <= c) lo = m;
        else hi = m;
    }
    return lo;
}

// the 16 input bytes at p of a stream at b (bytes past the batch read 0)
__device__ __forceinline__ V16 jbytes(const uint8_t *b, int32_t p, const uint8_t *lo, const uint8_t *hi) {
    const uint8_t *y = b + p;
    return y + 16 <= hi ? ld16v(y) : ld_clamped(y, lo, hi);
}

// input bytes the token (or padding run, or meta) at p takes; -1 for a form to hand over (a walk
// that goes on steps 1 byte)
__device__ __forceinline__ int32_t jadv(const uint8_t *b, int32_t p, int32_t nb, int32_t lim32, int64_t limit, const uint8_t *lo,
                                        const uint8_t *hi, K2Tok &t, int &r) {
    r = k2_scan(jbytes(b, p, lo, hi), p, nb, lim32, limit, t);
    return r == kParseHandOver ? -1 : t.adv;
}

// The walks of kj_spec / kj_verify / kj_tok read their chunk's tokens from LDS: a block's 64 chunks are
// consecutive in the batch's input (a stream's chunks follow each other, and so do the streams), so
// the block stages the bytes from its first chunk's start to 16 past its last chunk's end with
// coalesced 16-byte loads, and every token step is then an LDS read instead of a dependent global
// load (a 61 KiB stream: the three walks 840 -> see DESIGN §4 K2j).
// kj_spec starts each chunk's speculative parse kJWarm bytes before it (positions before the chunk are
// not recorded), so that its chain has usually met the true one by the chunk's start: kj_verify's
// walks then end at their first step and kj_fix has (almost) nothing to redo
constexpr int32_t kJWarm = 256;
constexpr int32_t kJStage = 64 * kJC + kJWarm + 32;  // LDS bytes of a block's staged input
struct JStage {
    uint8_t *lds;
    uint64_t base;  // batch offset of lds[0]
    __device__ __forceinline__ V16 at(uint64_t y) const {  // 16 bytes at batch offset y (staged)
        const uint8_t *q = lds + (y - base);
        typedef uint64_t __attribute__((aligned(1))) u64u;
        return V16{*(const u64u *)q, *(const u64u *)(q + 8)};
    }
};
// stage [first chunk's start, last chunk's end + 16) of the batch (zeros past its end); every lane of
// the block calls it (a lane without a chunk passes live = false); returns the block's staging
__device__ __forceinline__ JStage kj_stage(const DecompressArgs &A, bool live, uint64_t start, uint64_t end, uint8_t *lds) {
    __shared__ uint64_t ext[2];
    if (threadIdx.x == 0) {
        ext[0] = ~0ull;
        ext[1] = 0;
    }
    __syncthreads();
    if (live) {
        atomicMin((unsigned long long *)&ext[0], (unsigned long long)start);
        atomicMax((unsigned long long *)&ext[1], (unsigned long long)end);
    }
    __syncthreads();
    const uint64_t base = ext[0], stop = ext[1] + 16, total = A.in_off[A.count];
    if (base < stop) {
        for (uint64_t o = (uint64_t)threadIdx.x * 16; base + o < stop; o += (uint64_t)blockDim.x * 16) {
            const uint64_t y = base + o;
            const V16 v = y + 16 <= total ? ld16v(A.in + y) : ld_clamped(A.in + y, A.in, A.in + total);
            typedef uint64_t __attribute__((aligned(8))) u64a;
            *(u64a *)(lds + o) = v.lo;
            *(u64a *)(lds + o + 8) = v.hi;
        }
    }
    __syncthreads();
    return JStage{lds, base};
}
// jadv on staged bytes (the token at stream position p; b0 = the stream's batch offset)
__device__ __forceinline__ int32_t jadv_s(const JStage &S, uint64_t b0, int32_t p, int32_t nb, int32_t lim32, int64_t limit, K2Tok &t,
                                          int &r, bool partial = false) {
    r = k2_scan(S.at(b0 + (uint64_t)p), p, nb, lim32, limit, t, partial);
    return r == kParseHandOver ? -1 : t.adv;
}

// The input bytes the token (or padding run, or meta) at the 16 bytes h takes, for the speculative
// walks (kj_spec, kj_verify, kj_fix): the same advance as k2_scan for every form it accepts, from 32-bit
// arithmetic on the header's first 8 bytes and no checks (a form k2_scan hands over advances by some
// amount >= 1 here; kj_tok's full parse of the true chain then hands the stream over)
__device__ __forceinline__ int32_t jadv_fast(V16 h) {
    const uint32_t w0 = (uint32_t)h.lo, w1 = (uint32_t)(h.lo >> 32);
    const uint32_t t0 = w0 & 0xff, l7 = t0 & 0x7f;
    if (t0 == 0) return h.lo ? (int32_t)(__builtin_ctzll(h.lo) >> 3) : (h.hi ? 8 + (int32_t)(__builtin_ctzll(h.hi) >> 3) : 16);
    if (t0 == 0x80) {
        const uint32_t ml = (w0 >> 8) & 7;
        return 2 + (ml == 7 ? 0 : (1 << ml));
    }
    const uint32_t ln = l7 >= 124 ? 1u << (l7 - 124 < 2 ? l7 - 124 : 2) : 0u;  // extra length bytes
    const uint32_t j = 1 + ln;
    if (!(t0 & 0x80)) {  // literal: the tag, then L bytes
        const uint32_t lx = __builtin_amdgcn_alignbyte(w1, w0, 1);  // bytes 1..4
        const uint32_t lmask = ln == 4 ? 0x3fffffffu : (1u << (8 * ln)) - 1;
        const uint32_t L = l7 >= 124 ? 124u + (l7 >= 125 ? 256u : 0u) + (l7 >= 126 ? 65536u : 0u) + (lx & lmask) : l7;
        const uint32_t adv = j + L;
        return adv > 0x7fffffffu ? 0x7fffffff : (int32_t)adv;
    }
    // copy: the tag, the long prefix (0xff) if any, the offset byte and its 1, 2 or 4 extra bytes
    const uint32_t bj = (uint32_t)(h.lo >> (8 * j)) & 0xff;  // (j <= 5)
    const uint32_t jo = j + (bj == 0xff ? 1u : 0u);
    const uint32_t o = (uint32_t)(h.lo >> (8 * jo)) & 0xff;  // (jo <= 6)
    const uint32_t on = o >= 252 ? 1u << (o - 252 < 2 ? o - 252 : 2) : 0u;
    return (int32_t)(jo + 1 + on);
}

// ---- 0: chunks per stream
__global__ __launch_bounds__(1024) void kj_init(DecompressArgs A, JWork W) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < (uint32_t)A.count; base += 1024) {
        const uint32_t s = base + t;
        uint32_t nch = 0;
        if (s < A.count) {
            const uint64_t nb = A.in_off[s + 1] - A.in_off[s];
            const uint64_t cap = A.out_off[s + 1] - A.out_off[s];
            nch = nb == 0 ? 1u : (uint32_t)((nb + W.jc - 1) / W.jc);
            JHead h{};
            // (pointers are 32-bit offsets from the batch's first output slot, rounded down to 16 bytes)
            h.state = (nb >= (1ull << 31) || cap >= (1ull << 32) - 2 || A.out_off[s + 1] - jg0(A) >= (1ull << 32) - 2) ? 1u : 0u;
            h.bsl = -1;
            h.tstop = (int32_t)(nb < (1ull << 31) ? nb : 0);
            h.tj = 0;
            h.tL = 0;
            h.nchunk = nch;
            W.head[s] = h;
        }
        part[t] = nch;
        __syncthreads();
        for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive scan
            const uint32_t v = t >= d ? part[t - d] : 0;
            __syncthreads();
            part[t] += v;
            __syncthreads();
        }
        if (s < A.count) {
            const uint32_t c0 = carry + part[t] - nch;
            W.cbase[s] = c0;
            W.head[s].chunk0 = c0;
        }
        carry += part[1023];
        __syncthreads();
    }
    if (t == 0) W.cbase[A.count] = carry;
}

// ---- 1a: speculative parse of each chunk (from kJWarm bytes before it): the positions it visits in the
// chunk, and its exit
__global__ __launch_bounds__(64) void kj_spec(DecompressArgs A, JWork W) {
    __shared__ uint32_t bm[64][kJW + 1];
    __shared__ __attribute__((aligned(16))) uint8_t stage[kJStage];
    const uint32_t lane = threadIdx.x;
    const uint32_t total = W.cbase[A.count];
    const uint32_t c = blockIdx.x * 64 + lane;
    bool live = c < total;
    const uint32_t s = live ? chunk_stream(W.cbase, (uint32_t)A.count, c) : 0;
    live = live && !W.head[s].state;
    const uint64_t b0 = A.in_off[s];
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int32_t c0 = (int32_t)(c - W.cbase[s]) * W.jc, ce = c0 + W.jc < nb ? c0 + W.jc : nb;
    const int32_t w0 = c0 > kJWarm ? c0 - kJWarm : 0;
    const JStage S = kj_stage(A, live, b0 + (uint64_t)w0, b0 + (uint64_t)ce, stage);
    if (!live) return;
    for (int k = 0; k < kJW; k++) bm[lane][k] = 0;
    int32_t p = w0;
    while (p < c0) p += jadv_fast(S.at(b0 + (uint64_t)p));  // (the warm-up: nothing recorded)
    while (p < ce) {
        bm[lane][(p - c0) >> 5] |= 1u << ((p - c0) & 31);
        p += jadv_fast(S.at(b0 + (uint64_t)p));
    }
    uint32_t *g = W.bits + (uint64_t)c * kJW;
    for (int k = 0; k < kJW; k++) g[k] = bm[lane][k];
    W.sexit[c] = (uint32_t)p;
}

// ---- 1b: the true entry of every chunk.  Chunk c's entry is its predecessor's speculative exit when
// the predecessor's speculative chain merged with the true chain inside it (a wrong start meets the
// true chain within ~110 bytes on the logs, 99 % within 1 KiB); every chunk checks that at once
// (kj_verify: thread per chunk, walking the true chain from that entry until a position its own
// speculative parse visited -- its speculative exit is then its true exit -- or its end), and a wave
// per stream then redoes, in order, only the chunks whose predecessor did not merge (kj_fix).
// texit[c]: chunk c's true exit given that entry; entry[c]: the entry the check assumed
__device__ __forceinline__ int32_t kj_walk_true(const JWork &W, uint32_t cg, const uint8_t *b, int32_t a, int32_t cs, int32_t ce,
                                                const uint8_t *lo, const uint8_t *hi) {
    const uint32_t *g = W.bits + (uint64_t)cg * kJW;
    int32_t q = a;
    while (q < ce) {
        if ((g[(q - cs) >> 5] >> ((q - cs) & 31)) & 1u) return (int32_t)W.sexit[cg];  // merged: its exit is the chain's
        q += jadv_fast(jbytes(b, q, lo, hi));
    }
    return q;
}

__global__ __launch_bounds__(64) void kj_verify(DecompressArgs A, JWork W) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kJStage];
    const uint32_t total = W.cbase[A.count];
    const uint32_t c = blockIdx.x * 64 + threadIdx.x;
    bool live = c < total;
    const uint32_t s = live ? chunk_stream(W.cbase, (uint32_t)A.count, c) : 0;
    live = live && !W.head[s].state;
    const uint64_t b0 = A.in_off[s];
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint32_t k = c - W.cbase[s];
    const int32_t c0 = (int32_t)k * W.jc, ce = c0 + W.jc < nb ? c0 + W.jc : nb;
    const JStage S = kj_stage(A, live, b0 + (uint64_t)c0, b0 + (uint64_t)ce, stage);
    if (!live) return;
    const int32_t a = k == 0 ? 0 : (int32_t)W.sexit[c - 1];
    int32_t x;
    if (k == 0) {
        x = (int32_t)W.sexit[c];  // (chunk 0's speculation starts at the stream's start: it is the true chain)
    } else if (a >= ce) {
        x = a;  // an entry past the chunk (inside a long token) passes through
    } else {
        const uint32_t *g = W.bits + (uint64_t)c * kJW;
        int32_t q = a < c0 ? c0 : a;  // (a < c0 cannot happen: a speculative exit is >= its chunk's end)
        x = -1;
        while (q < ce) {
            if ((g[(q - c0) >> 5] >> ((q - c0) & 31)) & 1u) {
                x = (int32_t)W.sexit[c];
                break;
            }
            q += jadv_fast(S.at(b0 + (uint64_t)q));
        }
        if (x < 0) x = q;
    }
    W.entry[c] = (uint32_t)a;
    W.cnt[c] = (uint32_t)x;  // (the true exit; kj_tok overwrites cnt with the token count)
}

__global__ __launch_bounds__(64) void kj_fix(DecompressArgs A, JWork W) {
    const uint32_t s = blockIdx.x, lane = threadIdx.x;
    JHead &H = W.head[s];
    if (H.state) return;
    const uint8_t *b = A.in + A.in_off[s], *lo = A.in, *hi = A.in + A.in_off[A.count];
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint32_t c00 = H.chunk0, nch = H.nchunk;
    uint32_t *texit = W.cnt;
    // chunks [0, k) are right; chunk j's entry is right iff its predecessor's true exit is the
    // speculative exit it assumed.  The true exit of the chunk fixed last is kept in a register
    // (fx_at, fx_val): this kernel's own stores are not read back.
    uint32_t k = 1, fx_at = ~0u;
    int32_t fx_val = 0;
    while (k < nch) {
        const uint32_t j = k + lane;
        bool bad = false;
        if (j < nch) {
            const uint32_t tx = j - 1 == fx_at ? (uint32_t)fx_val : texit[c00 + j - 1];
            bad = tx != W.sexit[c00 + j - 1];
        }
        const uint64_t m = __ballot(bad);
        if (m == 0) {
            k += 64;
            continue;
        }
        const uint32_t jf = k + (uint32_t)__builtin_ctzll(m);  // the first chunk entered wrongly
        const int32_t e = jf - 1 == fx_at ? fx_val : (int32_t)texit[c00 + jf - 1];  // its true entry
        // an entry past chunk jf (inside a long token): no token starts in the chunks it covers
        uint32_t kw = jf;
        if (e >= nb || e >= (int32_t)(jf + 1) * W.jc) {
            kw = e >= nb ? nch : (uint32_t)(e / W.jc);
            for (uint32_t x = jf + lane; x < kw; x += 64) {
                W.entry[c00 + x] = (uint32_t)e;
                texit[c00 + x] = (uint32_t)e;
            }
            if (kw >= nch) {
                fx_at = nch - 1;
                fx_val = e;
                break;
            }
        }
        // chunk kw holds e: the true chain from there (one lane; rare)
        int32_t x = 0;
        if (lane == 0) {
            const int32_t cs = (int32_t)kw * W.jc, ce = cs + W.jc < nb ? cs + W.jc : nb;
            x = kj_walk_true(W, c00 + kw, b, e, cs, ce, lo, hi);
            W.entry[c00 + kw] = (uint32_t)e;
            texit[c00 + kw] = (uint32_t)x;
        }
        fx_at = kw;
        fx_val = __shfl(x, 0);
        k = kw + 1;
    }
    // the chain must end exactly at the stream's end (else the last token runs past the input; a
    // Reader's read-ahead, c_on, stops before that token: kj_tok finds it)
    const int32_t last = nch - 1 == fx_at ? fx_val : (int32_t)texit[c00 + nch - 1];
    if (lane == 0 && (A.c_on ? last < nb : last != nb)) H.state = 1;
}

// ---- 2a: the true chain of each chunk, parsed once: tokens, output bytes, forms and metas, a record
// per token (chunk-local: output positions from the chunk's start; kj_place moves them into the
// stream's array once the chunks' positions are known), the longest distance, Break positions
__global__ __launch_bounds__(64) void kj_tok(DecompressArgs A, JWork W) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kJStage];
    const uint32_t total = W.cbase[A.count];
    const uint32_t c = blockIdx.x * 64 + threadIdx.x;
    bool live = c < total;
    const uint32_t s = live ? chunk_stream(W.cbase, (uint32_t)A.count, c) : 0;
    live = live && !W.head[s].state;
    const uint64_t b0 = A.in_off[s];
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int32_t c0 = (int32_t)(c - W.cbase[s]) * W.jc, ce = c0 + W.jc < nb ? c0 + W.jc : nb;
    const JStage S = kj_stage(A, live, b0 + (uint64_t)c0, b0 + (uint64_t)ce, stage);
    if (!live) return;
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;
    int32_t p = (int32_t)W.entry[c];
    uint32_t n = 0, fl = 0, maxd = 0;
    uint64_t out = 0;
    const bool partial = A.c_on != 0;
    JTok *rec = W.ltok + (uint64_t)c * kJRec;
    while (p < ce) {
        K2Tok t;
        int r;
        const int32_t ad = jadv_s(S, b0, p, nb, lim32, limit, t, r, partial);
        if (ad < 0 || (r == kParseToken && n >= kJRec)) {
            fl |= kJFBad;
            break;
        }
        if (r == kScanTail) {  // the chain stops here (one chunk of the stream meets it)
            JHead &H = W.head[s];
            H.tstop = p;
            H.tj = t.adv ? t.j : 0;
            H.tL = t.adv ? t.L : 0;
            break;
        }
        if (r == kScanReset) {
            fl |= (out ? kJFResetLate : 0) | kJFReset | (n == 0 ? 0 : kJFOutFirst);
            fl = (fl & 0xffu) | (t.marg << 8);
        } else if (r == kParseToken) {
            rec[n++] = JTok{(uint32_t)out, (uint32_t)t.L, t.cp ? (kJCopy | t.D) : 0u, (uint32_t)(p + t.j)};
            maxd = t.cp && t.D > maxd ? t.D : maxd;
            out += (uint64_t)t.L;
        } else if (r == kParseSkip && A.breaks) {  // (one-stream batches) a Break: (chunk, local position)
            const V16 h = S.at(b0 + (uint64_t)p);
            if (((uint32_t)h.lo & 0xffffu) == (0x80u | ((kMetaBreak | kMetaLen0) << 8))) {
                const uint64_t at = atomicAdd((unsigned long long *)A.breaks, 1ull);
                if (at < A.breaks_cap) A.breaks[1 + at] = ((uint64_t)c << 32) | (out & 0xffffffffull);
            }
        }
        p += ad;
    }
    W.cnt[c] = n;
    W.cout[c] = out;
    W.cflag[c] = fl;
    W.cmaxd[c] = maxd;
}

// ---- 2b: token and output positions of the chunks; the stream's checks (wave per stream)
__global__ __launch_bounds__(64) void kj_scan(DecompressArgs A, JWork W, uint64_t *tok_alloc) {
    const uint32_t s = blockIdx.x, lane = threadIdx.x;
    JHead &H = W.head[s];
    if (H.state) return;
    const uint32_t c00 = H.chunk0, nch = H.nchunk;
    uint64_t tcarry = 0, ocarry = 0;
    int32_t bsl = A.c_on ? A.c_bsl : -1;  // (a Reader's read-ahead: the window its stream has set)
    bool bad = false;
    uint32_t maxd = 0;
    for (uint32_t k = 0; k < nch; k += 64) {
        const uint32_t j = k + lane;
        const bool mine = j < nch;
        const uint64_t n = mine ? W.cnt[c00 + j] : 0, o = mine ? W.cout[c00 + j] : 0;
        const uint32_t fl = mine ? W.cflag[c00 + j] : 0;
        uint32_t md = mine ? W.cmaxd[c00 + j] : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) md = max(md, (uint32_t)__shfl_xor((int)md, d, 64));
        maxd = max(maxd, md);
        uint64_t in = n, io = o;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t vn = __shfl_up(in, d, 64), vo = __shfl_up(io, d, 64);
            if ((int)lane >= d) {
                in += vn;
                io += vo;
            }
        }
        const uint64_t obefore = ocarry + io - o;
        if (mine) {
            W.ctbase[c00 + j] = tcarry + in - n;
            W.cobase[c00 + j] = obefore;
        }
        // a MetaReset only before any output (and the window it sets is the last such one)
        const bool rbad = mine && (fl & kJFReset) && (obefore != 0 || (fl & (kJFOutFirst | kJFResetLate)) || (A.c_on && A.c_pos0 != 0));
        if (__ballot(rbad || (mine && (fl & kJFBad)))) bad = true;
        const uint64_t rm = __ballot(mine && (fl & kJFReset));
        if (rm) bsl = (int32_t)((__shfl(fl, 63 - __builtin_clzll(rm)) >> 8) & 0xff);
        tcarry = __shfl(tcarry + in, 63);
        ocarry = __shfl(ocarry + io, 63);
    }
    if (lane != 0) return;
    const uint64_t cap = A.out_off[s + 1] - A.out_off[s];
    // a literal at the input's end (c_on) whose body runs past it: the bytes there are are output too
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint64_t tail = A.c_on && H.tj > 0 ? (uint64_t)min((int64_t)H.tL, (int64_t)(nb - H.tstop - H.tj)) : 0;
    // "missed meta": a token (or a literal's header) before the window is set
    if (!bad && (ocarry > 0 || (A.c_on && H.tj > 0)) && bsl < 0) bad = true;
    // ErrOverflow (reader.go:256-258): a distance past the window -- the exact decoder reports it
    if (!bad && bsl >= 0 && bsl < 30 && maxd > (1u << bsl)) bad = true;
    if (!bad && ocarry + tail > cap) {
        bad = true;
        if (A.end_state) A.end_state[0] = -2;  // (a caller that sizes its slot grows it and retries)
    }
    if (!bad) {
        const uint64_t t0 = atomicAdd((unsigned long long *)tok_alloc, (unsigned long long)tcarry);
        if (t0 + tcarry > W.tok_cap) bad = true;
        H.tok0 = t0;
    }
    H.bsl = bsl;
    H.total = ocarry;
    H.ntok = tcarry;
    if (bad) H.state = 1;
}

// ---- 2c: the chunks' records into the stream's array, positions from the stream's start (block per chunk)
__global__ __launch_bounds__(64) void kj_place(DecompressArgs A, JWork W) {
    const uint32_t c = blockIdx.x;
    if (c >= W.cbase[A.count]) return;
    const uint32_t s = chunk_stream(W.cbase, (uint32_t)A.count, c);
    const JHead &H = W.head[s];
    if (H.state) return;
    const JTok *src = W.ltok + (uint64_t)c * kJRec;
    JTok *dst = W.tok + H.tok0 + W.ctbase[c];
    const uint32_t n = W.cnt[c], ob = (uint32_t)W.cobase[c];
    for (uint32_t k = threadIdx.x; k < n; k += 64) {
        JTok t = src[k];
        t.dst += ob;
        dst[k] = t;
    }
}

// ---- 3: literal and zero bytes, and a pointer for every copied byte (thread per 16 output bytes)
// output bytes [q, q + n) of stream s (n <= 16, inside its output): bytes into by, pointers into pt.
// Pointers and the ptr array count from g0 = out_off[0] rounded down to 16 bytes: a batch may be a view
// into a larger one (absolute offsets), whose bytes before out_off[0] are never touched.
__device__ __forceinline__ void kj_piece(const DecompressArgs &A, const JWork &W, const JHead &H, uint32_t s, uint64_t q, uint32_t n,
                                         uint64_t g0, uint32_t *by, uint32_t *pt) {
    const uint64_t base = A.out_off[s];
    const uint32_t hb = A.c_on ? (uint32_t)A.c_hist : 0u;  // history bytes before the output (a copy may read them)
    const uint32_t p0 = (uint32_t)(q - base);
    // the token holding p0: the last record with dst <= p0; the next ones by walking on
    const JTok *tk = W.tok + H.tok0;
    uint64_t a = 0, z = H.ntok;
    while (z - a > 1) {
        const uint64_t m = (a + z) >> 1;
        if (tk[m].dst <= p0) a = m;
        else z = m;
    }
    JTok t = tk[a];
    uint32_t nxt = a + 1 < H.ntok ? tk[a + 1].dst : 0xffffffffu;
    const uint8_t *in = A.in + A.in_off[s];
    if (n == 16 && p0 + 16 <= t.dst + t.L) {  // the 16 bytes inside one token (long literals, runs, zeros)
        const uint32_t x = (uint32_t)(base + p0 - g0);
        if (t.kd == 0) {
            const uint8_t *y = in + t.src + (p0 - t.dst);
            const V16 v = y + 16 <= A.in + A.in_off[A.count] ? ld16v(y) : ld_clamped(y, A.in, A.in + A.in_off[A.count]);
            by[0] = (uint32_t)v.lo, by[1] = (uint32_t)(v.lo >> 32), by[2] = (uint32_t)v.hi, by[3] = (uint32_t)(v.hi >> 32);
            for (uint32_t k = 0; k < 16; k++) pt[k] = x + k;
        } else if (t.kd == kJCopy) {
            for (uint32_t k = 0; k < 16; k++) pt[k] = x + k;
        } else {
            const uint32_t D = t.kd & ~kJCopy;
            for (uint32_t k = 0; k < 16; k++) pt[k] = p0 + k + hb >= D ? x + k - D : kJZero;
        }
        return;
    }
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t p = p0 + k;
        while (p >= nxt) {
            a++;
            t = tk[a];
            nxt = a + 1 < H.ntok ? tk[a + 1].dst : 0xffffffffu;
        }
        const uint32_t x = (uint32_t)(base + p - g0);
        uint32_t v = 0;
        if (t.kd == 0) {  // literal
            v = in[t.src + (p - t.dst)];
            pt[k] = x;
        } else if (t.kd == kJCopy) {  // zero region
            pt[k] = x;
        } else {
            const uint32_t D = t.kd & ~kJCopy;
            pt[k] = p + hb >= D ? x - D : kJZero;
        }
        by[k >> 2] |= v << (8 * (k & 3));
    }
}

__global__ __launch_bounds__(256) void kj_expand(DecompressArgs A, JWork W) {
    const uint64_t ob = A.out_off[0], g0 = jg0(A), end = A.out_off[A.count];
    const uint64_t hst = A.c_on ? ob - A.c_hist : ob;  // (c_on) the history [hst, ob): final bytes, pointing at themselves
    for (uint64_t g = g0 + ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; g < end; g += (uint64_t)gridDim.x * blockDim.x * 16) {
        // the stream of the piece's first byte of the batch (binary search over the slots)
        const uint64_t x0 = g > ob ? g : ob;
        uint32_t s = 0, hs = (uint32_t)A.count;
        while (hs - s > 1) {
            const uint32_t m = (s + hs) >> 1;
            if (A.out_off[m] <= x0) s = m;
            else hs = m;
        }
        const uint64_t ge = g + 16 < end ? g + 16 : end;
        const JHead H = W.head[s];
        if (!H.state && A.out_off[s] <= g && A.out_off[s] + H.total >= g + 16 && ge == g + 16) {
            // the common case: the 16 bytes all in stream s's output, one store of each kind
            uint32_t by[4] = {0, 0, 0, 0}, pt[16];
            kj_piece(A, W, H, s, g, 16, g0, by, pt);
            *(uint4 *)(A.out + g) = make_uint4(by[0], by[1], by[2], by[3]);  // (copied bytes: kj_gather)
            uint32_t *pp = W.ptr + (g - g0);
#pragma unroll
            for (int q = 0; q < 4; q++) *(uint4 *)(pp + 4 * q) = make_uint4(pt[4 * q], pt[4 * q + 1], pt[4 * q + 2], pt[4 * q + 3]);
            continue;
        }
        // a piece at a slot's end (or before the batch's first slot): each stream's output bytes in it,
        // byte by byte
        for (uint64_t y = g > hst ? g : hst; y < ob && y < ge; y++) W.ptr[y - g0] = (uint32_t)(y - g0);
        for (uint64_t x = x0; x < ge;) {
            while (s + 1 < (uint32_t)A.count && A.out_off[s + 1] <= x) s++;
            const JHead Hs = W.head[s];
            const uint64_t ob2 = A.out_off[s] + Hs.total, se = A.out_off[s + 1] < ge ? A.out_off[s + 1] : ge;
            if (!Hs.state && x < ob2) {
                const uint32_t n = (uint32_t)((ob2 < se ? ob2 : se) - x);
                uint32_t by[4] = {0, 0, 0, 0}, pt[16];
                kj_piece(A, W, Hs, s, x, n, g0, by, pt);
                for (uint32_t k = 0; k < n; k++) {
                    A.out[x + k] = (uint8_t)(by[k >> 2] >> (8 * (k & 3)));
                    W.ptr[x - g0 + k] = pt[k];
                }
            }
            x = se;
        }
    }
}

// ---- 4: one pointer-jumping pass (returns at once when the pass before changed nothing)
__global__ __launch_bounds__(256) void kj_jump(DecompressArgs A, JWork W, int pass) {
    if (pass > 0 && W.pass[pass - 1] == 0) return;
    const uint64_t end = A.out_off[A.count] - jg0(A);  // (ptr counts from g0)
    bool changed = false;
    for (uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; g < end; g += (uint64_t)gridDim.x * blockDim.x * 4) {
        uint4 v = g + 4 <= end ? *(const uint4 *)(W.ptr + g) : make_uint4(kJGap, kJGap, kJGap, kJGap);
        if (g + 4 > end)
            for (uint64_t k = g; k < end; k++) (&v.x)[k - g] = W.ptr[k];
        uint32_t *e = &v.x;
        // the four gathers issued together (a pointer to itself or a marker is final)
        uint32_t r[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t q = e[k];
            r[k] = q >= kJZero || q == (uint32_t)(g + k) ? q : W.ptr[q];
        }
        bool any = false;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            any |= r[k] != e[k];
            e[k] = r[k];
        }
        if (any) {
            changed = true;
            if (g + 4 <= end) *(uint4 *)(W.ptr + g) = v;
            else
                for (uint64_t k = g; k < end; k++) W.ptr[k] = e[k - g];
        }
    }
    if (__ballot(changed) != 0 && (threadIdx.x & 63) == 0) W.pass[pass] = 1;
}

// ---- 5a: every copied byte from its resolved source
__global__ __launch_bounds__(256) void kj_gather(DecompressArgs A, JWork W) {
    const uint64_t g0 = jg0(A), end = A.out_off[A.count] - g0;
    uint8_t *o = A.out + g0;
    for (uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; g < end; g += (uint64_t)gridDim.x * blockDim.x * 4) {
        for (uint64_t x = g; x < g + 4 && x < end; x++) {
            const uint32_t q = W.ptr[x];
            if (q == kJGap || q == (uint32_t)x) continue;
            o[x] = q == kJZero ? (uint8_t)0 : o[q];
        }
    }
}

// ---- 5b: results, or the stream to the exact decoder; a one-stream batch's Break positions from
// (chunk, local position) to the stream's output positions
__global__ __launch_bounds__(256) void kj_final(DecompressArgs A, JWork W) {
    if (A.breaks && A.count == 1 && blockIdx.x == 0 && !W.head[0].state) {
        const uint64_t nbrk = A.breaks[0] < A.breaks_cap ? A.breaks[0] : A.breaks_cap;
        for (uint64_t k = threadIdx.x; k < nbrk; k += blockDim.x) {
            const uint64_t v = A.breaks[1 + k];
            A.breaks[1 + k] = W.cobase[v >> 32] + (v & 0xffffffffull);
        }
    }
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < A.count; s += (uint64_t)gridDim.x * blockDim.x) {
        const JHead H = W.head[s];
        if (H.state) {
            const uint32_t at = atomicAdd(&A.slow[0], 1u);
            A.slow[1 + at] = (uint32_t)s;
            continue;
        }
        A.out_size[s] = H.total;
        if (A.status) A.status[s] = EZ_OK;
        if (A.end_state) {  // (one MetaReset, before any output: r.pos is the output since the start)
            A.end_state[0] = H.bsl < 0 ? 0 : (int64_t)1 << H.bsl;
            A.end_state[1] = (int64_t)H.total;
            if (A.c_on) {
                A.end_state[2] = H.tstop;
                A.end_state[3] = H.tj;
                A.end_state[4] = H.tL;
            }
        }
    }
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// the workspace layout of a batch (in_total / out_total: the end offsets in_off[count], out_off[count])
struct JLayout {
    uint64_t chunks, tok_cap;
    size_t o_head, o_cbase, o_entry, o_sexit, o_bits, o_cnt, o_cout, o_cflag, o_ctb, o_cob, o_tok, o_ltok, o_maxd, o_ptr, o_pass, total;
    JLayout(uint64_t count, uint64_t in_total, uint64_t out_total) {
        chunks = in_total / (uint64_t)jchunk(in_total) + 2 * count + 2;
        tok_cap = in_total / 2 + chunks + 16;  // (a token takes >= 2 input bytes; one may start in each chunk's last byte)
        size_t off = 0;
        auto take = [&](size_t n) {
            const size_t o = off;
            off += al256(n);
            return o;
        };
        o_head = take(sizeof(JHead) * count), o_cbase = take(4 * (count + 1)), o_entry = take(4 * chunks), o_sexit = take(4 * chunks),
        o_bits = take(4 * kJW * chunks), o_cnt = take(4 * chunks), o_cout = take(8 * chunks), o_cflag = take(4 * chunks),
        o_ctb = take(8 * chunks), o_cob = take(8 * chunks), o_tok = take(sizeof(JTok) * tok_cap),
        o_ltok = take(sizeof(JTok) * kJRec * chunks), o_maxd = take(4 * chunks), o_ptr = take(4 * out_total + 16),
        o_pass = take(8 * (kJPasses + 2));
        total = off;
    }
};
}  // namespace

// K2j's workspaces per (device, HIP stream) (ez_cache.h)
DevCache &jump_cache() {
    static DevCache *c = new DevCache();  // (never destroyed: no hipFree after the runtime's teardown)
    return *c;
}

// Streams K2j takes: a batch of at most 1,024 streams (slots below 4 GiB in all)
bool jump_applies(const DecompressArgs &a) { return a.count >= 1 && a.count <= 1024; }

uint64_t jump_workspace_bytes(uint64_t count, uint64_t in_total, uint64_t out_total) {
    return JLayout(count, in_total, out_total).total;
}

hipError_t batch_extents(const DecompressArgs &a, hipStream_t st, uint64_t *in_bytes, uint64_t *out_bytes) {
    if (a.in_bytes || a.out_bytes) {
        *in_bytes = a.in_bytes;
        *out_bytes = a.out_bytes;
        return hipSuccess;
    }
    uint64_t ext[4] = {0, 0, 0, 0};  // (the offsets may be a view into a larger batch's: absolute)
    hipError_t e;
    if ((e = hipMemcpyAsync(&ext[0], a.in_off, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&ext[1], a.in_off + a.count, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&ext[2], a.out_off, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&ext[3], a.out_off + a.count, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    *in_bytes = ext[1] - ext[0];
    *out_bytes = ext[3] - ext[2];
    return hipSuccess;
}

hipError_t launch_decompress_jump(const DecompressArgs &a, hipStream_t st) {
    // the batch's input and output extents (the caller's hints, else one read back): the workspace is
    // sized from them; the ptr array covers out_off[0] rounded down to 16 bytes .. out_off[count]
    uint64_t in_total = 0, out_bytes = 0;
    hipError_t e = batch_extents(a, st, &in_total, &out_bytes);
    if (e != hipSuccess) return e;
    const uint64_t out_total = out_bytes + (a.c_on ? a.c_hist : 0) + 16;  // (+ the history a continuation reads)
    const JLayout Y(a.count, in_total, out_total);
    const uint64_t chunks = Y.chunks, tok_cap = Y.tok_cap;
    const size_t o_head = Y.o_head, o_cbase = Y.o_cbase, o_entry = Y.o_entry, o_sexit = Y.o_sexit, o_bits = Y.o_bits, o_cnt = Y.o_cnt,
                 o_cout = Y.o_cout, o_cflag = Y.o_cflag, o_ctb = Y.o_ctb, o_cob = Y.o_cob, o_tok = Y.o_tok, o_ptr = Y.o_ptr,
                 o_pass = Y.o_pass;
    // the caller's workspace when it gives one large enough, else this (device, stream)'s (its lease
    // is held through the launches: another host thread growing it meanwhile would free it under them)
    CacheLease lease;
    uint8_t *w = (uint8_t *)a.jws;
    if (!w || a.jws_cap < Y.total) {
        int dev = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        lease = jump_cache().acquire(dev, (void *)st);
        if (!lease->ensure(Y.total)) return hipErrorOutOfMemory;  // (the caller decodes the batch on K2t)
        w = (uint8_t *)lease->p;
    }
    JWork W{};
    W.head = (JHead *)(w + o_head);
    W.cbase = (uint32_t *)(w + o_cbase);
    W.entry = (uint32_t *)(w + o_entry);
    W.sexit = (uint32_t *)(w + o_sexit);
    W.bits = (uint32_t *)(w + o_bits);
    W.cnt = (uint32_t *)(w + o_cnt);
    W.cout = (uint64_t *)(w + o_cout);
    W.cflag = (uint32_t *)(w + o_cflag);
    W.ctbase = (uint64_t *)(w + o_ctb);
    W.cobase = (uint64_t *)(w + o_cob);
    W.tok = (JTok *)(w + o_tok);
    W.tok_cap = tok_cap;
    W.ltok = (JTok *)(w + Y.o_ltok);
    W.cmaxd = (uint32_t *)(w + Y.o_maxd);
    W.ptr = (uint32_t *)(w + o_ptr);
    W.pass = (uint32_t *)(w + o_pass);
    W.jc = jchunk(in_total);
    uint64_t *tok_alloc = (uint64_t *)(W.pass + kJPasses + 2);
    if ((e = hipMemsetAsync(W.pass, 0, 8 * (kJPasses + 2), st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(W.ptr, 0xff, 4 * out_total + 16, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(kj_init, dim3(1), dim3(1024), 0, st, a, W);
    const unsigned cgrid = (unsigned)((chunks + 63) / 64);
    hipLaunchKernelGGL(kj_spec, dim3(cgrid), dim3(64), 0, st, a, W);
    hipLaunchKernelGGL(kj_verify, dim3(cgrid), dim3(64), 0, st, a, W);
    hipLaunchKernelGGL(kj_fix, dim3((unsigned)a.count), dim3(64), 0, st, a, W);
    hipLaunchKernelGGL(kj_tok, dim3(cgrid), dim3(64), 0, st, a, W);
    hipLaunchKernelGGL(kj_scan, dim3((unsigned)a.count), dim3(64), 0, st, a, W, tok_alloc);
    hipLaunchKernelGGL(kj_place, dim3((unsigned)chunks), dim3(64), 0, st, a, W);
    const uint64_t pieces = (out_total + 15) / 16;  // (out_total: the batch's output and the alignment slack)
    const unsigned egrid = (unsigned)(pieces / 256 + 1 < 8192 ? pieces / 256 + 1 : 8192);
    hipLaunchKernelGGL(kj_expand, dim3(egrid), dim3(256), 0, st, a, W);
    const uint64_t quads = (out_total + 3) / 4;
    const unsigned jgrid = (unsigned)(quads / 256 + 1 < 8192 ? quads / 256 + 1 : 8192);
    // every pass at least halves the longest pointer chain, and a chain is shorter than the output:
    // ceil(log2(output)) + 1 passes finish it (the ones after it return at once)
    int passes = 1;
    while (passes < kJPasses && ((uint64_t)1 << (passes - 1)) < out_total) passes++;
    for (int k = 0; k < passes; k++) hipLaunchKernelGGL(kj_jump, dim3(jgrid), dim3(256), 0, st, a, W, k);
    hipLaunchKernelGGL(kj_gather, dim3(jgrid), dim3(256), 0, st, a, W);
    hipLaunchKernelGGL(kj_final, dim3((unsigned)((a.count + 255) / 256)), dim3(256), 0, st, a, W);
    return hipGetLastError();
}

}  // namespace ez
