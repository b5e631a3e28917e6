// ez_decompress_jump.hip — K2j: the decode of a few long streams with the whole chip.
//
// Reader.read (reader.go:143-216) is a chain twice over: every token starts where the previous one
// ends (readTag :218-270), and every copied byte reads output written before it (:173-201).  K2t
// runs both chains on one wave per stream, which leaves a batch of a few long streams (a Reader
// handle's one stream, C4's 64 buckets, 1 MiB streams) to a handful of waves on a 1,024-SIMD chip.
// K2j cuts both chains into data-parallel steps:
//
//  1. token starts (kj_spec, kj_prop): the compressed stream is cut into 2 KiB chunks; a lane per
//     chunk parses speculatively from the chunk's first byte and records the positions it visits
//     (a bitmap) and where it leaves the chunk.  A wrong start parses garbage, but its chain meets
//     the true one within a few tokens (median ~110 bytes on the log streams; 99 % within 1 KiB),
//     after which both are the same chain.  One wave per stream then carries the true entry
//     through the chunks 64 at a time: lane j takes chunk j's entry to be chunk j-1's speculative
//     exit and walks the true chain from it until it meets a recorded position (the chunks agree)
//     or leaves the chunk (the first lane that does ends the step with the true exit it walked);
//     an entry past a chunk (inside a long token) skips to the chunk it lies in.
//  2. tokens (kj_count, kj_scan, kj_emit): a lane per chunk walks the true chain from its entry,
//     counts tokens and output bytes, and checks every form (k2_scan, ez_k2_parse.h); a wave per
//     stream scans the chunks' counts into token and output positions and validates the stream
//     as K2t does (one MetaReset before any output, the window set before the first token, every
//     distance within the window, the output within the slot); the lanes then write one record
//     per token (output position, length, distance or input position).
//  3. bytes (kj_expand): a thread per 16 output bytes finds its tokens (a binary search over the
//     stream's records), writes literal bytes and zero regions, and for every copied byte p a
//     pointer ptr[p] = p - D (a marker for bytes before the stream start: the fresh window's zeros,
//     SURVEY A.12); literal and zero bytes point at themselves.
//  4. copies (kj_jump): pointer jumping, ptr[p] = ptr[ptr[p]] over all bytes, until every pointer
//     names a literal byte, a zero byte or the zero marker: ceil(log2(chain depth)) passes, each a
//     sequential read and a gather that stays mostly local (copy distances are short).  Passes
//     after the one that changed nothing return at once (the launcher queues a fixed number, so
//     nothing waits on the host).
//  5. kj_gather writes every copied byte from its resolved source; kj_final reports each stream
//     (out_size, status, a Reader's end state) or hands it to the exact decoder.
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

constexpr int32_t kJC = 2048;                        // compressed bytes per chunk
constexpr int32_t kJW = kJC / 32;                    // bitmap words per chunk
constexpr uint32_t kJGap = 0xffffffffu;              // ptr: not a byte of any stream's output
constexpr uint32_t kJZero = 0xfffffffeu;             // ptr: a zero byte of the history before the stream
constexpr uint32_t kJCopy = 0x80000000u;             // JTok.kd: a copy (distance in the low bits; 0: zero region)
constexpr int kJPasses = 34;                         // pointer-jumping passes queued (chains up to 2^34)

struct JHead {
    uint32_t chunk0, nchunk;  // the stream's chunks
    uint32_t state;           // 0: K2j decodes it; 1: handed over
    int32_t bsl;              // log2 of the window (MetaReset)
    uint64_t total;           // output bytes
    uint64_t ntok;            // token records
    uint64_t tok0;            // its first record
};

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
    uint32_t *ptr;
    uint32_t *pass;     // [kJPasses]: the pass changed something; [kJPasses]: token records allocated
};

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
            nch = nb == 0 ? 1u : (uint32_t)((nb + kJC - 1) / kJC);
            JHead h{};
            // (pointers are 32-bit offsets from the batch's first output slot, rounded down to 16 bytes)
            h.state = (nb >= (1ull << 31) || cap >= (1ull << 32) - 2 || A.out_off[s + 1] - (A.out_off[0] & ~15ull) >= (1ull << 32) - 2) ? 1u : 0u;
            h.bsl = -1;
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

// ---- 1a: speculative parse of each chunk from its first byte: the positions visited, the exit
__global__ __launch_bounds__(64) void kj_spec(DecompressArgs A, JWork W) {
    __shared__ uint32_t bm[64][kJW + 1];
    const uint32_t lane = threadIdx.x;
    const uint32_t total = W.cbase[A.count];
    const uint32_t c = blockIdx.x * 64 + lane;
    if (c >= total) return;
    const uint32_t s = chunk_stream(W.cbase, (uint32_t)A.count, c);
    if (W.head[s].state) return;
    const uint8_t *b = A.in + A.in_off[s], *lo = A.in, *hi = A.in + A.in_off[A.count];
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;
    const int32_t c0 = (int32_t)(c - W.cbase[s]) * kJC, ce = c0 + kJC < nb ? c0 + kJC : nb;
    for (int k = 0; k < kJW; k++) bm[lane][k] = 0;
    int32_t p = c0;
    while (p < ce) {
        bm[lane][(p - c0) >> 5] |= 1u << ((p - c0) & 31);
        K2Tok t;
        int r;
        const int32_t a = jadv(b, p, nb, lim32, limit, lo, hi, t, r);
        p += a > 0 ? a : 1;
    }
    uint32_t *g = W.bits + (uint64_t)c * kJW;
    for (int k = 0; k < kJW; k++) g[k] = bm[lane][k];
    W.sexit[c] = (uint32_t)p;
}

// ---- 1b: the true entry of every chunk, 64 chunks per step (wave per stream)
__global__ __launch_bounds__(64) void kj_prop(DecompressArgs A, JWork W) {
    const uint32_t s = blockIdx.x, lane = threadIdx.x;
    JHead &H = W.head[s];
    if (H.state) return;
    const uint8_t *b = A.in + A.in_off[s], *lo = A.in, *hi = A.in + A.in_off[A.count];
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;
    const uint32_t c00 = H.chunk0, nch = H.nchunk;
    uint32_t k = 0;     // the first chunk whose entry is not known yet
    int32_t e = 0;      // its entry (the true chain's first position at or after its first byte)
    bool bad = false;
    while (k < nch) {
        const uint32_t j = k + lane;
        const bool mine = j < nch;
        const int32_t cs = (int32_t)j * kJC, ce = cs + kJC < nb ? cs + kJC : nb;
        int32_t a = lane == 0 ? e : (mine ? (int32_t)W.sexit[c00 + j - 1] : 0);
        // walk the true chain from a until a position the speculative parse visited, or the chunk's end
        int32_t q = a;
        bool lbad = false, synced = false;
        if (mine && a < ce && a >= cs) {
            const uint32_t *g = W.bits + (uint64_t)(c00 + j) * kJW;
            while (q < ce) {
                if ((g[(q - cs) >> 5] >> ((q - cs) & 31)) & 1u) {
                    synced = true;
                    break;
                }
                K2Tok t;
                int r;
                const int32_t ad = jadv(b, q, nb, lim32, limit, lo, hi, t, r);
                lbad |= ad < 0;
                q += ad > 0 ? ad : 1;
            }
        }
        // a chunk whose entry lies past it (inside a long token), or one the chains do not meet in,
        // ends the step: its exit is the position the walk reached
        const uint64_t stop = __ballot(mine && !synced);
        const uint32_t js = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
        const uint32_t nw = js < 64 ? js + 1 : (nch - k < 64 ? nch - k : 64);
        if (lane < nw && mine) W.entry[c00 + j] = (uint32_t)a;
        if (__ballot(lane < nw && mine && lbad)) bad = true;
        if (js < 64) {
            e = __shfl(q > a ? q : a, (int)js);  // (an entry past the chunk passes through)
        } else {
            e = (int32_t)W.sexit[c00 + k + nw - 1];
        }
        k += nw;
        // chunks inside a long token: no token starts there
        if (k < nch && e >= (int32_t)(k + 1) * kJC) {
            const uint32_t k2 = e >= nb ? nch : (uint32_t)(e / kJC);
            for (uint32_t x = k + lane; x < k2; x += 64) W.entry[c00 + x] = (uint32_t)e;
            k = k2;
        }
        if (bad) break;
    }
    // the chain must end exactly at the stream's end (else the last token runs past the input)
    if (lane == 0 && (bad || e != nb)) H.state = 1;
}

// ---- 2a: the true chain of each chunk: tokens, output bytes, forms and metas
__global__ __launch_bounds__(64) void kj_count(DecompressArgs A, JWork W) {
    const uint32_t total = W.cbase[A.count];
    const uint32_t c = blockIdx.x * 64 + threadIdx.x;
    if (c >= total) return;
    const uint32_t s = chunk_stream(W.cbase, (uint32_t)A.count, c);
    if (W.head[s].state) return;
    const uint8_t *b = A.in + A.in_off[s], *lo = A.in, *hi = A.in + A.in_off[A.count];
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;
    const int32_t c0 = (int32_t)(c - W.cbase[s]) * kJC, ce = c0 + kJC < nb ? c0 + kJC : nb;
    int32_t p = (int32_t)W.entry[c];
    uint32_t n = 0, fl = 0;
    uint64_t out = 0;
    while (p < ce) {
        K2Tok t;
        int r;
        const int32_t ad = jadv(b, p, nb, lim32, limit, lo, hi, t, r);
        if (ad < 0) {
            fl |= kJFBad;
            break;
        }
        if (r == kScanReset) {
            fl |= (out ? kJFResetLate : 0) | kJFReset | (n == 0 ? 0 : kJFOutFirst);
            fl = (fl & 0xffu) | (t.marg << 8);
        } else if (r == kParseToken) {
            n++;
            out += (uint64_t)t.L;
        }
        p += ad;
    }
    W.cnt[c] = n;
    W.cout[c] = out;
    W.cflag[c] = fl;
}

// ---- 2b: token and output positions of the chunks; the stream's checks (wave per stream)
__global__ __launch_bounds__(64) void kj_scan(DecompressArgs A, JWork W, uint64_t *tok_alloc) {
    const uint32_t s = blockIdx.x, lane = threadIdx.x;
    JHead &H = W.head[s];
    if (H.state) return;
    const uint32_t c00 = H.chunk0, nch = H.nchunk;
    uint64_t tcarry = 0, ocarry = 0;
    int32_t bsl = -1;
    bool bad = false;
    for (uint32_t k = 0; k < nch; k += 64) {
        const uint32_t j = k + lane;
        const bool mine = j < nch;
        const uint64_t n = mine ? W.cnt[c00 + j] : 0, o = mine ? W.cout[c00 + j] : 0;
        const uint32_t fl = mine ? W.cflag[c00 + j] : 0;
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
        const bool rbad = mine && (fl & kJFReset) && (obefore != 0 || (fl & (kJFOutFirst | kJFResetLate)));
        if (__ballot(rbad || (mine && (fl & kJFBad)))) bad = true;
        const uint64_t rm = __ballot(mine && (fl & kJFReset));
        if (rm) bsl = (int32_t)((__shfl(fl, 63 - __builtin_clzll(rm)) >> 8) & 0xff);
        tcarry = __shfl(tcarry + in, 63);
        ocarry = __shfl(ocarry + io, 63);
    }
    if (lane != 0) return;
    const uint64_t cap = A.out_off[s + 1] - A.out_off[s];
    if (!bad && ocarry > 0 && bsl < 0) bad = true;  // "missed meta": a token before the window is set
    if (!bad && ocarry > cap) {
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

// ---- 2c: one record per token (lane per chunk); distances against the window; Break positions
__global__ __launch_bounds__(64) void kj_emit(DecompressArgs A, JWork W) {
    const uint32_t total = W.cbase[A.count];
    const uint32_t c = blockIdx.x * 64 + threadIdx.x;
    if (c >= total) return;
    const uint32_t s = chunk_stream(W.cbase, (uint32_t)A.count, c);
    JHead &H = W.head[s];
    if (H.state) return;
    const uint8_t *b = A.in + A.in_off[s], *lo = A.in, *hi = A.in + A.in_off[A.count];
    const int32_t nb = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int64_t limit = A.block_size_limit;
    const int32_t lim32 = limit == 0 || limit > 0x7fffffff ? 0x7fffffff : (int32_t)limit;
    const int32_t c0 = (int32_t)(c - W.cbase[s]) * kJC, ce = c0 + kJC < nb ? c0 + kJC : nb;
    const int32_t bsl = H.bsl;
    JTok *rec = W.tok + H.tok0 + W.ctbase[c];
    uint64_t dst = W.cobase[c];
    int32_t p = (int32_t)W.entry[c];
    bool far = false;
    while (p < ce) {
        K2Tok t;
        int r;
        const int32_t ad = jadv(b, p, nb, lim32, limit, lo, hi, t, r);
        if (r == kParseToken) {
            far |= t.cp && bsl < 30 && t.D > (1u << bsl);  // ErrOverflow (reader.go:256-258): the exact decoder
            *rec++ = JTok{(uint32_t)dst, (uint32_t)t.L, t.cp ? (kJCopy | t.D) : 0u, (uint32_t)(p + t.j)};
            dst += (uint64_t)t.L;
        } else if (r == kParseSkip && A.breaks) {
            const V16 h = jbytes(b, p, lo, hi);
            if (((uint32_t)h.lo & 0xffffu) == (0x80u | ((kMetaBreak | kMetaLen0) << 8))) {
                const uint64_t at = atomicAdd((unsigned long long *)A.breaks, 1ull);
                if (at < A.breaks_cap) A.breaks[1 + at] = dst;
            }
        }
        p += ad > 0 ? ad : 1;
    }
    if (far) H.state = 1;
}

// ---- 3: literal and zero bytes, and a pointer for every copied byte (thread per 16 output bytes)
// output bytes [q, q + n) of stream s (n <= 16, inside its output): bytes into by, pointers into pt.
// Pointers and the ptr array count from g0 = out_off[0] rounded down to 16 bytes: a batch may be a view
// into a larger one (absolute offsets), whose bytes before out_off[0] are never touched.
__device__ __forceinline__ void kj_piece(const DecompressArgs &A, const JWork &W, const JHead &H, uint32_t s, uint64_t q, uint32_t n,
                                         uint64_t g0, uint32_t *by, uint32_t *pt) {
    const uint64_t base = A.out_off[s];
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
            for (uint32_t k = 0; k < 16; k++) pt[k] = p0 + k >= D ? x + k - D : kJZero;
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
            pt[k] = p >= D ? x - D : kJZero;
        }
        by[k >> 2] |= v << (8 * (k & 3));
    }
}

__global__ __launch_bounds__(256) void kj_expand(DecompressArgs A, JWork W) {
    const uint64_t ob = A.out_off[0], g0 = ob & ~15ull, end = A.out_off[A.count];
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
    const uint64_t end = A.out_off[A.count] - (A.out_off[0] & ~15ull);  // (ptr counts from g0)
    bool changed = false;
    for (uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; g < end; g += (uint64_t)gridDim.x * blockDim.x * 4) {
        uint4 v = g + 4 <= end ? *(const uint4 *)(W.ptr + g) : make_uint4(kJGap, kJGap, kJGap, kJGap);
        if (g + 4 > end)
            for (uint64_t k = g; k < end; k++) (&v.x)[k - g] = W.ptr[k];
        uint32_t *e = &v.x;
        bool any = false;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t q = e[k];
            if (q >= kJZero || q == (uint32_t)(g + k)) continue;
            const uint32_t r = W.ptr[q];
            if (r != q) {
                e[k] = r;
                any = true;
            }
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
    const uint64_t g0 = A.out_off[0] & ~15ull, end = A.out_off[A.count] - g0;
    uint8_t *o = A.out + g0;
    for (uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; g < end; g += (uint64_t)gridDim.x * blockDim.x * 4) {
        for (uint64_t x = g; x < g + 4 && x < end; x++) {
            const uint32_t q = W.ptr[x];
            if (q == kJGap || q == (uint32_t)x) continue;
            o[x] = q == kJZero ? (uint8_t)0 : o[q];
        }
    }
}

// ---- 5b: results, or the stream to the exact decoder
__global__ __launch_bounds__(256) void kj_final(DecompressArgs A, JWork W) {
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
        }
    }
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// the workspace layout of a batch (in_total / out_total: the end offsets in_off[count], out_off[count])
struct JLayout {
    uint64_t chunks, tok_cap;
    size_t o_head, o_cbase, o_entry, o_sexit, o_bits, o_cnt, o_cout, o_cflag, o_ctb, o_cob, o_tok, o_ptr, o_pass, total;
    JLayout(uint64_t count, uint64_t in_total, uint64_t out_total) {
        chunks = in_total / kJC + 2 * count + 2;
        tok_cap = in_total + 16;
        size_t off = 0;
        auto take = [&](size_t n) {
            const size_t o = off;
            off += al256(n);
            return o;
        };
        o_head = take(sizeof(JHead) * count), o_cbase = take(4 * (count + 1)), o_entry = take(4 * chunks), o_sexit = take(4 * chunks),
        o_bits = take(4 * kJW * chunks), o_cnt = take(4 * chunks), o_cout = take(8 * chunks), o_cflag = take(4 * chunks),
        o_ctb = take(8 * chunks), o_cob = take(8 * chunks), o_tok = take(sizeof(JTok) * tok_cap), o_ptr = take(4 * out_total + 16),
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
    const uint64_t out_total = out_bytes + 16;
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
    W.ptr = (uint32_t *)(w + o_ptr);
    W.pass = (uint32_t *)(w + o_pass);
    uint64_t *tok_alloc = (uint64_t *)(W.pass + kJPasses + 2);
    if ((e = hipMemsetAsync(W.pass, 0, 8 * (kJPasses + 2), st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(W.ptr, 0xff, 4 * out_total + 16, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(kj_init, dim3(1), dim3(1024), 0, st, a, W);
    const unsigned cgrid = (unsigned)((chunks + 63) / 64);
    hipLaunchKernelGGL(kj_spec, dim3(cgrid), dim3(64), 0, st, a, W);
    hipLaunchKernelGGL(kj_prop, dim3((unsigned)a.count), dim3(64), 0, st, a, W);
    hipLaunchKernelGGL(kj_count, dim3(cgrid), dim3(64), 0, st, a, W);
    hipLaunchKernelGGL(kj_scan, dim3((unsigned)a.count), dim3(64), 0, st, a, W, tok_alloc);
    hipLaunchKernelGGL(kj_emit, dim3(cgrid), dim3(64), 0, st, a, W);
    const uint64_t pieces = (out_total + 15) / 16;  // (out_total: the batch's output and the alignment slack)
    const unsigned egrid = (unsigned)(pieces / 256 + 1 < 8192 ? pieces / 256 + 1 : 8192);
    hipLaunchKernelGGL(kj_expand, dim3(egrid), dim3(256), 0, st, a, W);
    const uint64_t quads = (out_total + 3) / 4;
    const unsigned jgrid = (unsigned)(quads / 256 + 1 < 8192 ? quads / 256 + 1 : 8192);
    for (int k = 0; k < kJPasses; k++) hipLaunchKernelGGL(kj_jump, dim3(jgrid), dim3(256), 0, st, a, W, k);
    hipLaunchKernelGGL(kj_gather, dim3(jgrid), dim3(256), 0, st, a, W);
    hipLaunchKernelGGL(kj_final, dim3((unsigned)((a.count + 255) / 256)), dim3(256), 0, st, a, W);
    return hipGetLastError();
}

}  // namespace ez
