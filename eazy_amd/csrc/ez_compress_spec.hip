// ez_compress_spec.hip — K1x: data-parallel rounds for long fresh streams.
//
// The general kernel runs one wave per stream, so a batch of few long Writes (C4: 64 x 4 MiB
// gradient buckets) keeps 64 of 1,024 SIMDs busy with a serial chain.  But between two emitting
// positions Writer.Write (writer.go:206-337) is easy to predict: with the pending literal starting
// at `from` (done = from, w.pos = from), every position x >= from is visited until one is
// accepted, so the table at x is the table at `from` updated with every position of [from, x):
// for each hash, the nearest earlier position of [from, x) with that hash, else the entry at
// `from`.  Whether x is accepted then depends on x, that candidate and `from` only, so all
// positions of a stream are judged at once and the first accepted one is kept.  A round:
//   kx_reset  a stream without an accepted position last round is finished: one literal from
//             `from` to its end (writer.go:324-329); the others are listed as active;
//   kx_judge  (a thread per position of the active streams, from `from` on): candidate and test
//             as writer.go:219-301 (writeRunlen :441-489, writeZeros :407-424) would have them;
//             the first accepted position of a stream is kept (atomicMin);
//   kx_merge  the table at that position, from the table at `from`, the scanned tables (below)
//             and the positions of its chunk;
//   general   (spec_mode 1) resumes each stream at that position with that table, takes the one
//             action Go takes there (copy, cut or zero run) and stores its state back: the next
//             round starts where that action ended.
// Before the rounds: kx_init writes the headers; kx_pred hashes every position and finds the
// nearest earlier same-hash position within its 16 Ki-position chunk, and each chunk's last
// positions per hash; kx_scan turns those into each chunk's incoming table (the latest earlier
// chunk's entry).  After the rounds the general kernel (spec_mode 2) takes the streams still
// active from where they stand, and kx_copy writes every literal's bytes (the rounds and the
// spec_mode 1 calls only write the tags and record the literals: a literal can be megabytes).
// Exactness: x is judged against the table Go has there as long as no position of [from, x)
// was accepted, and the first accepted one is found exactly; a position flagged wrongly would
// only cost time (the general kernel judges it again and goes on), a missed one would not, so
// the test below restates the general kernel's lane evaluation term for term.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

namespace ez {
namespace {

constexpr int64_t kChunk = 16384;     // positions per kx_pred chunk (chunk-local distances fit u16)
constexpr uint32_t kNone = 0xffffffffu;
constexpr int64_t kCopyPiece = 65536; // kx_copy: bytes per block step
constexpr int kRounds = 8;            // rounds before the general kernel takes the rest (EZ_K1X_ROUNDS)
// A stream whose accepted position lay within kDenseGap bytes of the round's start in kDenseRounds
// rounds in a row is dense (logs, C4s: one accepted position per round, ~180 k per stream): it
// leaves the rounds for the continuation (K1c / K1L); C4 fp32 has no accepted position and C4h a
// handful per stream.  (Counted in kx_judge instead, any store there cost kx_judge 1 ms at C4.)
constexpr uint32_t kDenseGap = 256, kDenseRounds = 2, kHanded = 0xffffffffu;

struct KxBufs {
    uint64_t kmax;     // chunks per stream
    uint16_t *pred;    // per input byte: distance to the nearest earlier same-hash position of its chunk (0: none)
    uint32_t *tabs;    // per chunk and hash: the incoming entry (after kx_scan)
    uint32_t *first;   // per stream: the round's first accepted position (kNone: none)
    uint32_t *act;     // active streams of the round
    uint32_t *nact;    // [0] active count, [1] literal records
    uint64_t lit_cap;  // literal records reserved
    uint32_t *dense;   // per stream: {the round's start (kNone before round 1), dense rounds in a row (kHanded: left)}
};

__device__ __forceinline__ uint32_t hash4(const uint8_t *q, uint32_t hsh) {
    const uint32_t v = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    return (v * kHashMul) >> hsh;
}

__device__ __forceinline__ uint32_t hshift(int64_t hs) { return 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1))); }

__device__ __forceinline__ int64_t slen(const CompressArgs &A, uint64_t s) { return (int64_t)(A.in_off[s + 1] - A.in_off[s]); }

// stream s's header (writer.go:495-517), its state at position 0, its table zeroed
__global__ __launch_bounds__(64) void kx_init(CompressArgs A, KxBufs B) {
    const uint64_t s = blockIdx.x;
    const int lane = (int)threadIdx.x;
    if (s == 0 && lane == 0) B.nact[1] = 0;
    for (int64_t h = lane; h < A.hs; h += 64) A.spec_tab[s * (uint64_t)A.hs + h] = 0;
    if (lane != 0) return;
    Hdr h;
    if (A.append_magic) { h.put(0x80); h.put(0x02); h.put('e'); h.put('a'); h.put('z'); h.put('y'); }
    if (A.ver != 0) { h.put(0x80); h.put(0x08); h.put((uint32_t)A.ver); }
    h.put(0x80); h.put(0x10); h.put((uint32_t)__builtin_ctzll((uint64_t)A.bs));
    const int64_t cap = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    B.first[s] = 0;  // active in round 1
    B.dense[2 * s] = kNone;
    B.dense[2 * s + 1] = 0;
    // the launcher sized the scratch from max_len: longer streams are refused (as K1s does);
    // a header that does not fit is not written (put_hdr)
    const int err = (uint64_t)slen(A, s) > A.max_len ? EZ_EINVAL : (h.n > cap ? EZ_ENOSPC : EZ_OK);
    if (err) {
        A.spec[s] = SpecState{0u, 0u, 0u, 1u};
        A.out_size[s] = 0;
        if (A.status) A.status[s] = err;
        return;
    }
    uint8_t *o = A.out + A.out_off[s];
    for (int k = 0; k < h.n; k++) o[k] = h.byte(k);
    A.spec[s] = SpecState{0u, 0u, (uint32_t)h.n, 0u};
}

// chunk (s, k): block s * kmax + k, one wave.  The chunk's bytes pass through a 4 KiB LDS ring in
// 1 KiB pieces (one 16-byte load per lane), each loaded two pieces ahead, so the positions'
// sequential lane-ordered exchanges read their 4 bytes from LDS and no step waits for a load.
constexpr int32_t kPredPiece = 1024;
constexpr int32_t kPredRing = 4 * kPredPiece;
__device__ __forceinline__ uint4 kx_ld16z(const uint8_t *w, const uint8_t *blo, const uint8_t *bhi) {
    if (w >= blo && w + 16 <= bhi) return *(const uint4 *)w;
    uint32_t d[4] = {0, 0, 0, 0};
    for (int u = 0; u < 16; u++)
        if (w + u >= blo && w + u < bhi) d[u >> 2] |= (uint32_t)w[u] << (8 * (u & 3));
    return make_uint4(d[0], d[1], d[2], d[3]);
}
__global__ __launch_bounds__(64) void kx_pred(CompressArgs A, KxBufs B) {
    extern __shared__ __attribute__((aligned(16))) uint32_t T[];  // hs entries, then the ring
    const uint64_t s = blockIdx.x / B.kmax, k = blockIdx.x % B.kmax;
    const int lane = (int)threadIdx.x;
    const int64_t n = slen(A, s);
    const int64_t lo = (int64_t)k * kChunk;
    if (lo + 4 > n || (uint64_t)n > A.max_len) return;
    const uint8_t *p = A.in + A.in_off[s];
    uint16_t *pr = B.pred + s * A.max_len;  // per stream: a refused over-long stream cannot shift the others
    const uint32_t hsh = hshift(A.hs);
    uint32_t *R = T + A.hs;
    const uint8_t *blo = A.in, *bhi = A.in + A.in_off[A.count];
    const uint8_t *wa = (const uint8_t *)((uintptr_t)(p + lo) & ~(uintptr_t)3);
    const uint32_t r0 = (uint32_t)((uintptr_t)(p + lo) & 3);
    const int64_t hi = lo + kChunk < n - 3 ? lo + kChunk : n - 3;  // hashed positions: x + 4 <= n
    // pieces of the stage, from floor4(p + lo): piece c holds its bytes [c * 1 KiB, +1 KiB)
    const int32_t np = (int32_t)((hi - lo + r0 + 3 + kPredPiece - 1) / kPredPiece);
    const uint4 v0 = kx_ld16z(wa + 16 * lane, blo, bhi);
    const uint4 v1 = np > 1 ? kx_ld16z(wa + kPredPiece + 16 * lane, blo, bhi) : make_uint4(0, 0, 0, 0);
    for (int64_t h = lane; h < A.hs; h += 64) T[h] = kNone;
    *(uint4 *)(R + 4 * lane) = v0;
    *(uint4 *)(R + kPredPiece / 4 + 4 * lane) = v1;
    for (int32_t c = 0; c < np; c++) {
        // piece c + 2 into registers now, into the ring after this piece's steps (its slot held c - 2)
        const bool more = c + 2 < np;
        const uint4 vn = more ? kx_ld16z(wa + (int64_t)(c + 2) * kPredPiece + 16 * lane, blo, bhi) : make_uint4(0, 0, 0, 0);
        // positions whose first byte lies in piece c
        const int64_t xa = lo + (int64_t)c * kPredPiece - r0, xz = xa + kPredPiece < hi ? xa + kPredPiece : hi;
        for (int64_t b = xa > lo ? xa : lo; b < xz; b += 64) {
            const int64_t x = b + lane;
            if (x < xz) {
                const uint32_t o = (uint32_t)(x - lo) + r0, kq = o >> 2, r = o & 3;
                const uint32_t w0 = R[kq & (kPredRing / 4 - 1)], w1 = R[(kq + 1) & (kPredRing / 4 - 1)];
                const uint32_t h = (__builtin_amdgcn_alignbyte(w1, w0, r) * kHashMul) >> hsh;
                // lane-ordered exchange: the previous value is the nearest earlier position of the
                // chunk with this hash (an earlier lane of this step, or an earlier step)
                const uint32_t prev = atomicExch(&T[h], (uint32_t)x);
                pr[x] = prev == kNone ? (uint16_t)0 : (uint16_t)(x - (int64_t)prev);
            }
        }
        if (more) *(uint4 *)(R + ((c + 2) & 3) * (kPredPiece / 4) + 4 * lane) = vn;
    }
    uint32_t *tab = B.tabs + (uint64_t)blockIdx.x * (uint64_t)A.hs;
    for (int64_t h = lane; h < A.hs; h += 64) tab[h] = T[h];
}

// thread (s, h): incoming entry of every chunk of stream s, in place (0: none before the chunk)
__global__ __launch_bounds__(256) void kx_scan(CompressArgs A, KxBufs B) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t s = t / (uint64_t)A.hs, h = t % (uint64_t)A.hs;
    if (s >= A.count) return;
    const int64_t n = slen(A, s);
    const uint64_t kn = n > 3 ? (uint64_t)((n - 3 + kChunk - 1) / kChunk) : 0;
    uint32_t run = 0;
    const uint64_t ke = kn < B.kmax ? kn : B.kmax;
    uint32_t *e = B.tabs + (s * B.kmax) * (uint64_t)A.hs + h;
    const uint64_t st = (uint64_t)A.hs;
    uint64_t k = 0;
    // eight chunks' entries loaded before any is rewritten (the loads do not wait for each other)
    for (; k + 8 <= ke; k += 8) {
        uint32_t v[8];
#pragma unroll
        for (int t = 0; t < 8; t++) v[t] = e[(k + t) * st];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            e[(k + t) * st] = run;
            if (v[t] != kNone) run = v[t];
        }
    }
    for (; k < ke; k++) {
        const uint32_t v = e[k * st];
        e[k * st] = run;
        if (v != kNone) run = v;
    }
}

// the trailing literal of a stream with nothing more to accept: its tag now, its bytes in kx_copy
__device__ void kx_tail(const CompressArgs &A, const KxBufs &B, uint64_t s) {
    const SpecState sp = A.spec[s];
    const int64_t n = slen(A, s), done = sp.done;
    int64_t op = sp.op;
    const int64_t cap = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    int err = EZ_OK;
    if (done < n) {
        Hdr h;
        if (!hdr_tag(h, kLiteral, n - done)) err = EZ_EINVAL;
        else if (op + h.n > cap) err = EZ_ENOSPC;
        else {
            uint8_t *o = A.out + A.out_off[s] + op;
            for (int k = 0; k < h.n; k++) o[k] = h.byte(k);
            op += h.n;
            if (op + (n - done) > cap) err = EZ_ENOSPC;
            else {
                A.spec_lit[atomicAdd(&B.nact[1], 1u)] = SpecLit{A.in_off[s] + (uint64_t)done, A.out_off[s] + (uint64_t)op, (uint64_t)(n - done)};
                op += n - done;
            }
        }
    }
    A.out_size[s] = (uint64_t)op;
    if (A.status) A.status[s] = err;
    A.spec[s].flags = 1u;
}

// one block: finish the streams whose last round accepted nothing, list the active ones
__global__ __launch_bounds__(1024) void kx_reset(CompressArgs A, KxBufs B, uint32_t dense_rounds) {
    __shared__ uint32_t cnt, pend;
    if (threadIdx.x == 0) cnt = pend = 0;
    __syncthreads();
    for (uint64_t s = threadIdx.x; s < A.count; s += 1024) {
        if (A.spec[s].flags != 0) continue;
        if (B.dense[2 * s + 1] == kHanded) {
            atomicAdd(&pend, 1u);
            continue;
        }
        const uint32_t f = B.first[s];
        if (f == kNone) {
            kx_tail(A, B, s);
            continue;
        }
        atomicAdd(&pend, 1u);
        const uint32_t rs = B.dense[2 * s];
        const uint32_t streak = rs != kNone && f - rs < kDenseGap ? B.dense[2 * s + 1] + 1 : 0u;
        B.first[s] = kNone;
        if (dense_rounds != 0 && streak >= dense_rounds) {  // dense: the continuation takes it
            B.dense[2 * s + 1] = kHanded;
        } else {
            B.dense[2 * s] = A.spec[s].from;
            B.dense[2 * s + 1] = streak;
            B.act[atomicAdd(&cnt, 1u)] = (uint32_t)s;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        B.nact[0] = cnt;
        B.nact[2] = pend;  // streams not finished: the active ones and those handed to the continuation
    }
}

// Would Go's parse, at x with the pending literal from `done` = w.pos (a fresh stream: start 0)
// and candidate cand, take an action?  The general kernel's lane evaluation (ez_compress.hip,
// "per-lane capped evaluation"), with 8-byte extensions: acceptance needs 6 bytes, and an
// extension capped at 8 is accepted there before its exact length is known.
// 16 bytes at y from dword-aligned loads (a dwordx4 and a dword) + v_alignbyte: a byte-unaligned
// 16-byte gather costs the L1 an access per dword it touches (tools/mb_ta.hip); near the batch's
// edges the clamped path
__device__ __forceinline__ V16 ld16_al(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    const uint8_t *a = (const uint8_t *)((uintptr_t)y & ~(uintptr_t)3);
    if (a < lo || a + 20 > hi) return ld_clamped(y, lo, hi);
    const uint32_t r = (uint32_t)((uintptr_t)y & 3);
    const uint4 q = *(const uint4 *)a;
    const uint32_t w4 = *(const uint32_t *)(a + 16);
    const uint32_t e0 = __builtin_amdgcn_alignbyte(q.y, q.x, r), e1 = __builtin_amdgcn_alignbyte(q.z, q.y, r);
    const uint32_t e2 = __builtin_amdgcn_alignbyte(q.w, q.z, r), e3 = __builtin_amdgcn_alignbyte(w4, q.w, r);
    return V16{(uint64_t)e0 | ((uint64_t)e1 << 32), (uint64_t)e2 | ((uint64_t)e3 << 32)};
}

// vx = stream bytes x-8 .. x+7.  Positions in 32 bits (K1x takes streams under 2 GiB): the
// judgement is most of K1x's time and every 64-bit compare or min is two instructions; only the
// window size bs stays 64-bit
// CL(y) gives stream bytes y .. y+15 (y >= -8; kx_judge: from its LDS window when staged)
template <class CL>
__device__ __forceinline__ bool kx_accepts(const CompressArgs &A, const uint8_t *p, int32_t n, int32_t x, int32_t cand, int32_t done,
                                           const V16 vx, const CL &cl16) {
    const int64_t bs = A.bs;
    if (cand >= done && x > cand) {
        // off >= 0 and i > done + off: writeRunlen with st = cand (writer.go:227-231, 441-473)
        const V16 vc = cl16(cand - 8);
        if (cand + 8 < n && vc.hi == 0) return true;  // writeZeros: >= 8 zeros at st
        const uint64_t df = vx.hi ^ vc.hi, db = vx.lo ^ vc.lo;
        int32_t f = df ? (int32_t)(__builtin_ctzll(df) >> 3) : 8;
        f = f < n - x ? f : n - x;
        int32_t c = db ? (int32_t)(__builtin_clzll(db) >> 3) : 8;
        const int32_t cl = cand < x - done ? cand : x - done;
        c = c < cl ? c : cl;
        return f + c >= kMinCopyChunk;  // a run or the cut branch: both emit
    }
    if ((int64_t)(done - cand) > bs) return false;  // far skip (writer.go:221-224)
    // window match against the ring image at w.pos = done (writer.go:233-301): block[y & mask]
    // holds stream byte done - bs + ((y - done) & mask), zero before the stream
    V16 vc;
    if (cand - 8 >= 0 && (int64_t)cand - 8 >= (int64_t)done - bs && cand + 8 <= done) {
        vc = cl16(cand - 8);
    } else {
        vc = V16{0, 0};
        const int64_t mask = bs - 1;
        for (int t = 0; t < 16; t++) {
            const int64_t q = (int64_t)done - bs + (((int64_t)cand - 8 + t - done) & mask);
            const uint64_t b = q >= 0 ? p[q] : 0;
            if (t < 8) vc.lo |= b << (8 * t);
            else vc.hi |= b << (8 * (t - 8));
        }
    }
    const uint64_t df = vx.hi ^ vc.hi, db = vx.lo ^ vc.lo;
    int32_t f = df ? (int32_t)(__builtin_ctzll(df) >> 3) : 8;
    f = f < n - x ? f : n - x;
    int32_t c = db ? (int32_t)(__builtin_clzll(db) >> 3) : 8;
    c = c < x - done ? c : x - done;
    // the two trims (writer.go:280-291): the copy stays within bs of x and ends by w.pos
    int64_t len = f + c;
    const int64_t t1 = bs - (int64_t)(x - cand), t2 = (int64_t)(done - cand + c);
    len = len < t1 ? len : t1;
    len = len < t2 ? len : t2;
    return len >= kMinCopyChunk;
}

// Blocks step over (segment j, active stream a): segments of kSeg positions from `from` on (one
// kx_pred chunk each), in steps of 256 positions, so the early segments of every active stream are
// judged first and the rest of a stream's segment is skipped once an accepted position before its
// step is known.  The block stages the segment's bytes and the kBack bytes before it in LDS by
// coalesced 16-byte loads: a candidate is the nearest earlier same-hash position (C4's fp32 buckets:
// ~1 KiB back with 1,024 hashes), so nearly every candidate's 16 bytes come from LDS instead of a
// gather that missed the CU's caches (the staged bytes of that piece were another block's); a
// candidate farther back is loaded from the batch.
constexpr int32_t kSeg = (int32_t)kChunk;  // positions per block task
constexpr int32_t kBack = 8192;            // history bytes staged before the segment
constexpr int32_t kStageWords = (kBack + kSeg + 48) / 4;
static_assert(kStageWords % 4 == 0, "the stage is loaded in 16-byte pieces");
__global__ __launch_bounds__(256) void kx_judge(CompressArgs A, KxBufs B) {
    extern __shared__ __attribute__((aligned(16))) uint32_t S[];  // kStageWords: bytes [xs - kBack - 8, xs + kSeg + 40), aligned
    __shared__ bool skip;
    const uint64_t nact = B.nact[0];
    const uint64_t ks = (A.max_len + kSeg - 1) / kSeg + 1;
    const uint32_t hsh = hshift(A.hs);
    const int lane = (int)(threadIdx.x & 63);
    const uint8_t *lo = A.in, *hi = A.in + A.in_off[A.count];
    for (uint64_t q = blockIdx.x; q < nact * ks; q += gridDim.x) {
        const uint64_t j = q / nact, s = B.act[q % nact];
        const SpecState sp = A.spec[s];
        const int32_t n = (int32_t)slen(A, s), from = (int32_t)sp.from, done = (int32_t)sp.done;  // (< 2 GiB)
        const int32_t xs = (from & ~(kSeg - 1)) + (int32_t)j * kSeg;
        if (xs + 4 > n) continue;  // uniform: the block's values only
        const uint8_t *p = A.in + A.in_off[s];
        const uint16_t *prow = B.pred + s * A.max_len;
        const uint32_t *trow = B.tabs + (s * B.kmax + (uint64_t)(xs / kChunk)) * (uint64_t)A.hs;
        const uint32_t *srow = A.spec_tab + s * (uint64_t)A.hs;
        // the stage: aligned words from floor4(p + xs - kBack - 8), bytes outside the batch 0
        const int32_t base = xs - kBack - 8;  // stream offset of the stage's first byte (less r0)
        const uint8_t *wa = (const uint8_t *)((uintptr_t)(p + base) & ~(uintptr_t)3);
        const int32_t r0 = (int32_t)((uintptr_t)(p + base) & 3);
        __syncthreads();  // the previous task's readers are done
        if (threadIdx.x == 0) skip = (int64_t)xs > (int64_t)__atomic_load_n(&B.first[s], __ATOMIC_RELAXED);
        __syncthreads();
        if (skip) continue;
        for (int32_t k = 4 * (int32_t)threadIdx.x; k < kStageWords; k += 4 * 256) {
            const uint8_t *w = wa + 4 * k;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (w >= lo && w + 16 <= hi) {
                v = *(const uint4 *)w;
            } else {
                uint32_t d[4] = {0, 0, 0, 0};
                for (int t = 0; t < 16; t++)
                    if (w + t >= lo && w + t < hi) d[t >> 2] |= (uint32_t)w[t] << (8 * (t & 3));
                v = make_uint4(d[0], d[1], d[2], d[3]);
            }
            *(uint4 *)(S + k) = v;
        }
        // the chunk's incoming entries (a position whose hash has no earlier one in the chunk)
        uint32_t *T = S + kStageWords;
        for (int32_t h = (int32_t)threadIdx.x; h < (int32_t)A.hs; h += 256) T[h] = trow[h];
        __syncthreads();
        // bytes y .. y+15 of the stream: staged when y >= base, else from the batch
        auto cl16 = [&](int32_t y) -> V16 {
            if (y >= base) {
                const uint32_t o = (uint32_t)(y - base + r0), kq = o >> 2, r = o & 3;
                const uint32_t d0 = S[kq], d1 = S[kq + 1], d2 = S[kq + 2], d3 = S[kq + 3], d4 = S[kq + 4];
                return V16{(uint64_t)__builtin_amdgcn_alignbyte(d1, d0, r) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, r) << 32),
                           (uint64_t)__builtin_amdgcn_alignbyte(d3, d2, r) | ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, r) << 32)};
            }
            return ld16_al(p + y, lo, hi);
        };
        // The steps: no barrier among them (the stage is read-only now), each wave decides alone
        // whether an accepted position before its steps is known (a wave that skips steps only skips
        // positions after an accepted one, so the first accepted position stays exact, stale reads
        // included).  Four steps of 256 positions per group; the next group's kx_pred distances and
        // the first accepted position are loaded at the top of a group, four steps before their use.
        const int32_t xe = xs + kSeg < n - 3 ? xs + kSeg : n - 3;  // positions x with x + 4 <= n
        const int32_t tid = (int32_t)threadIdx.x;
        auto ldd = [&](int32_t x) -> uint32_t { return x < xe ? (uint32_t)prow[x] : 0u; };
        int32_t xb = xs;
        uint32_t fa = __atomic_load_n(&B.first[s], __ATOMIC_RELAXED);
        uint32_t dA = ldd(xb + tid), dB = ldd(xb + 256 + tid), dC = ldd(xb + 512 + tid), dD = ldd(xb + 768 + tid);
        auto step = [&](int32_t x, uint32_t d) {
            bool acc = false;
            if (x >= from && x < xe) {
                const uint32_t o = (uint32_t)(x - 8 - base + r0), kq = o >> 2, r = o & 3;
                const uint32_t d0 = S[kq], d1 = S[kq + 1], d2 = S[kq + 2], d3 = S[kq + 3], d4 = S[kq + 4];
                const V16 vx{(uint64_t)__builtin_amdgcn_alignbyte(d1, d0, r) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, r) << 32),
                             (uint64_t)__builtin_amdgcn_alignbyte(d3, d2, r) | ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, r) << 32)};
                const uint32_t h = ((uint32_t)vx.hi * kHashMul) >> hsh;
                // nearest earlier same-hash position (chunk-local, else the chunk's incoming entry);
                // before `from` the table at `from` holds the entry
                const int32_t pc = d ? x - (int32_t)d : (int32_t)T[h];
                const int32_t cand = pc >= from ? pc : (int32_t)srow[h];
                acc = kx_accepts(A, p, n, x, cand, done, vx, cl16);
            }
            const uint64_t m = wballot(acc);
            if (m && lane == ffs64(m)) atomicMin(&B.first[s], (uint32_t)x);
        };
        for (; xb < xe; xb += 1024) {
            if ((int64_t)xb > (int64_t)fa) break;  // (wave-uniform)
            const int32_t xn = xb + 1024 + tid;
            const uint32_t nA = ldd(xn), nB = ldd(xn + 256), nC = ldd(xn + 512), nD = ldd(xn + 768);
            const uint32_t fn = __atomic_load_n(&B.first[s], __ATOMIC_RELAXED);
            step(xb + tid, dA);
            if (xb + 256 < xe) step(xb + 256 + tid, dB);
            if (xb + 512 < xe) step(xb + 512 + tid, dC);
            if (xb + 768 < xe) step(xb + 768 + tid, dD);
            dA = nA;
            dB = nB;
            dC = nC;
            dD = nD;
            fa = fn;
        }
    }
}

// the table at first[s]: the table at `from`, then every position of [from, first) in order,
// last writer wins (not the largest: after a cut, writer.go:464-473, `from` can lie before
// positions the table already holds, and Go visits them again)
__global__ __launch_bounds__(256) void kx_merge(CompressArgs A, KxBufs B) {
    extern __shared__ uint32_t T[];
    uint32_t *U = T + A.hs;  // 1 + the last position of the current chunk's part, 0: none
    const uint64_t s = blockIdx.x;
    if (A.spec[s].flags != 0 || B.first[s] == kNone) return;
    const int64_t from = A.spec[s].from, f = B.first[s];
    uint32_t *tab = A.spec_tab + s * (uint64_t)A.hs;
    const int64_t c = f / kChunk, cs = c * kChunk;
    const uint32_t *inc = B.tabs + (s * B.kmax + (uint64_t)c) * (uint64_t)A.hs;
    for (int64_t h = threadIdx.x; h < A.hs; h += 256) {
        uint32_t v = tab[h];
        // positions of [from, cs): the latest before the chunk, when it is not before `from`
        if (from < cs && (int64_t)inc[h] >= from) v = inc[h];
        T[h] = v;
        U[h] = 0;
    }
    __syncthreads();
    const uint8_t *p = A.in + A.in_off[s];
    const uint32_t hsh = hshift(A.hs);
    for (int64_t x = (cs > from ? cs : from) + threadIdx.x; x < f; x += 256) atomicMax(&U[hash4(p + x, hsh)], (uint32_t)x + 1u);
    __syncthreads();
    for (int64_t h = threadIdx.x; h < A.hs; h += 256) tab[h] = U[h] ? U[h] - 1u : T[h];
}

// every recorded literal's bytes, 64 KiB per block step
__global__ __launch_bounds__(256) void kx_copy(CompressArgs A, KxBufs B) {
    const uint64_t nl = B.nact[1] < B.lit_cap ? B.nact[1] : B.lit_cap;
    const uint64_t kp = (A.max_len + kCopyPiece - 1) / kCopyPiece;
    const uint8_t *lo = A.in, *hi = A.in + A.in_off[A.count];
    for (uint64_t q = blockIdx.x; q < nl * kp; q += gridDim.x) {
        const SpecLit L = A.spec_lit[q / kp];
        const uint64_t b = (q % kp) * (uint64_t)kCopyPiece;
        if (b >= L.len) continue;
        const uint64_t e = b + kCopyPiece < L.len ? b + kCopyPiece : L.len;
        const uint8_t *src = A.in + L.src;
        uint8_t *dst = A.out + L.dst;
        for (uint64_t k = b + 16 * threadIdx.x; k < e; k += 16 * 256) {
            const V16 v = src + k + 16 <= hi ? ld16v(src + k) : ld_clamped(src + k, lo, hi);
            if (k + 16 <= e) st16v(dst + k, v);
            else put_small(dst + k, v, (uint32_t)(e - k));
        }
    }
}

int rounds() {
    static const int r = [] {
        const int v = knob("EZ_K1X_ROUNDS", kRounds);
        return v >= 0 && v <= 1024 ? v : kRounds;
    }();
    return r;
}

struct Layout {
    uint64_t pred, tabs, first, spec, spec_tab, act, nact, dense, lit, lrec, total, lit_cap;
};

Layout layout(const CompressArgs &a) {
    const uint64_t kmax = (a.max_len + kChunk - 1) / kChunk;
    auto up = [](uint64_t v) { return (v + 255) & ~255ull; };
    Layout l;
    l.lit_cap = a.count * (uint64_t)(2 * rounds() + 1);  // <= 2 per stream per round (general), 1 tail
    l.pred = 0;
    l.tabs = l.pred + up(a.count * a.max_len * 2);
    l.first = l.tabs + up(a.count * kmax * (uint64_t)a.hs * 4);
    l.spec = l.first + up(a.count * 4);
    l.spec_tab = l.spec + up(a.count * sizeof(SpecState));
    l.act = l.spec_tab + up(a.count * (uint64_t)a.hs * 4);
    l.nact = l.act + up(a.count * 4);
    l.dense = l.nact + 256;
    l.lit = l.dense + up(a.count * 8);
    l.lrec = l.lit + up(l.lit_cap * sizeof(SpecLit));
    l.total = l.lrec + (long_applies(a) ? up(long_scratch_bytes(a)) : 0);  // K1L's records
    return l;
}

}  // namespace

// Streams qualify when fresh, one Write each, at least 64 KiB long (below that the general
// kernel's chain is short), their positions and outputs fit u32 and the table fits LDS; the
// scratch (u16 per input byte, one table per chunk) stays bounded.
bool spec_applies(const CompressArgs &a, bool any_len) {
    static const bool off = knob("EZ_K1X", 1) == 0;  // A/B: the general kernel alone
    if (off || a.max_len == 0 || a.ring || a.write_idx || a.start != 0 || !a.header || a.hs > 4096 || (a.max_len < (64u << 10) && !any_len) ||
        a.max_len >= (1ull << 31) || a.count == 0)
        return false;
    const uint64_t chunks = a.count * ((a.max_len + kChunk - 1) / kChunk);
    // kx_pred relies on lane-ordered LDS exchanges, as K1s-T32 (checked on the device once)
    return chunks <= (1u << 20) && a.count * a.max_len <= (64ull << 30) && lds_exchange_in_lane_order();
}

uint64_t spec_scratch_bytes(const CompressArgs &a) { return layout(a).total; }

hipError_t launch_compress_spec(const CompressArgs &a0, uint8_t *scratch, hipStream_t st) {
    const Layout l = layout(a0);
    KxBufs B;
    B.kmax = (a0.max_len + kChunk - 1) / kChunk;
    B.pred = (uint16_t *)(scratch + l.pred);
    B.tabs = (uint32_t *)(scratch + l.tabs);
    B.first = (uint32_t *)(scratch + l.first);
    B.act = (uint32_t *)(scratch + l.act);
    B.nact = (uint32_t *)(scratch + l.nact);
    B.dense = (uint32_t *)(scratch + l.dense);
    B.lit_cap = l.lit_cap;
    CompressArgs a = a0;
    a.spec = (SpecState *)(scratch + l.spec);
    a.spec_first = B.first;
    a.spec_tab = (uint32_t *)(scratch + l.spec_tab);
    a.spec_lit = (SpecLit *)(scratch + l.lit);
    a.spec_nlit = &B.nact[1];
    hipError_t e;
    auto check = [&]() { return (e = hipGetLastError()) == hipSuccess; };
    const unsigned count = (unsigned)a.count;
    const unsigned chunks = (unsigned)(a.count * B.kmax);
    const size_t tlds = (size_t)a.hs * 4;
    static bool pattr = false;
    if (!pattr) {
        (void)hipFuncSetAttribute((const void *)kx_pred, hipFuncAttributeMaxDynamicSharedMemorySize, 4096 * 4 + kPredRing);
        pattr = true;
    }
    hipLaunchKernelGGL(kx_init, dim3(count), dim3(64), 0, st, a, B);
    if (!check()) return e;
    hipLaunchKernelGGL(kx_pred, dim3(chunks), dim3(64), tlds + (size_t)kPredRing, st, a, B);
    if (!check()) return e;
    hipLaunchKernelGGL(kx_scan, dim3((unsigned)((a.count * (uint64_t)a.hs + 255) / 256)), dim3(256), 0, st, a, B);
    if (!check()) return e;
    const unsigned jgrid = 2048;  // 8 blocks of 4 waves per CU (kx_judge: as many as its LDS stage lets fit)
    static bool jattr = false;
    if (!jattr) {
        (void)hipFuncSetAttribute((const void *)kx_judge, hipFuncAttributeMaxDynamicSharedMemorySize, (kStageWords + 4096) * 4);
        jattr = true;
    }
    static const uint32_t dense_rounds = (uint32_t)knob("EZ_K1X_DENSE", (int)kDenseRounds);  // (0: never, A/B)
    for (int r = 0; r < rounds(); r++) {
        hipLaunchKernelGGL(kx_reset, dim3(1), dim3(1024), 0, st, a, B, dense_rounds);
        if (!check()) return e;
        hipLaunchKernelGGL(kx_judge, dim3(jgrid), dim3(256), (size_t)(kStageWords + a.hs) * 4, st, a, B);
        if (!check()) return e;
        hipLaunchKernelGGL(kx_merge, dim3(count), dim3(256), 2 * tlds, st, a, B);
        if (!check()) return e;
        a.spec_mode = 1;
        if ((e = launch_general(a, st)) != hipSuccess) return e;
    }
    // the streams still active (dense accepts, C4s): K1L from where they stand (the general kernel
    // where K1L cannot take the batch); then every recorded literal's bytes
    hipLaunchKernelGGL(kx_reset, dim3(1), dim3(1024), 0, st, a, B, dense_rounds);
    if (!check()) return e;
    a.spec_mode = 2;
    // K1c's passes wait for the host from their third on; when they would run, the host first reads
    // whether any stream is left at all (C4 / C4h: none, and the continuation's ~15 empty launches
    // and K1c's host round trip are skipped)
    bool none_left = false;
    if (long_applies(a0) && chunk_applies(a)) {
        uint32_t h_pend = 1;
        if ((e = hipMemcpyAsync(&h_pend, &B.nact[2], 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        none_left = h_pend == 0;
    }
    if (none_left) e = hipSuccess;
    else if (long_applies(a0)) e = launch_long(a, scratch + l.lrec, st);
    else e = launch_general(a, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kx_copy, dim3(jgrid), dim3(256), 0, st, a, B);
    if (!check()) return e;
    if (knob_str("EZ_K1X_DEBUG")) {  // diagnostics: streams left to the general kernel's serial continuation
        std::vector<SpecState> h(a.count);
        uint32_t nl[2];
        (void)hipStreamSynchronize(st);
        (void)hipMemcpy(h.data(), a.spec, a.count * sizeof(SpecState), hipMemcpyDeviceToHost);
        (void)hipMemcpy(nl, B.nact, 8, hipMemcpyDeviceToHost);
        fprintf(stderr, "K1x: %d rounds, %u literal records; active after the rounds: %u\n", rounds(), nl[1], nl[0]);
    }
    return hipSuccess;
}

}  // namespace ez
