// ez_compress_split.hip — K1s: batch compression of fresh streams in two
// kernels, the greedy parse (K1p) and the token writer (K1e).
//
// Writer.Write (writer.go:206-337) for a fresh stream (SURVEY §8 unit of
// work; 2n <= block, so the ring is the linear history with zeros from `done`
// on: no far skip, no cut, no trim 1).
//
// Why two kernels.  The parse is a serial chain per stream: every window's
// decision needs the table after the previous one.  Writing the tokens
// (Encoder.Tag/Offset :537-597, appendLiteral/appendCopy :519-527) does not
// feed back into that chain, but done inside it (a one-kernel form, round 1) it puts the literal
// loads, the encodes and the stores on every iteration's critical path.  Here
//   K1p (G lanes per stream, the table in LDS) runs only the chain: visit,
//       capped judgement, exact extension of an accepted match, the i+1
//       insert, and one 8-byte match record per accepted match
//       {lit_end, copy length, distance, flag} into a per-stream record slot;
//   K1e (one wave per stream) turns the records into the byte stream: token
//       sizes, a wave prefix sum for their output positions, then every lane
//       writes its token (literal tag, literal bytes, copy tag + offset) with
//       16-byte stores and exact-length tails; long literals are copied by the
//       whole wave.  Streams whose tokens do not fit their slot stop at the
//       last token that fits (EZ_ENOSPC), as the single-kernel path does.
//
// The window.  The G lanes of a stream judge positions i .. i+G-1 at once
// against the table as Go's sequential visits (writer.go:213-217) would leave
// it, and the first accepting lane wins.  Two ways to visit a window:
//   T16 (u16 table, 2 bytes per entry, twice the streams per CU of T32):
//       lanes read the table, a lane's candidate is the nearest earlier lane of
//       the window with the same hash (DPP row shifts) or else the table value,
//       and after the decision the lanes Go visits (those up to the accepting
//       one) store their positions with one ds_write_b16, where same-address
//       stores of one instruction land in ascending lane order (checked on the
//       device once per process; T32 is used if it fails).  Exact for any
//       table contents, so backward jumps need nothing special.
//   T32 (u32 table): one ds_wrxchg_rtn_b32 visits the window in lane order,
//       inserts of lanes Go does not visit are undone with one ds_min_u32,
//       which needs inserts monotone in position: windows that start at or
//       below the highest inserted position are judged one position at a time.
// Acceptance is decided with capped counts, 24 bytes forward and 8 backward
// (minCopyChunk = 6 < 8, writer.go:119, 301); only a saturated count is
// extended, forward and backward at once, 16 bytes per lane.  Each accepted match advances `done` by
// its copy length (>= 6), so a stream of n bytes makes at most n/6 records.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_k1_common.h"

#include <cstdio>
#include <cstring>
#include <atomic>
#include <mutex>
#include <type_traits>
#include <algorithm>
#include <vector>

#ifndef EZ_EXP
#define EZ_EXP 0  // diagnostic builds only: bit 2 = cycle profile of the parse loop
#endif

namespace ez {
namespace {
using namespace k1;

#if (EZ_EXP & 4)
#define EZ_PROF_MARK(k)                                   \
    do {                                                  \
        __builtin_amdgcn_s_waitcnt(0);                    \
        const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
        prof[k] += t_ - prof_t;                           \
        prof_t = t_;                                      \
    } while (0)
#else
#define EZ_PROF_MARK(k) do {} while (0)
#endif

// a match record, 8 bytes: lit_end | copy length << 20 | distance << 40 | force << 60
// (positions < 2^20: streams <= kMaxT32); force: the literal is emitted even when
// empty (writeRunlen :480)
__host__ __device__ __forceinline__ uint64_t rec_pack(int32_t lit_end, int32_t clen, int32_t dist, bool force) {
    return (uint64_t)(uint32_t)lit_end | ((uint64_t)(uint32_t)clen << 20) | ((uint64_t)(uint32_t)dist << 40) | ((uint64_t)force << 60);
}
constexpr int64_t kMaxT16 = 65536;   // T16 positions fit 16 bits (a stream's visited positions are < n - 3)
constexpr int64_t kMaxT32 = 1 << 19; // the judgement packs the candidate into 20 bits (and 2n <= block)

// record slot of stream s: s * rec_cap .. ; every match advances done by >= 6,
// and every Write but the last ends with a marker record
__host__ __device__ __forceinline__ uint64_t rec_cap(const CompressArgs &a) {
    return a.max_len / 6 + 1 + (a.write_idx ? a.max_writes : 0);
}

// bytes [0, k) of v kept, the rest 0 (k <= 0: none, k >= 16: all)
__device__ __forceinline__ V16 keep_low16(V16 v, int32_t k) {
    const uint64_t ml = k >= 8 ? ~0ull : (k <= 0 ? 0ull : (1ull << (8 * k)) - 1);
    const uint64_t mh = k >= 16 ? ~0ull : (k <= 8 ? 0ull : (1ull << (8 * (k - 8))) - 1);
    return V16{v.lo & ml, v.hi & mh};
}

// 16 bytes from y of the match's source side: mode 0 zeros (zero region),
// 1 the stream itself (run length), 2 the ring image of a fresh window
// (bytes before the stream start and from `done` on read 0)
template <class SRC>
__device__ __forceinline__ V16 src16(const SRC &P, int32_t y, int mode, int32_t done) {
    if (mode == 0) return V16{0, 0};
    uint64_t lo, hi;
    P.around(y + 8, lo, hi);  // bytes y .. y+15, zeros before the stream start
    const V16 v{lo, hi};
    return mode == 2 ? keep_low16(v, done - y) : v;
}

// Exact forward and backward match counts of one group at once, past the
// bytes the capped judgement already compared (fromf forward, 8 backward):
// lanes 0..G/2-1 scan forward
// (a+k vs b+k), lanes G/2..G-1 backward (a-1-k vs b-1-k), 16 bytes per lane
// per step, so a count below fromf + 8G bytes costs one load round trip.
template <int G, class SRC>
__device__ __forceinline__ void gext(const SRC &P, bool runf, bool runb, int g, int lj, int32_t a, int32_t b, int mode,
                                     int32_t done, int32_t fromf, int32_t limf, int32_t limb, int32_t &resf, int32_t &resb) {
    constexpr int H = G / 2;
    constexpr uint32_t kHalf = (1u << H) - 1;
    const bool fw = lj < H;
    const int t = lj % H;
    resf = fromf < limf ? fromf : limf;
    resb = 8 < limb ? 8 : limb;
    bool gof = runf && fromf < limf, gob = runb && 8 < limb;
    int32_t basef = fromf, baseb = 8;
    while (__ballot(gof || gob) != 0) {
        const bool mine = fw ? gof : gob;
        const int32_t lim = fw ? limf : limb;
        const int32_t k = (fw ? basef : baseb) + 16 * t;
        int32_t mb = 16;
        if (mine) {
            if (k < lim) {
                const int32_t ya = fw ? a + k : a - k - 16, yb = fw ? b + k : b - k - 16;
                uint64_t alo, ahi;
                P.around(ya + 8, alo, ahi);
                const V16 vb = src16(P, yb, mode, done);
                const uint64_t dl = alo ^ vb.lo, dh = ahi ^ vb.hi;
                if (fw) mb = dl ? (int32_t)(__builtin_ctzll(dl) >> 3) : (dh ? 8 + (int32_t)(__builtin_ctzll(dh) >> 3) : 16);
                else mb = dh ? (int32_t)(__builtin_clzll(dh) >> 3) : (dl ? 8 + (int32_t)(__builtin_clzll(dl) >> 3) : 16);
                if (mb > lim - k) mb = lim - k;
            } else {
                mb = 0;
            }
        }
        const uint32_t bad = gball<G>(mine && mb < 16, g);
        const uint32_t bf = bad & kHalf, bb = bad >> H;
        const int lf = bf ? __builtin_ctz(bf) : 0, lb = bb ? __builtin_ctz(bb) : 0;
        const int32_t mbf = bcast(mb, G * g + lf), mbb = bcast(mb, G * g + H + lb);
        if (gof) {
            if (bf) {
                resf = basef + 16 * lf + mbf;
                resf = resf < limf ? resf : limf;
                gof = false;
            } else {
                basef += 16 * H;
                if (basef >= limf) { resf = limf; gof = false; }
            }
        }
        if (gob) {
            if (bb) {
                resb = baseb + 16 * lb + mbb;
                resb = resb < limb ? resb : limb;
                gob = false;
            } else {
                baseb += 16 * H;
                if (baseb >= limb) { resb = limb; gob = false; }
            }
        }
    }
}

// v of the lane K below in the same 16-lane row (~0u where there is none)
template <int K>
__device__ __forceinline__ uint32_t row_shr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)~0u, (int)v, 0x110 + K, 0xf, 0xf, false);
}
// distance to the nearest earlier lane of the group with the same hash (0: none)
// (ROW: the group is the whole 16-lane row, so a lane K below outside it reads ~0u and never matches)
template <int K, bool ROW>
struct Pred {
    __device__ __forceinline__ static int32_t get(uint32_t h, int lj, int32_t d) {
        const uint32_t hk = row_shr<K>(h);
        d = ((ROW || K <= lj) && hk == h) ? K : d;  // descending K: the nearest one stays
        return Pred<K - 1, ROW>::get(h, lj, d);
    }
};
template <bool ROW>
struct Pred<0, ROW> {
    __device__ __forceinline__ static int32_t get(uint32_t, int, int32_t d) { return d; }
};

// The same search on hashes offset to be nonzero, with DPP bound_ctrl (a lane K below outside the
// row reads 0, which never equals): no v_mov of the row-edge default per step.  Each step is still
// v_mov_dpp + v_cmp + v_cndmask: gfx950 has no DPP form of the VOPC compares.
template <int K>
struct PredZ {
    __device__ __forceinline__ static int32_t get(uint32_t hp, int32_t d) {
        const uint32_t hk = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hp, 0x110 + K, 0xf, 0xf, true);
        d = hk == hp ? K : d;  // descending K: the nearest one stays
        return PredZ<K - 1>::get(hp, d);
    }
};
template <>
struct PredZ<0> {
    __device__ __forceinline__ static int32_t get(uint32_t, int32_t d) { return d; }
};

// ---------------------------------------------------------------- K1p
// MW: streams of several Writes (CompressArgs::write_idx), else one Write each
template <int G, bool T16, bool MW>
__global__ __launch_bounds__(64, 5) void k1_parse(CompressArgs A, uint32_t stride_words, uint32_t table_words, uint64_t *recs,
                                                  uint64_t rcap, int prio) {
    constexpr int S = 64 / G;
    static_assert(!T16 || G <= 16, "T16 predecessor search works within 16-lane DPP rows");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / G, lj = lane % G;
    const int32_t hs = (int32_t)A.hs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));
    uint32_t *htw = (uint32_t *)smem + (uint32_t)g * stride_words;
    uint16_t *hth = (uint16_t *)htw;

    const uint64_t s = (uint64_t)blockIdx.x * S + g;
    const bool have = s < A.count;
    int32_t n = 0;
    const uint8_t *gp = A.in;
    if (have) {
        n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        gp = A.in + A.in_off[s];
    }
    GW P;  // stream bytes through L1/L2 (staging them in LDS after the table cost residency: round 1)
    P.p = gp;
    P.blo = A.in;
    P.bhi = A.in + A.in_off[A.count];
    uint64_t *rec = recs + (have ? s * rcap : 0);
    // ht zero = stream position 0 (writer.go:183, A.2)
    for (int32_t k = 4 * lj; k < (int32_t)table_words; k += 4 * G) *(uint4 *)(htw + k) = make_uint4(0, 0, 0, 0);

    // the launcher sized records and tables from max_len: longer streams are refused
    int err = have && (uint64_t)n > A.max_len ? EZ_EINVAL : 0;
    int32_t i = 0, done = 0, hiw = -1, nrec = 0;  // hiw: highest position in the table (T32)
    // Writes of the stream (writer.go:206: each Write's loop runs to its own len(p)):
    // wend = the current Write's end, wk / wlast = its index / the last one's
    uint64_t wk = 0, wlast = 0;
    int32_t wend = n, wstart = 0;
    if (MW && have) {
        wk = A.write_idx[s];
        wlast = A.write_idx[s + 1] - 1;
        if (A.write_idx[s + 1] <= wk) err = EZ_EINVAL;
        else wend = (int32_t)(A.write_end[wk] - A.in_off[s]);
    }
    bool live = have && !err && (n >= 4 || wk < wlast);
    int32_t guard = 4 * n + 64 + 2 * (int32_t)(wlast - wk);
    // bytes x-8 .. x+7 around this lane's position x (loaded one window ahead)
    // and x+8 .. x+23 (px2, px3), loaded with them: off the table -> candidate chain
    uint64_t pxb = 0, pxf = 0, px2 = 0, px3 = 0;
    if (live) {
        P.around(i + lj, pxb, pxf);
        P.around(i + lj + 16, px2, px3);
    }
#if (EZ_EXP & 4)
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_t = __builtin_amdgcn_s_memtime(), prof_it = 0;
#endif
    while (__ballot(live) != 0) {
#if (EZ_EXP & 4)
        prof_it++;
#endif
        if (live && --guard < 0) { err = EZ_ESTUCK; live = false; }
        // a Write that has no position left ends (its trailing literal, writer.go:324-329, is
        // the emitter's: a marker record), and the next Write starts where it ended
        while (MW && live && i + 4 > wend && wk < wlast) {
            if (lj == 0 && (uint64_t)nrec < rcap) __builtin_nontemporal_store(rec_pack(wend, 0, 0, false), rec + nrec);
            if ((uint64_t)nrec >= rcap) { err = EZ_ESTUCK; live = false; }
            nrec++;
            i = done = wstart = wend;
            wk++;
            wend = (int32_t)(A.write_end[wk] - A.in_off[s]);
            if (live) {
                P.around(i + lj, pxb, pxf);
                P.around(i + lj + 16, px2, px3);
            }
        }
        if (live && i + 4 > wend) live = false;  // the last Write has no position left
        int32_t nvalid = wend - 3 - i < G ? wend - 3 - i : G;
        if (!T16 && i <= hiw) nvalid = 1;  // T32, not monotone: one position per window
        const int32_t x = i + lj;
        const bool valid = live && lj < nvalid;

        // ---- visit: hash, lookup (+ insert for T32) in lane order, writer.go:213-217
        // (the chain up to the candidate loads' issue at high wave priority: the loads leave
        // sooner when several waves of the SIMD are ready)
        if (prio & 1) __builtin_amdgcn_s_setprio(3);
        const uint32_t h = valid ? ((uint32_t)pxf * kHashMul) >> hsh : 0u;
        int32_t cand = 0;
        if constexpr (T16) {
            const int32_t tv = valid ? (int32_t)hth[h] : 0;
            const int32_t d = Pred<G - 1, G == 16>::get(h, lj, 0);
            cand = d ? x - d : tv;
        } else {
            if (valid) cand = (int32_t)atomicExch(&htw[h], (uint32_t)x);
        }
        EZ_PROF_MARK(0);

        // ---- capped judgement (exact decision), writer.go:219-301, writeRunlen :441-463
        bool acc = false;
        int32_t info = 0;  // cand | forward count << 20 | backward count << 25 | rl << 29 | zr << 30
        uint64_t pcb = 0, pcf = 0, pc2 = 0, pc3 = 0;
        if (valid) {  // the candidate's bytes, in one wait
            P.around(cand, pcb, pcf);
            P.around(cand + 16, pc2, pc3);
        }
        if (prio & 1) __builtin_amdgcn_s_setprio(0);
        EZ_PROF_MARK(5);
        if (valid) {
            const bool rl = cand >= done && cand < x;
            const bool zr = rl && cand + 8 < wend && pcf == 0;
            // writeRunlen's backward scan stays inside this Write's p (st+jb >= 0, writer.go:458)
            const int32_t bl = rl ? ((x - done) < cand - wstart ? (x - done) : cand - wstart) : x - done;
            int32_t jb = clz_bytes(pxb ^ pcb);
            jb = jb < bl ? jb : bl;
            // forward, 24 bytes capped; the window branch compares the ring image (0 from done on)
            V16 c2{pc2, pc3};
            if (!rl) c2 = keep_low16(c2, done - cand - 8);
            const uint64_t d0 = pxf ^ (rl ? pcf : low_bytes(pcf, done - cand));
            const uint64_t d1 = px2 ^ c2.lo, d2 = px3 ^ c2.hi;
            int32_t jf = d0 ? ctz_bytes(d0) : (d1 ? 8 + ctz_bytes(d1) : 16 + ctz_bytes(d2));
            jf = jf < wend - x ? jf : wend - x;
            acc = rl ? (zr || jf + jb >= kMinCopyChunk) : ((jf < done - cand ? jf : done - cand) + jb >= kMinCopyChunk);
            int32_t zb = clz_bytes(pcb);
            zb = zb < cand - done ? zb : cand - done;
            // zero region: the zeros from cand on, 24 bytes capped
            int32_t zf = pc2 ? 8 + ctz_bytes(pc2) : 16 + ctz_bytes(pc3);
            zf = zf < wend - cand ? zf : wend - cand;
            const int32_t fk = zr ? zf : jf, bk = zr ? zb : jb;
            info = cand | (fk << 20) | (bk << 25) | ((int32_t)rl << 29) | ((int32_t)zr << 30);
        }
        EZ_PROF_MARK(1);
        const uint32_t am = gball<G>(acc, g);
        const int a = am ? __builtin_ctz(am) : -1;  // the group's first accepting lane

        // ---- T32: undo the inserts of the lanes Go does not visit
        if constexpr (!T16) {
            if (valid && a >= 0 && lj > a) atomicMin(&htw[h], (uint32_t)cand);
        }

        // ---- the accepted match: exact lengths (cooperative extension of saturated counts)
        const int32_t ib = bcast(info, G * g + (a < 0 ? 0 : a));
        // the hash of xa+1 is lane a+1's (when it visited), for the extra insert
        const uint32_t h1v = (uint32_t)bcast((int32_t)h, G * g + (a + 1 < G ? a + 1 : G - 1));
        const bool act = live && a >= 0;
        const int32_t xa = i + a;
        const int32_t ca = ib & 0xfffff, fk = (ib >> 20) & 0x1f, bk8 = (ib >> 25) & 0xf;
        const bool rl = (ib >> 29) & 1, zr = (ib >> 30) & 1;
        const int mode = zr ? 0 : (rl ? 1 : 2);
        const int32_t fa = zr ? ca : xa;
        EZ_PROF_MARK(2);
        const int32_t blim = zr ? ca - done : (rl ? ((xa - done) < ca - wstart ? (xa - done) : ca - wstart) : xa - done);
        int32_t fx, cx;
        gext<G, GW>(P, act && fk == 24, act && bk8 == 8, g, lj, fa, ca, mode, done, 24, wend - fa, blim, fx, cx);
        const int32_t f = fk == 24 ? fx : fk;
        const int32_t c = bk8 == 8 ? cx : bk8;
        EZ_PROF_MARK(3);
        int32_t lit_end = 0, nxt = 0;
        if (act) {
            if (zr) {  // writeZeros :407-439
                lit_end = ca - c;
                nxt = ca + f;
            } else if (rl) {  // writeRunlen :441-489
                lit_end = xa - c;
                nxt = xa + f;
            } else {  // window match, trim 2 (:292-296)
                const int32_t over = ca + f - done;
                lit_end = xa - c;
                nxt = xa + f - (over > 0 ? over : 0);
            }
            const int32_t top = rl ? xa : xa + 1;
            hiw = hiw > top ? hiw : top;
            i = done = nxt;
        } else if (live) {
            const int32_t top = i + nvalid - 1;
            hiw = hiw > top ? hiw : top;
            i += nvalid;
        }
        if (live && (err || (i + 4 > wend && wk == wlast))) live = false;
        // the next window's bytes, in flight while this window's table writes and record go out
        EZ_PROF_MARK(6);
        if (prio & 2) __builtin_amdgcn_s_setprio(3);
        if (live) {
            P.around(i + lj, pxb, pxf);
            P.around(i + lj + 16, px2, px3);
        }
        if (prio & 2) __builtin_amdgcn_s_setprio(0);
        EZ_PROF_MARK(7);

        // ---- T16: the lanes Go visits store their positions (the last of a hash wins)
        if constexpr (T16) {
            if (valid && (a < 0 || lj <= a)) hth[h] = (uint16_t)x;
        }
        if (act && lj == 0) {
            if ((uint64_t)nrec < rcap)
                // non-temporal: the records must not evict the streams' inputs from L2
                __builtin_nontemporal_store(rec_pack(lit_end, nxt - lit_end, zr ? 0 : xa - ca, rl && !zr), rec + nrec);
            // the extra insert of i+1 after a window match (writer.go:315-318)
            if (!rl && xa + 1 + 4 <= wend) {
                const uint32_t h1 = a + 1 < nvalid ? h1v : ((P.u32(xa + 1) * kHashMul) >> hsh);
                if constexpr (T16) hth[h1] = (uint16_t)(xa + 1);
                else htw[h1] = (uint32_t)(xa + 1);
            }
        }
        if (act) {
            if ((uint64_t)nrec >= rcap) { err = EZ_ESTUCK; live = false; }
            nrec++;
        }
        EZ_PROF_MARK(4);
    }
#if (EZ_EXP & 4)
    if (blockIdx.x < 4 && lane == 0)
        printf("prof blk %u it %llu: visit %llu cload %llu judge %llu ballot %llu ext %llu upd %llu xload %llu fin %llu\n", blockIdx.x,
               (unsigned long long)prof_it, (unsigned long long)prof[0], (unsigned long long)prof[5], (unsigned long long)prof[1],
               (unsigned long long)prof[2], (unsigned long long)prof[3], (unsigned long long)prof[6], (unsigned long long)prof[7],
               (unsigned long long)prof[4]);
#endif
    if (have && lj == 0) A.out_size[s] = (uint64_t)nrec | ((uint64_t)err << 48);
}

// ---------------------------------------------------------------- K1p, lean single-Write form
// The same parse as k1_parse<16, true, true, false> (one Write per fresh stream, u16 table,
// 16 lanes per stream, inputs through L1/L2) with a shorter per-window chain:
//  * loads need no bounds logic on waves whose streams all have 8 readable bytes before
//    and 48 after them inside the batch (every wave but the batch's first and last);
//  * the capped forward count compares real stream bytes and takes min(count, done - cand)
//    for window matches: below `done` the ring image is the stream, and trim 2
//    (writer.go:292-296) cuts any window match at w.pos = done, so the zeros the ring holds
//    from done on never reach a decision or a length;
//  * the accepting lane computes its own record and the group's next position; the other
//    lanes take that position with one v_readlane per group (no LDS round trip); the
//    extra insert of i+1 (writer.go:315-318) is the accepting lane's own second store, after
//    the visited lanes' one (LDS stores of one wave land in issue order), hashed from its
//    own bytes x+1 .. x+4;
//  * only saturated counts (24 forward / 8 backward with room left) take the cooperative
//    extension (gext), as a rare branch.
// Loads of the lean parse carry no bounds logic: every stream the loop reads has 64 readable bytes
// before it and 64 after it (k1_lean copies the few streams at the batch's edges into padded
// slots first), so each piece is one plain aligned load.
// (global address space: plain global_load instructions, not flat ones, which would also count
// against the LDS counter and wait on the ds_bpermute traffic)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) uint32_t *gu32p;
typedef const __attribute__((address_space(1))) u32x4 *gu128p;
struct LeanIn {
    __device__ __forceinline__ uint32_t dw(const uint8_t *w) const { return *(gu32p)w; }
    __device__ __forceinline__ uint4 dw4(const uint8_t *w) const {
#if (EZ_EXP & 16)
        const u32x4 v = __builtin_nontemporal_load((gu128p)w);
#else
        const u32x4 v = *(gu128p)w;
#endif
        return make_uint4(v.x, v.y, v.z, v.w);
    }
};
// gext's view of a padded stream: GW::around without the batch-bounds branch (bytes before the
// stream start read 0; gext reads at most 16 bytes before it and 16 after its end)
struct GWU {
    const uint8_t *p;
    __device__ __forceinline__ void around(int32_t y, uint64_t &before, uint64_t &from) const {
        V16 v = ld16v(p + (y - 8));
        if (y < 8) {
            const int32_t k = 8 - y;
            v.lo &= k >= 8 ? 0ull : ~0ull << (8 * k);
            v.hi &= k >= 16 ? 0ull : (k <= 8 ? ~0ull : ~0ull << (8 * (k - 8)));
        }
        before = v.lo;
        from = v.hi;
    }
};

// The window's bytes of a group by one coalesced dword per lane: lane k of the group loads
// dword k of the 64-byte region from floor4(p + i - 8), and every lane assembles its 32 bytes
// (x-8 .. x+23) from 9 of those dwords with ds_bpermute + v_alignbyte.  One global load of 64 lanes
// touching ~4 cache lines, instead of two 16-byte loads per lane at 64 overlapping unaligned
// addresses: the parse is bound by the vector-memory path's per-lane L1 accesses (TA/TD ~90 % busy
// at two byte-unaligned 16-byte loads per lane and window), not by HBM.
struct WinDw {
    uint32_t dw, r0;  // this lane's dword of the region; the region's start offset (0..3) from p + i - 8
    __device__ __forceinline__ void load(const LeanIn &L, const uint8_t *p, int32_t i, int lj) {
        const uintptr_t a = (uintptr_t)(p + i - 8);
        r0 = (uint32_t)(a & 3);
        dw = L.dw((const uint8_t *)((a & ~(uintptr_t)3) + 4 * (uint32_t)lj));
    }
    __device__ __forceinline__ void bytes(int g, int lj, V16 &w0, V16 &w1) const {
        const uint32_t o = (uint32_t)lj + r0, q = o >> 2, r = o & 3;
        const int src = 4 * (16 * g + (int)q);
        uint32_t d[9];
#pragma unroll
        for (int t = 0; t < 9; t++) d[t] = (uint32_t)__builtin_amdgcn_ds_bpermute(src + 4 * t, (int)dw);
        uint32_t b[8];
#pragma unroll
        for (int t = 0; t < 8; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
        w0.lo = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
        w0.hi = (uint64_t)b[2] | ((uint64_t)b[3] << 32);
        w1.lo = (uint64_t)b[4] | ((uint64_t)b[5] << 32);
        w1.hi = (uint64_t)b[6] | ((uint64_t)b[7] << 32);
    }
};

// The window's bytes from a 128-byte region held across windows, with the next one in flight.
// Lane k of a group holds dwords 2k and 2k+1 of the region [p + cb, p + cb + 128) (one aligned
// dwordx2 per lane); a window at i reads bytes i-8 .. i+38, so the region serves every window with
// 0 <= i - 8 - cb <= 80.  Most windows advance by 16 (no accept) or by a short match, so a region
// serves ~4 of them, and the region 64 bytes further on (f, issued one region switch earlier, after
// that window's candidate gathers) is usually resident when the parse gets there: the window-bytes
// load leaves the per-window chain (window bytes -> table -> candidate gather -> decision -> next
// window) except after long jumps.  Regions never start past bmax (their 128 bytes end at most 64
// bytes after the stream) nor more than 64 bytes before it: k1_lean's edge slots guarantee both.
struct WinRoll {
    uint32_t c0, c1, f0, f1;  // this lane's dwords of the current and the prefetched region
    int32_t cb, fb, bmax, pm; // region starts relative to p (4-byte aligned addresses); p & 3
    __device__ __forceinline__ int32_t floor4(int32_t y) const { return y - ((pm + y) & 3); }
    __device__ __forceinline__ void ld(const uint8_t *p, int32_t b, int lj, uint32_t &d0, uint32_t &d1) const {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        typedef const __attribute__((address_space(1))) u32x2 *gu64p;
        const u32x2 v = *(gu64p)(p + b + 8 * lj);
        d0 = v.x;
        d1 = v.y;
    }
    __device__ __forceinline__ void init(const uint8_t *p, int32_t n, int lj, bool live) {
        pm = (int32_t)((uintptr_t)p & 3);
        bmax = floor4(n - 64);
        cb = min(floor4(-8), bmax);
        fb = min(cb + 64, bmax);
        f0 = f1 = 0;
        if (live) ld(p, cb, lj, f0, f1);
        // (c only ever from these moves: no load is pending on c's registers at the loop's head, where
        // a wait for one would wait for the prefetch behind it too)
        asm volatile("v_mov_b32 %0, %1" : "=v"(c0) : "v"(f0));
        asm volatile("v_mov_b32 %0, %1" : "=v"(c1) : "v"(f1));
        if (live) ld(p, fb, lj, f0, f1);
    }
    // the region for the window at i (group-uniform), after this window's gathers
    // (one path for both cases -- the region moves from f to c, the next one is loaded into f -- so
    // that the prefetch lands in f's registers: with the long jump loading c in a branch of its own,
    // the merged c took f's registers, the prefetch went to others and was copied into f's at once,
    // a wait for the load just issued on every region switch)
    __device__ __forceinline__ void advance(const uint8_t *p, int32_t i, int lj, bool live) {
        const int32_t y = i - 8;
        if (live && !(y >= cb && y - cb <= 80)) {
            if (!(y >= fb && y - fb <= 80)) {  // a long jump: the region is loaded on the chain
                fb = min(floor4(y), bmax);
                ld(p, fb, lj, f0, f1);
            }
            cb = fb;
            // (moves the compiler cannot sink past the load below: phi copies placed after it made
            // it load f elsewhere and copy at once)
            asm volatile("v_mov_b32 %0, %1" : "=v"(c0) : "v"(f0));
            asm volatile("v_mov_b32 %0, %1" : "=v"(c1) : "v"(f1));
            fb = min(cb + 64, bmax);
            ld(p, fb, lj, f0, f1);
        }
    }
    __device__ __forceinline__ void bytes(int32_t i, int g, int lj, V16 &w0, V16 &w1) const {
        const uint32_t o = (uint32_t)(i - 8 - cb + lj), q = o >> 2, r = o & 3;
        const int src = 4 * (16 * g + (int)(q >> 1));
        uint32_t e[10];
#pragma unroll
        for (int t = 0; t < 5; t++) {
            e[2 * t] = (uint32_t)__builtin_amdgcn_ds_bpermute(src + 4 * t, (int)c0);
            e[2 * t + 1] = (uint32_t)__builtin_amdgcn_ds_bpermute(src + 4 * t, (int)c1);
        }
        // an odd first dword starts one further (bit selects: a ?: on the array became a scratch index)
        const uint32_t m = 0u - (q & 1);
        uint32_t d[9];
#pragma unroll
        for (int t = 0; t < 9; t++) d[t] = (e[t + 1] & m) | (e[t] & ~m);
        uint32_t b[8];
#pragma unroll
        for (int t = 0; t < 8; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
        w0.lo = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
        w0.hi = (uint64_t)b[2] | ((uint64_t)b[3] << 32);
        w1.lo = (uint64_t)b[4] | ((uint64_t)b[5] << 32);
        w1.hi = (uint64_t)b[6] | ((uint64_t)b[7] << 32);
    }
};

// WinRoll with the current region in LDS (LW): the group's 144-byte buffer holds stream bytes
// [cb, cb + 128); a window's 32 bytes are nine aligned dword reads and eight v_alignbyte, instead
// of ten ds_bpermute, nine selects and eight v_alignbyte from the lanes' registers.  R: the
// farthest window start the region serves (80 for 32-byte windows; 64 for the 48-byte windows of
// the 40-byte judgement, whose bytes reach i + 15 + 39)
template <int R = 80, int G = 16>
struct WinLds {
    static constexpr int LB = 128 / G;  // bytes of the 128-byte region per lane (8 or 16)
    typedef unsigned int u32v __attribute__((ext_vector_type(LB / 4)));
    u32v f;  // this lane's dwords of the prefetched region
    int32_t cb, fb, bmax, pm;
    uint8_t *wl;  // the group's buffer (LDS)
    __device__ __forceinline__ int32_t floor4(int32_t y) const { return y - ((pm + y) & 3); }
    __device__ __forceinline__ void ld(const uint8_t *p, int32_t b, int lj, u32v &d) const {
        typedef const __attribute__((address_space(1))) u32v *gp;
        d = *(gp)(p + b + LB * lj);
    }
    __device__ __forceinline__ void put(int lj) const { *(u32v *)(wl + LB * lj) = f; }
    __device__ __forceinline__ void init(const uint8_t *p, int32_t n, int lj, bool live) {
        pm = (int32_t)((uintptr_t)p & 3);
        bmax = floor4(n - 64);
        cb = min(floor4(-8), bmax);
        fb = min(cb + 64, bmax);
        f = u32v{};
        if (live) ld(p, cb, lj, f);
        put(lj);
        if (live) ld(p, fb, lj, f);
    }
    __device__ __forceinline__ void advance(const uint8_t *p, int32_t i, int lj, bool live) {
        const int32_t y = i - 8;
        if (live && !(y >= cb && y - cb <= R)) {
            if (!(y >= fb && y - fb <= R)) {
                fb = min(floor4(y), bmax);
                ld(p, fb, lj, f);
            }
            cb = fb;
            put(lj);
            fb = min(cb + 64, bmax);
            ld(p, fb, lj, f);
        }
    }
    __device__ __forceinline__ void bytes(int32_t i, int g, int lj, V16 &w0, V16 &w1) const {
        const uint32_t o = (uint32_t)(i - 8 - cb + lj), r = o & 3;
        const uint32_t *q = (const uint32_t *)(wl + (o & ~3u));
        uint32_t d[9];
#pragma unroll
        for (int t = 0; t < 9; t++) d[t] = q[t];
        uint32_t b[8];
#pragma unroll
        for (int t = 0; t < 8; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
        w0.lo = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
        w0.hi = (uint64_t)b[2] | ((uint64_t)b[3] << 32);
        w1.lo = (uint64_t)b[4] | ((uint64_t)b[5] << 32);
        w1.hi = (uint64_t)b[6] | ((uint64_t)b[7] << 32);
    }
    // x-8 .. x+39 (R = 64: o <= 79, the reads end at byte 131 of the 144-byte buffer).  (EZ_EXP &
    // 131072 builds: three byte-addressed ds_read_b128 -- the LDS runs in unaligned mode under ROCm --
    // which save 14 VALU per window, the 12 v_alignbyte among them, but measured slower: C1 K1 2.13
    // against 1.96 ms, two alternating runs on one box; the unaligned reads cost the LDS more cycles)
    __device__ __forceinline__ void bytes48(int32_t i, int g, int lj, V16 &w0, V16 &w1, V16 &w2) const {
        static_assert(R <= 64, "48-byte windows need the region to reach i + 54");
#if (EZ_EXP & 131072)
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        typedef u32x4 __attribute__((aligned(1))) u32x4u;
        const uint8_t *u = wl + (uint32_t)(i - 8 - cb + lj);
        const u32x4 ua = *(const u32x4u *)u, ub = *(const u32x4u *)(u + 16), uc = *(const u32x4u *)(u + 32);
        w0 = V16{(uint64_t)ua.x | ((uint64_t)ua.y << 32), (uint64_t)ua.z | ((uint64_t)ua.w << 32)};
        w1 = V16{(uint64_t)ub.x | ((uint64_t)ub.y << 32), (uint64_t)ub.z | ((uint64_t)ub.w << 32)};
        w2 = V16{(uint64_t)uc.x | ((uint64_t)uc.y << 32), (uint64_t)uc.z | ((uint64_t)uc.w << 32)};
        return;
#endif
        const uint32_t o = (uint32_t)(i - 8 - cb + lj), r = o & 3;
        const uint32_t *q = (const uint32_t *)(wl + (o & ~3u));
        uint32_t d[13];
#pragma unroll
        for (int t = 0; t < 13; t++) d[t] = q[t];
        uint32_t b[12];
#pragma unroll
        for (int t = 0; t < 12; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
        w0 = V16{(uint64_t)b[0] | ((uint64_t)b[1] << 32), (uint64_t)b[2] | ((uint64_t)b[3] << 32)};
        w1 = V16{(uint64_t)b[4] | ((uint64_t)b[5] << 32), (uint64_t)b[6] | ((uint64_t)b[7] << 32)};
        w2 = V16{(uint64_t)b[8] | ((uint64_t)b[9] << 32), (uint64_t)b[10] | ((uint64_t)b[11] << 32)};
    }
};
constexpr int32_t kWinLdsBytes = 144;


// The 32 bytes y-8 .. y+23 by dword-aligned loads (dwordx4, dwordx4, dword from floor4(p + y - 8))
// and v_alignbyte: a 16-byte load at a byte-unaligned address costs the L1 one access per dword it
// touches, an aligned one a single access (tools/mb_ta.hip, L1-resident: 64 vs 16 ns per scattered
// wave-load), so this is 3 accesses per lane instead of ~8.
// The candidate's 28 bytes y-8 .. y+19 from two dword-aligned 16-byte loads (floor4(p + y - 8)),
// for a forward cap of 20 instead of 24 (EZ_EXP & 8 builds, A/B: one load fewer per lane, more
// matches taking gext)
#if (EZ_EXP & 8)
constexpr int32_t kFwdCap = 20;
#else
constexpr int32_t kFwdCap = 24;
#endif
__device__ __forceinline__ void bytes28(const LeanIn &L, const uint8_t *p, int32_t y, V16 &c0, V16 &c1) {
    const uintptr_t a = (uintptr_t)(p + y - 8);
    const uint32_t r = (uint32_t)(a & 3);
    const uint8_t *w = (const uint8_t *)(a & ~(uintptr_t)3);
    const uint4 q0 = L.dw4(w), q1 = L.dw4(w + 16);
    const uint32_t d[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    uint32_t b[7];
#pragma unroll
    for (int t = 0; t < 7; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
    c0.lo = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
    c0.hi = (uint64_t)b[2] | ((uint64_t)b[3] << 32);
    c1.lo = (uint64_t)b[4] | ((uint64_t)b[5] << 32);
    c1.hi = (uint64_t)b[6];
}

__device__ __forceinline__ void bytes32(const LeanIn &L, const uint8_t *p, int32_t y, V16 &c0, V16 &c1) {
    const uintptr_t a = (uintptr_t)(p + y - 8);
    const uint32_t r = (uint32_t)(a & 3);
    const uint8_t *w = (const uint8_t *)(a & ~(uintptr_t)3);
    const uint4 q0 = L.dw4(w), q1 = L.dw4(w + 16);
    const uint32_t q2 = L.dw(w + 32);
    const uint32_t d[9] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2};
    uint32_t b[8];
#pragma unroll
    for (int t = 0; t < 8; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
    c0.lo = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
    c0.hi = (uint64_t)b[2] | ((uint64_t)b[3] << 32);
    c1.lo = (uint64_t)b[4] | ((uint64_t)b[5] << 32);
    c1.hi = (uint64_t)b[6] | ((uint64_t)b[7] << 32);
}

// y-8 .. y+39 (the 40-byte judgement): dwordx4 x3 + dword from floor4(p + y - 8), unchecked (padded
// streams: k1_lean's edge slots leave 64 readable bytes after every stream)
__device__ __forceinline__ void bytes48(const LeanIn &L, const uint8_t *p, int32_t y, V16 &c0, V16 &c1, V16 &c2) {
    // (floor4(p + y - 8) = floor4(p + y) - 8: one address add, the -8 in the loads' offsets)
    const uintptr_t a = (uintptr_t)(p + y);
    const uint32_t r = (uint32_t)(a & 3);
    const uint8_t *w = (const uint8_t *)(a & ~(uintptr_t)3) - 8;
    const uint4 q0 = L.dw4(w), q1 = L.dw4(w + 16), q2 = L.dw4(w + 32);
    const uint32_t q3 = L.dw(w + 48);
    const uint32_t d[13] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3};
    uint32_t b[12];
#pragma unroll
    for (int t = 0; t < 12; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
    c0 = V16{(uint64_t)b[0] | ((uint64_t)b[1] << 32), (uint64_t)b[2] | ((uint64_t)b[3] << 32)};
    c1 = V16{(uint64_t)b[4] | ((uint64_t)b[5] << 32), (uint64_t)b[6] | ((uint64_t)b[7] << 32)};
    c2 = V16{(uint64_t)b[8] | ((uint64_t)b[9] << 32), (uint64_t)b[10] | ((uint64_t)b[11] << 32)};
}

// Byte counts without branches: v_ffbl / v_ffbh return ~0u for 0, and saturating adds keep that
// "no bit here" through the word offsets, so a min over the words finds the first set bit.
__device__ __forceinline__ uint32_t ffbl32(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t ffbh32(uint32_t x) {
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) { return __builtin_elementwise_add_sat(a, b); }
// equal leading (low-address) bytes of the 24 bytes whose xor is (e0, e1, e2): 0 .. 24
__device__ __forceinline__ int32_t first_diff24(uint64_t e0, uint64_t e1, uint64_t e2) {
    uint32_t m = ffbl32((uint32_t)e0);
    m = min(m, sat_add(ffbl32((uint32_t)(e0 >> 32)), 32u));
    m = min(m, sat_add(ffbl32((uint32_t)e1), 64u));
    m = min(m, sat_add(ffbl32((uint32_t)(e1 >> 32)), 96u));
    m = min(m, sat_add(ffbl32((uint32_t)e2), 128u));
    m = min(m, sat_add(ffbl32((uint32_t)(e2 >> 32)), 160u));
    return (int32_t)min(m >> 3, 24u);
}
// the same over 40 bytes: 0 .. 40
__device__ __forceinline__ int32_t first_diff40(uint64_t e0, uint64_t e1, uint64_t e2, uint64_t e3, uint64_t e4) {
    uint32_t m = ffbl32((uint32_t)e0);
    m = min(m, sat_add(ffbl32((uint32_t)(e0 >> 32)), 32u));
    m = min(m, sat_add(ffbl32((uint32_t)e1), 64u));
    m = min(m, sat_add(ffbl32((uint32_t)(e1 >> 32)), 96u));
    m = min(m, sat_add(ffbl32((uint32_t)e2), 128u));
    m = min(m, sat_add(ffbl32((uint32_t)(e2 >> 32)), 160u));
    m = min(m, sat_add(ffbl32((uint32_t)e3), 192u));
    m = min(m, sat_add(ffbl32((uint32_t)(e3 >> 32)), 224u));
    m = min(m, sat_add(ffbl32((uint32_t)e4), 256u));
    m = min(m, sat_add(ffbl32((uint32_t)(e4 >> 32)), 288u));
    return (int32_t)min(m >> 3, 40u);
}
// the same over 20 bytes (e2: the last 4): 0 .. 20
__device__ __forceinline__ int32_t first_diff20(uint64_t e0, uint64_t e1, uint32_t e2) {
    uint32_t m = ffbl32((uint32_t)e0);
    m = min(m, sat_add(ffbl32((uint32_t)(e0 >> 32)), 32u));
    m = min(m, sat_add(ffbl32((uint32_t)e1), 64u));
    m = min(m, sat_add(ffbl32((uint32_t)(e1 >> 32)), 96u));
    m = min(m, sat_add(ffbl32(e2), 128u));
    return (int32_t)min(m >> 3, 20u);
}
// equal trailing (high-address) bytes of the 8 bytes whose xor is e: 0 .. 8
__device__ __forceinline__ int32_t last_diff8(uint64_t e) {
    const uint32_t m = min(ffbh32((uint32_t)(e >> 32)), sat_add(ffbh32((uint32_t)e), 32u));
    return (int32_t)min(m >> 3, 8u);
}

// Visit by one LDS atomic (MSK): ds_mskor_rtn_b32 sets the lane's u16 table entry to its position
// and returns the word as it was -- lanes of one wave instruction that hit the same word apply in
// ascending lane order (probed once per process, k_lds_mskor_order), so a lane reads the position
// of the nearest earlier lane of its window with the same hash, or the table's entry when there is
// none: the table read, the 15-step DPP predecessor search and the visited lanes' table store in
// one instruction.  Lanes after the window's acceptor, which Go never visits, then put back what
// they found unless it is a position of another such lane (only the first of a hash past the
// acceptor restores; its value is the one Go's table holds).  (The wait is in the asm: the
// compiler does not count an asm's LDS operation.)
__device__ __forceinline__ uint32_t lds_mskor16(uint16_t *hth, uint32_t h, uint32_t val) {
    const uint32_t sh = (h & 1u) << 4;
    const uint32_t addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t *)hth) + ((h >> 1) << 2);
    uint32_t r;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr), "v"(0xffffu << sh), "v"(val << sh) : "memory");
    return (r >> sh) & 0xffffu;
}

// 12-bit entries, five to a 64-bit LDS word (streams of <= 4099 bytes: every position a table
// holds is below 4096): 1,640 B per 1,024-entry table instead of 2,048, so 24 blocks of 4 streams fit
// a CU's LDS instead of 20.  ds_mskor_rtn_b64 reads and sets one entry the way lds_mskor16 does.
__device__ __forceinline__ void t12_at(uint32_t h, uint32_t &addr_off, uint32_t &sh) {
    const uint32_t w = (h * 0x3334u) >> 16;  // h / 5 (h < 4096)
    addr_off = w << 3;
    sh = 12u * (h - 5u * w);
}
__device__ __forceinline__ uint32_t lds_mskor12(uint64_t *tab, uint32_t h, uint32_t val) {
    uint32_t off, sh;
    t12_at(h, off, sh);
    const uint32_t addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t *)tab) + off;
    const uint64_t m = 0xfffull << sh, v = (uint64_t)val << sh;
    uint64_t r;
    asm volatile("ds_mskor_rtn_b64 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr), "v"(m), "v"(v) : "memory");
    return (uint32_t)(r >> sh) & 0xfffu;
}
// one entry set (no return: LDS operations of a wave complete in order, nothing waits for it)
__device__ __forceinline__ void lds_put12(uint64_t *tab, uint32_t h, uint32_t val) {
    uint32_t off, sh;
    t12_at(h, off, sh);
    const uint32_t addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t *)tab) + off;
    const uint64_t m = 0xfffull << sh, v = (uint64_t)val << sh;
    asm volatile("ds_mskor_b64 %0, %1, %2" : : "v"(addr), "v"(m), "v"(v) : "memory");
}

#if (EZ_EXP & 65536)
__device__ unsigned long long g_lean_hist[18];
__device__ unsigned long long g_kc_diag[8];
#endif
constexpr int kEdgeSlots = 40;
constexpr int32_t kEdgeBefore = 64;  // readable bytes before a stream (WinRoll's regions), 64 after it
__host__ __device__ __forceinline__ uint64_t edge_slot_bytes(const CompressArgs &a) { return (a.max_len + kEdgeBefore + 64 + 15) & ~15ull; }
__host__ __device__ __forceinline__ uint64_t edge_area_bytes(const CompressArgs &a) { return 128 + kEdgeSlots * edge_slot_bytes(a) + 16; }

// k1_lean's parse of fresh single-Write streams, 16 lanes (a group) per stream, 4 groups per wave.
// TB: the table's visit -- 0 the DPP search over a u16 table, 16 lds_mskor16, 12 lds_mskor12;
// LW: the window's region in LDS (WinLds) or in the lanes' registers (WinRoll);
// FW: the judgement's forward cap, 24 or 40 bytes (40: 48-byte windows and candidates, LW only);
// PERSIST: a group whose stream ends takes the next one from the batch's queue (a global counter)
// instead of idling until the wave's other three groups end theirs; the grid is then the resident
// waves of the chip, and a wave ends when the queue is empty and its groups are done.
template <int TB, bool LW, int FW, bool PERSIST, int G = 16>
__device__ __forceinline__ void lean_run(const CompressArgs &A, int lj, int g, uint16_t *hth, uint32_t table_words, uint32_t hsh,
                                         uint64_t *recs, uint64_t rcap, int prio, uint8_t *edge, uint8_t *wl) {
    constexpr int S = 64 / G;
    constexpr uint32_t kGMask = (1u << G) - 1;
    constexpr bool W40 = FW == 40;
    static_assert(FW == 24 || (W40 && LW), "the 40-byte judgement reads its windows from the LDS region");
    constexpr int32_t CAP = W40 ? 40 : kFwdCap;
    const LeanIn L{};
    const uint8_t *blo = A.in, *bhi = A.in + A.in_off[A.count];
    uint32_t *queue = (uint32_t *)(edge + 128 + kEdgeSlots * edge_slot_bytes(A)) + 1;  // [0]: edge slots taken
    const uint32_t rcap32 = (uint32_t)rcap;

    // the group's stream: index, bytes, size, error, record base; its parse state
    uint64_t s = (uint64_t)blockIdx.x * S + (uint64_t)g;
    const uint8_t *p = edge + 16;
    int32_t n = 0, i = 0, done = 0, nrec = 0;
    int err = 0;
    bool live = false, pending = false;
    uint64_t *rec = recs;
    V16 z0{0, 0}, z1{0, 0}, z2{0, 0};
    static_assert(G == 16 || LW, "8-lane groups read their windows from the LDS region");
    typename std::conditional<LW, WinLds<W40 ? 64 : 80, G>, WinRoll>::type wr;
    if constexpr (LW) wr.wl = wl;
    // iterations left to the wave (SALU): every stream opened adds its parse's bound, so a correct
    // parse never reaches 0 and a wrong one cannot hang the grid
    int64_t budget = 0;

    // open stream s for the group (group-uniform, in a branch of the group's lanes): table zeroed,
    // edge streams copied into a padded slot, the first region of the window loaded
    auto open = [&]() {
        pending = s < A.count;
        n = 0;
        const uint8_t *src = blo;
        if (pending) {
            n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
            src = A.in + A.in_off[s];
        }
        for (int32_t k = 4 * lj; k < (int32_t)table_words; k += 4 * G) *(uint4 *)((uint32_t *)hth + k) = make_uint4(0, 0, 0, 0);
        // the launcher sized records and tables from max_len: longer streams are refused
        err = !pending || (uint64_t)n > A.max_len ? EZ_EINVAL : 0;
        live = !err && n >= 4;
        p = live ? src : edge + 16;
        const bool edge_stream = live && (src - kEdgeBefore < blo || src + n + 64 > bhi);
        if (edge_stream) {
            // [64 zero bytes][the stream][64 zero bytes]
            int32_t slot = 0;
            if (lj == 0) slot = (int32_t)atomicAdd(queue - 1, 1u);
            slot = bcast(slot, G * g);
            if (slot >= kEdgeSlots) {  // cannot happen (the batch has at most two edge regions)
                err = EZ_ESTUCK;
                live = false;
                p = edge + 16;
            } else {
                uint8_t *d = edge + 128 + (uint64_t)slot * edge_slot_bytes(A);
                for (int32_t k = lj; k < n + kEdgeBefore + 64; k += G)
                    d[k] = (k >= kEdgeBefore && k < n + kEdgeBefore) ? src[k - kEdgeBefore] : (uint8_t)0;
                p = d + kEdgeBefore;
            }
            __threadfence_block();
        }
        i = done = nrec = 0;
        rec = recs + (pending ? s : 0) * rcap;
        wr.init(p, n, lj, live);
        // the bytes around stream position 0, the candidate of every zero table entry:
        // judged without a load (a load for every lane measured 2.35 against 2.00 ms at C1: the
        // vector-memory path is the parse's busiest)
        z0 = z1 = z2 = V16{0, 0};
        if (live) {
            if constexpr (W40) bytes48(L, p, 0, z0, z1, z2);
            else bytes32(L, p, 0, z0, z1);
            z0.lo = 0;
        }
    };
    open();
    budget += (int64_t)(4 * A.max_len + 64) * S;

    V16 w0{0, 0}, w1{0, 0}, w2{0, 0};  // bytes x-8 .. x+7, x+8 .. x+23 (and x+24 .. x+39) of this lane's x
    for (;;) {
        // groups whose stream ended: its size word, then (PERSIST) the next stream
        if (__builtin_amdgcn_ballot_w64(!live && pending) != 0) {
            if (!live && pending) {
                if (lj == 0) A.out_size[s] = (uint64_t)((EZ_EXP & 32768) ? 0 : nrec) | ((uint64_t)err << 48);
                pending = false;
                if (PERSIST) {
                    uint32_t q = 0;
                    if (lj == 0) q = atomicAdd(queue, 1u);
                    s = (uint64_t)gridDim.x * S + (uint64_t)(uint32_t)bcast((int32_t)q, G * g);
                    open();
                }
            }
            if (PERSIST) budget += (int64_t)(4 * A.max_len + 64) * (__builtin_popcountll(__builtin_amdgcn_ballot_w64(pending)) / G);
        }
        if (__builtin_amdgcn_ballot_w64(live) == 0) {
            if (PERSIST && __builtin_amdgcn_ballot_w64(pending) != 0) continue;
            break;
        }
        if (budget < 0) {
            if (live) err = EZ_ESTUCK;
            live = false;
            continue;
        }
        // the parse, until one of the groups' streams ends (the bookkeeping above stays out of it)
        const uint64_t lm = __builtin_amdgcn_ballot_w64(live);
        do {
        budget--;
        if constexpr (W40) wr.bytes48(i, g, lj, w0, w1, w2);
        else wr.bytes(i, g, lj, w0, w1);
        const int32_t nvalid = n - 3 - i < G ? n - 3 - i : G;
        const int32_t x = i + lj;
        const bool valid = live && lj < nvalid;

        // ---- visit (writer.go:213-217): hash, table, nearest earlier lane with the same hash
        if (prio & 1) __builtin_amdgcn_s_setprio(3);
        const uint32_t h = valid ? ((uint32_t)w0.hi * kHashMul) >> hsh : 0u;
        int32_t cand = 0;
        if (TB == 12) {
            if (valid) cand = (int32_t)lds_mskor12((uint64_t *)hth, h, (uint32_t)x);
        } else if (TB == 16) {
            if (valid) cand = (int32_t)lds_mskor16(hth, h, (uint32_t)x);
        } else {
            const int32_t tv = valid ? (int32_t)hth[h] : 0;
            const int32_t d = PredZ<G - 1>::get(valid ? h + 1 : 0u, 0);
            cand = valid ? (d ? x - d : tv) : 0;
        }
        V16 c0 = z0, c1 = z1, c2 = z2;
        if (cand != 0) {
            if constexpr (W40) bytes48(L, p, cand, c0, c1, c2);
            else if (kFwdCap == 20) bytes28(L, p, cand, c0, c1);
            else bytes32(L, p, cand, c0, c1);
            // bytes before the stream start are the fresh ring's zeros (rare: a branch)
            if (__builtin_expect(cand < 8, 0)) c0.lo &= ~0ull << (8 * (8 - cand));
        }
        if (prio & 1) __builtin_amdgcn_s_setprio(0);

        // ---- capped judgement, writer.go:219-301 (window) and :441-463 (writeRunlen)
        const bool rl = cand >= done && cand < x;
        const uint64_t e0 = w0.hi ^ c0.hi, e1 = w1.lo ^ c1.lo, e2 = w1.hi ^ c1.hi;
        int32_t jf = W40 ? first_diff40(e0, e1, e2, w2.lo ^ c2.lo, w2.hi ^ c2.hi)
                         : (kFwdCap == 20 ? first_diff20(e0, e1, (uint32_t)e2) : first_diff24(e0, e1, e2));
        jf = jf < n - x ? jf : n - x;
        int32_t bl = x - done;
        if (rl) bl = bl < cand ? bl : cand;
        int32_t jb = last_diff8(w0.lo ^ c0.lo);
        jb = jb < bl ? jb : bl;
        const bool zr = rl && c0.hi == 0 && cand + 8 < n;
        const int32_t fw = rl ? jf : (jf < done - cand ? jf : done - cand);
        const bool acc = valid && (zr || fw + jb >= kMinCopyChunk);

        // ---- this lane's action if it is the group's first acceptor
        int32_t lit, nx, dist, ext;
        bool force = false;
        if (zr) {  // writeZeros :407-439
            int32_t zf = W40 ? first_diff40(0, c1.lo, c1.hi, c2.lo, c2.hi)
                             : (kFwdCap == 20 ? first_diff20(0, c1.lo, (uint32_t)c1.hi) : first_diff24(0, c1.lo, c1.hi));
            zf = zf < n - cand ? zf : n - cand;
            int32_t zb = last_diff8(c0.lo);
            zb = zb < cand - done ? zb : cand - done;
            lit = cand - zb;
            nx = cand + zf;
            dist = 0;
            ext = (zf == CAP && n - cand > CAP ? 1 : 0) | (zb == 8 && cand - done > 8 ? 2 : 0);
        } else {  // writeRunlen :441-489 / window match :303-321
            lit = x - jb;
            nx = x + fw;
            dist = x - cand;
            force = rl;
            ext = (jf == CAP && (rl ? n - x : (done - cand < n - x ? done - cand : n - x)) > CAP ? 1 : 0) |
                  (jb == 8 && bl > 8 ? 2 : 0);
        }
        const uint64_t am64 = __builtin_amdgcn_ballot_w64(acc);
        const uint32_t am = (uint32_t)(am64 >> (G * g)) & kGMask;
        const int a = am ? __builtin_ctz(am) : -1;
#if (EZ_EXP & 65536)
        if (live && lj == 0) atomicAdd(&g_lean_hist[a + 1], 1ull);  // (experiment builds: the acceptor lane, -1 none)
#endif
        const bool act = live && a >= 0;
        // the group's next position, whether the acceptor needs an exact extension, and whether it
        // makes the i+1 insert (a window match, writer.go:315-318)
        const bool ins1 = !rl && !zr && x + 1 + 4 <= n;
        const int32_t pack = nx | (ext << 28) | ((int32_t)ins1 << 30);
        // (one ds_bpermute from each group's first acceptor: fewer VALU than four v_readlane + selects)
        const int32_t sel = __builtin_amdgcn_ds_bpermute(4 * (G * g + (a < 0 ? 0 : a)), pack);
        int32_t nxt = sel & 0x0fffffff;
        if (__builtin_amdgcn_ballot_w64(act && ((sel >> 28) & 3) != 0) != 0) {
            // rare: a saturated count; exact lengths by the whole group (as k1_parse)
            // the acceptor's candidate, capped backward count (<= 8) and branch
            const int32_t info = cand | (((zr ? cand : x) - lit) << 16) | ((int32_t)rl << 29) | ((int32_t)zr << 30);
            const int32_t ib = bcast(info, G * g + (a < 0 ? 0 : a));
            const int32_t xa = i + (a < 0 ? 0 : a);
            const int32_t ca = ib & 0xffff;
            const bool rla = (ib >> 29) & 1, zra = (ib >> 30) & 1;
            const int32_t e = (sel >> 28) & 3;
            const bool need = act && e != 0;
            const int mode = zra ? 0 : (rla ? 1 : 2);
            const int32_t fa = zra ? ca : xa;
            const int32_t blim = zra ? ca - done : (rla ? ((xa - done) < ca ? (xa - done) : ca) : xa - done);
            const int32_t flim = zra ? n - ca : (rla ? n - xa : ((done - ca) < n - xa ? done - ca : n - xa));
            int32_t fx, cx;
            gext<G, GWU>(GWU{p}, need && (e & 1), need && (e & 2), g, lj, fa, ca, mode, done, CAP, flim, blim, fx, cx);
            if (need) {
                const int32_t f = (e & 1) ? fx : (sel & 0x0fffffff) - fa;
                const int32_t c = (e & 2) ? cx : ((ib >> 16) & 0xf);
                nxt = fa + f;
                if (lj == a) {
                    lit = fa - c;
                    nx = nxt;
                }
            }
        }
        // ---- table: the visited lanes' positions (the last of a hash wins), then lane a's i+1.
        // Lanes past the acceptor put back what their visit found (visits Go never makes); lane a+1
        // hashed position i+1 itself and is the only lane past a that restores that entry, so it
        // writes i+1 there instead when the acceptor makes the insert (prio bit 2; the acceptor
        // still does it when a is the group's last lane)
        const bool ins_next = TB != 0 && (prio & 4) && a >= 0 && a < G - 1 && ((sel >> 30) & 1);
        if (TB == 12) {
            if (valid && a >= 0 && lj > a && cand <= i + a) lds_put12((uint64_t *)hth, h, (uint32_t)(ins_next && lj == a + 1 ? x : cand));
        } else if (TB == 16) {
            if (valid && a >= 0 && lj > a && cand <= i + a) hth[h] = (uint16_t)(ins_next && lj == a + 1 ? x : cand);
        } else {
            if (valid && (a < 0 || lj <= a)) hth[h] = (uint16_t)x;
        }
        if (act && lj == a && !ins_next) {
            if (ins1) {
                const uint32_t h1 = ((uint32_t)(w0.hi >> 8) * kHashMul) >> hsh;
                if (TB == 12) lds_put12((uint64_t *)hth, h1, (uint32_t)(x + 1));
                else hth[h1] = (uint16_t)(x + 1);
            }
        }
        // the record, stored after the next region's load is issued (a region switch waits for every
        // vector-memory operation before it, stores included)
        const bool st_rec = act && lj == a;
        const uint64_t rv = rec_pack(lit, nx - lit, dist, force);
        const uint32_t rat = (uint32_t)nrec;
        const bool rec_room = (uint32_t)nrec < rcap32;
        if (act) {
            if (!rec_room) { err = EZ_ESTUCK; live = false; }
            nrec++;
            i = done = nxt;
        } else if (live) {
            i += nvalid;
        }
        if (live && (err || i + 4 > n)) live = false;
        wr.advance(p, i, lj, live);  // the next window's region
        __builtin_amdgcn_sched_barrier(0);
        if (st_rec) {
#if !(EZ_EXP & 32768)
            if (rec_room) __builtin_nontemporal_store(rv, rec + rat);
#else  // (timing builds: the records' traffic without their lines -- k1_emit then sees none)
            __builtin_nontemporal_store(rv, rec + (uint32_t)(nrec & 1));
#endif
        }
        } while (__builtin_amdgcn_ballot_w64(live) == lm && budget >= 0);
    }
}

// ---------------------------------------------------------------- K1L: long fresh streams
// k1_lean's parse for Writes longer than half the block (C4's gradient buckets, where K1x's rounds
// leave dense streams such as C4s to it): the same window, DPP predecessor search and capped
// judgement, plus the window's ring semantics of writer.go -- far skip (:219-221), the cut branch of
// writeRunlen (:464-473), trim 1 (:280-286) and the ring image before the window, block[y & mask] =
// stream byte y + bs for y < w.pos - bs -- a u32 table, bounds-checked loads (any
// stream of a batch, no edge slots), and 16-byte records.  It resumes the streams K1x hands over
// (spec state: position, pending literal, output so far, table).
struct WideRec {
    uint32_t lit_end, clen, dist, flags;  // flags bit 0: force the literal (writeRunlen, A.6)
};

// a dword at w, 0 for bytes outside the batch [lo, hi)
__device__ __forceinline__ uint32_t dw_chk(const uint8_t *w, const uint8_t *lo, const uint8_t *hi) {
    if (w >= lo && w + 4 <= hi) return *(const uint32_t *)w;
    uint32_t v = 0;
    for (int t = 0; t < 4; t++)
        if (w + t >= lo && w + t < hi) v |= (uint32_t)w[t] << (8 * t);
    return v;
}
// K1L's window bytes (x-8 .. x+39 of each lane's x) from a 128-byte region held across windows
// with the next one in flight (WinRoll's scheme with bounds-checked loads: any stream of any batch)
struct WinRollL {
    uint32_t c0, c1, f0, f1;  // this lane's dwords 2k, 2k+1 of the current and the prefetched region
    int32_t cb, fb, pm;       // region starts relative to p (4-byte aligned addresses); p & 3
    __device__ __forceinline__ int32_t floor4(int32_t y) const { return y - ((pm + y) & 3); }
    __device__ __forceinline__ static void ld(const uint8_t *p, int32_t b, int lj, const uint8_t *lo, const uint8_t *hi,
                                              uint32_t &d0, uint32_t &d1) {
        const uint8_t *a = p + b + 8 * lj;
        if (a >= lo && a + 8 <= hi) {
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            typedef const __attribute__((address_space(1))) u32x2 *gu64p;
            const u32x2 v = *(gu64p)a;
            d0 = v.x;
            d1 = v.y;
        } else {
            d0 = dw_chk(a, lo, hi);
            d1 = dw_chk(a + 4, lo, hi);
        }
    }
    // (as WinRoll: c only from moves after f's load, so the prefetch lands in f's registers and no wait
    // for it is put at the loop's head)
    __device__ __forceinline__ void init(const uint8_t *p, int32_t i, int lj, bool live, const uint8_t *lo, const uint8_t *hi) {
        pm = (int32_t)((uintptr_t)p & 3);
        cb = floor4(i - 8);
        fb = cb + 64;
        f0 = f1 = 0;
        if (live) ld(p, cb, lj, lo, hi, f0, f1);
        asm volatile("v_mov_b32 %0, %1" : "=v"(c0) : "v"(f0));
        asm volatile("v_mov_b32 %0, %1" : "=v"(c1) : "v"(f1));
        if (live) ld(p, fb, lj, lo, hi, f0, f1);
    }
    // the region for the window at i (group-uniform: 0 <= i - 8 - cb <= 64), after this window's gathers
    __device__ __forceinline__ void advance(const uint8_t *p, int32_t i, int lj, bool live, const uint8_t *lo, const uint8_t *hi) {
        const int32_t y = i - 8;
        if (live && !(y >= cb && y - cb <= 64)) {
            if (!(y >= fb && y - fb <= 64)) {  // a long jump (or back: the cut branch): loaded on the chain
                fb = floor4(y);
                ld(p, fb, lj, lo, hi, f0, f1);
            }
            cb = fb;
            asm volatile("v_mov_b32 %0, %1" : "=v"(c0) : "v"(f0));
            asm volatile("v_mov_b32 %0, %1" : "=v"(c1) : "v"(f1));
            fb = cb + 64;
            ld(p, fb, lj, lo, hi, f0, f1);
        }
    }
    __device__ __forceinline__ void bytes48(int32_t i, int g, int lj, V16 &w0, V16 &w1, V16 &w2) const {
        const uint32_t o = (uint32_t)(i - 8 - cb + lj), q = o >> 2, r = o & 3;  // o <= 79: q >> 1 <= 9
        const int src = 4 * (16 * g + (int)(q >> 1));
        uint32_t e[14];
#pragma unroll
        for (int t = 0; t < 7; t++) {
            e[2 * t] = (uint32_t)__builtin_amdgcn_ds_bpermute(src + 4 * t, (int)c0);
            e[2 * t + 1] = (uint32_t)__builtin_amdgcn_ds_bpermute(src + 4 * t, (int)c1);
        }
        const uint32_t m = 0u - (q & 1);
        uint32_t d[13];
#pragma unroll
        for (int t = 0; t < 13; t++) d[t] = (e[t + 1] & m) | (e[t] & ~m);
        uint32_t b[12];
#pragma unroll
        for (int t = 0; t < 12; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
        w0 = V16{(uint64_t)b[0] | ((uint64_t)b[1] << 32), (uint64_t)b[2] | ((uint64_t)b[3] << 32)};
        w1 = V16{(uint64_t)b[4] | ((uint64_t)b[5] << 32), (uint64_t)b[6] | ((uint64_t)b[7] << 32)};
        w2 = V16{(uint64_t)b[8] | ((uint64_t)b[9] << 32), (uint64_t)b[10] | ((uint64_t)b[11] << 32)};
    }
};
// WinRollL with the current region in LDS (as WinLds): the group's buffer holds stream bytes
// [cb, cb + 128); a window's 48 bytes are thirteen aligned dword reads and twelve v_alignbyte
struct WinLdsL {
    uint32_t f0, f1;  // this lane's dwords of the prefetched region
    int32_t cb, fb, pm;
    uint8_t *wl;  // the group's buffer (LDS)
    __device__ __forceinline__ int32_t floor4(int32_t y) const { return y - ((pm + y) & 3); }
    __device__ __forceinline__ void put(int lj) const { *(uint64_t *)(wl + 8 * lj) = (uint64_t)f0 | ((uint64_t)f1 << 32); }
    __device__ __forceinline__ void init(const uint8_t *p, int32_t i, int lj, bool live, const uint8_t *lo, const uint8_t *hi) {
        pm = (int32_t)((uintptr_t)p & 3);
        cb = floor4(i - 8);
        fb = cb + 64;
        f0 = f1 = 0;
        if (live) WinRollL::ld(p, cb, lj, lo, hi, f0, f1);
        put(lj);
        if (live) WinRollL::ld(p, fb, lj, lo, hi, f0, f1);
    }
    __device__ __forceinline__ void advance(const uint8_t *p, int32_t i, int lj, bool live, const uint8_t *lo, const uint8_t *hi) {
        const int32_t y = i - 8;
        if (live && !(y >= cb && y - cb <= 64)) {
            if (!(y >= fb && y - fb <= 64)) {  // a long jump (or back: the cut branch): loaded on the chain
                fb = floor4(y);
                WinRollL::ld(p, fb, lj, lo, hi, f0, f1);
            }
            cb = fb;
            put(lj);
            fb = cb + 64;
            WinRollL::ld(p, fb, lj, lo, hi, f0, f1);
        }
    }
    __device__ __forceinline__ void bytes48(int32_t i, int g, int lj, V16 &w0, V16 &w1, V16 &w2) const {
        const uint32_t o = (uint32_t)(i - 8 - cb + lj), r = o & 3;  // o <= 79
        const uint32_t *q = (const uint32_t *)(wl + (o & ~3u));
        uint32_t d[13];
#pragma unroll
        for (int t = 0; t < 13; t++) d[t] = q[t];
        uint32_t b[12];
#pragma unroll
        for (int t = 0; t < 12; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
        w0 = V16{(uint64_t)b[0] | ((uint64_t)b[1] << 32), (uint64_t)b[2] | ((uint64_t)b[3] << 32)};
        w1 = V16{(uint64_t)b[4] | ((uint64_t)b[5] << 32), (uint64_t)b[6] | ((uint64_t)b[7] << 32)};
        w2 = V16{(uint64_t)b[8] | ((uint64_t)b[9] << 32), (uint64_t)b[10] | ((uint64_t)b[11] << 32)};
    }
};
// bytes y-8 .. y+39 (bytes outside the batch read 0)
__device__ __forceinline__ void bytes48_chk(const uint8_t *p, int32_t y, V16 &c0, V16 &c1, V16 &c2, const uint8_t *lo,
                                            const uint8_t *hi) {
    const uintptr_t a = (uintptr_t)(p + y - 8);
    const uint8_t *w = (const uint8_t *)(a & ~(uintptr_t)3);
    const uint32_t r = (uint32_t)(a & 3);
    uint32_t d[13];
    if (w >= lo && w + 52 <= hi) {
        const LeanIn L;
        const uint4 q0 = L.dw4(w), q1 = L.dw4(w + 16), q2 = L.dw4(w + 32);
        const uint32_t q3 = L.dw(w + 48);
        d[0] = q0.x, d[1] = q0.y, d[2] = q0.z, d[3] = q0.w, d[4] = q1.x, d[5] = q1.y, d[6] = q1.z, d[7] = q1.w;
        d[8] = q2.x, d[9] = q2.y, d[10] = q2.z, d[11] = q2.w, d[12] = q3;
    } else {
        for (int t = 0; t < 13; t++) d[t] = dw_chk(w + 4 * t, lo, hi);
    }
    uint32_t b[12];
#pragma unroll
    for (int t = 0; t < 12; t++) b[t] = __builtin_amdgcn_alignbyte(d[t + 1], d[t], r);
    c0 = V16{(uint64_t)b[0] | ((uint64_t)b[1] << 32), (uint64_t)b[2] | ((uint64_t)b[3] << 32)};
    c1 = V16{(uint64_t)b[4] | ((uint64_t)b[5] << 32), (uint64_t)b[6] | ((uint64_t)b[7] << 32)};
    c2 = V16{(uint64_t)b[8] | ((uint64_t)b[9] << 32), (uint64_t)b[10] | ((uint64_t)b[11] << 32)};
}
// 16 bytes from y of the window's ring image at w.pos = done (bytes y >= done: 0, capped away by
// trim 2; y < done - bs: stream byte y + bs; before the stream: 0)
template <class SRC>
__device__ __forceinline__ V16 ring16(const SRC &P, int32_t y, int32_t done, int64_t bs) {
    uint64_t lo, hi;
    P.around(y + 8, lo, hi);
    V16 v = keep_low16(V16{lo, hi}, done - y);
    const int64_t edge = (int64_t)done - bs;
    if ((int64_t)y < edge) {
        P.around((int32_t)((int64_t)y + bs + 8), lo, hi);
        const int32_t k = (int32_t)(edge - y);  // bytes 0 .. k-1 lie before the window
        const V16 m = keep_low16(V16{~0ull, ~0ull}, k);
        v = V16{(v.lo & ~m.lo) | (lo & m.lo), (v.hi & ~m.hi) | (hi & m.hi)};
    }
    return v;
}
// gext with the long window's ring image on the source side (mode 2: ring16; 0 zeros; 1 stream)
template <int G, class SRC>
__device__ __forceinline__ void gext_long(const SRC &P, bool runf, bool runb, int g, int lj, int32_t a, int32_t b, int mode,
                                          int32_t done, int64_t bs, int32_t fromf, int32_t limf, int32_t limb, int32_t &resf,
                                          int32_t &resb) {
    constexpr int H = G / 2;
    constexpr uint32_t kHalf = (1u << H) - 1;
    const bool fw = lj < H;
    const int t = lj % H;
    resf = fromf < limf ? fromf : limf;
    resb = 8 < limb ? 8 : limb;
    bool gof = runf && fromf < limf, gob = runb && 8 < limb;
    int32_t basef = fromf, baseb = 8;
    while (__ballot(gof || gob) != 0) {
        const bool mine = fw ? gof : gob;
        const int32_t lim = fw ? limf : limb;
        const int32_t k = (fw ? basef : baseb) + 16 * t;
        int32_t mb = 16;
        if (mine) {
            if (k < lim) {
                const int32_t ya = fw ? a + k : a - k - 16, yb = fw ? b + k : b - k - 16;
                uint64_t alo, ahi;
                P.around(ya + 8, alo, ahi);
                V16 vb{0, 0};
                if (mode == 1) P.around(yb + 8, vb.lo, vb.hi);
                else if (mode == 2) vb = ring16(P, yb, done, bs);
                const uint64_t dl = alo ^ vb.lo, dh = ahi ^ vb.hi;
                if (fw) mb = dl ? (int32_t)(__builtin_ctzll(dl) >> 3) : (dh ? 8 + (int32_t)(__builtin_ctzll(dh) >> 3) : 16);
                else mb = dh ? (int32_t)(__builtin_clzll(dh) >> 3) : (dl ? 8 + (int32_t)(__builtin_clzll(dl) >> 3) : 16);
                if (mb > lim - k) mb = lim - k;
            } else {
                mb = 0;
            }
        }
        const uint32_t bad = gball<G>(mine && mb < 16, g);
        const uint32_t bf = bad & kHalf, bb = bad >> H;
        const int lf = bf ? __builtin_ctz(bf) : 0, lb = bb ? __builtin_ctz(bb) : 0;
        const int32_t mbf = bcast(mb, G * g + lf), mbb = bcast(mb, G * g + H + lb);
        if (gof) {
            if (bf) {
                resf = basef + 16 * lf + mbf;
                resf = resf < limf ? resf : limf;
                gof = false;
            } else {
                basef += 16 * H;
                if (basef >= limf) { resf = limf; gof = false; }
            }
        }
        if (gob) {
            if (bb) {
                resb = baseb + 16 * lb + mbb;
                resb = resb < limb ? resb : limb;
                gob = false;
            } else {
                baseb += 16 * H;
                if (baseb >= limb) { resb = limb; gob = false; }
            }
        }
    }
}

// The history a window match compares against, as a linear byte view (positions relative to the
// parse's p; ring16 turns it into the ring image).  FreshSrc: a fresh Writer, nothing before p (the
// zero ring).  RingSrc: a Writer handle's Write at stream position start: the bytes before p are the
// handle's ring as the Write found it (block[(start + y) & mask]; zeros where the stream
// has not reached yet), p's own from 0 on.
struct FreshSrc : GW {
    __device__ __forceinline__ void bytes48(int32_t cand, V16 &c0, V16 &c1, V16 &c2) const {
        bytes48_chk(p, cand, c0, c1, c2, blo, bhi);
        c0.lo &= cand >= 8 ? ~0ull : (cand <= 0 ? 0ull : ~0ull << (8 * (8 - cand)));  // before the stream: zeros
    }
};
struct RingSrc {
    const uint8_t *p, *blo, *bhi;  // the Write (blo = p, bhi = p + n)
    const uint8_t *ring;
    int64_t start;
    uint32_t mask;
    __device__ __forceinline__ V16 ring_at(int32_t y) const {  // 16 ring bytes of positions y .. y+15 (< 0)
        const uint32_t r = (uint32_t)((start + y) & mask);
        if (r + 16 <= mask + 1) return ld16v(ring + r);
        V16 v{0, 0};
        for (int t = 0; t < 16; t++) {
            const uint64_t c = ring[(r + t) & mask];
            if (t < 8) v.lo |= c << (8 * t);
            else v.hi |= c << (8 * (t - 8));
        }
        return v;
    }
    __device__ __forceinline__ void around(int32_t y, uint64_t &before, uint64_t &from) const {
        V16 v;
        if (y - 8 >= 0) {
            const uint8_t *a = p + (y - 8);
            v = a + 16 <= bhi ? ld16v(a) : ld_clamped(a, blo, bhi);  // (past the Write: 0)
        } else if (y + 8 <= 0) {
            v = ring_at(y - 8);
        } else {  // across the Write's start: the ring's bytes, then p's
            const V16 r = ring_at(y - 8);
            const uint8_t *a = p;
            const V16 q = a + 16 <= bhi ? ld16v(a) : ld_clamped(a, blo, bhi);
            const uint32_t k = (uint32_t)(8 - y);  // ring bytes (1 .. 15)
            const V16 qs = shl16(q, k), m = keep_low16(V16{~0ull, ~0ull}, (int32_t)k);
            v = V16{(r.lo & m.lo) | (qs.lo & ~m.lo), (r.hi & m.hi) | (qs.hi & ~m.hi)};
        }
        before = v.lo;
        from = v.hi;
    }
    __device__ __forceinline__ void bytes48(int32_t cand, V16 &c0, V16 &c1, V16 &c2) const {
        around(cand, c0.lo, c0.hi);
        around(cand + 16, c1.lo, c1.hi);
        around(cand + 32, c2.lo, c2.hi);
    }
};

// LdsSrc: RingSrc with the Write and the ring's last bytes before it staged in LDS (a handle's Write of
// at most kLdsWrite bytes): lds + kLdsRing + y holds position y for -rl <= y < n + 64 (zeros past
// the Write); the window's bytes and the candidates' come from there, anything else from RingSrc.
constexpr int32_t kLdsRing = 32768, kLdsWrite = 49152;
static_assert(kLdsWrite == (int32_t)kHandleLdsWrite, "the handle path's zero-copy bound is K1L's LDS-staged Write");
typedef uint64_t __attribute__((aligned(1))) u64_ua;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
struct LdsSrc {
    const uint8_t *lds;
    int32_t rl, n;
    RingSrc g;  // (the window's bytes come from here too: WindowFromSrc)
    __device__ __forceinline__ void around(int32_t y, uint64_t &before, uint64_t &from) const {
        if (y - 8 >= -rl && y + 8 <= n + 64) {
            const uint8_t *q = lds + kLdsRing + (y - 8);
            before = *(const u64_ua *)q;
            from = *(const u64_ua *)(q + 8);
        } else {
            g.around(y, before, from);
        }
    }
    __device__ __forceinline__ static V16 lds16(const uint8_t *q) { return V16{*(const u64_ua *)q, *(const u64_ua *)(q + 8)}; }
    __device__ __forceinline__ void bytes48(int32_t cand, V16 &c0, V16 &c1, V16 &c2) const {
        if (cand - 8 >= -rl && cand + 40 <= n + 64) {  // one check for the 48 bytes
            const uint8_t *q = lds + kLdsRing + (cand - 8);
            c0 = lds16(q);
            c1 = lds16(q + 16);
            c2 = lds16(q + 32);
        } else {
            g.around(cand, c0.lo, c0.hi);
            g.around(cand + 16, c1.lo, c1.hi);
            g.around(cand + 32, c2.lo, c2.hi);
        }
    }
    // the window's bytes x-8 .. x+39 (0 <= x < n: always staged)
    __device__ __forceinline__ void window48(int32_t x, V16 &w0, V16 &w1, V16 &w2) const {
        const uint8_t *q = lds + kLdsRing + (x - 8);
        w0 = lds16(q);
        w1 = lds16(q + 16);
        w2 = lds16(q + 32);
    }
};
template <class SRC>
struct WindowFromSrc {
    static constexpr bool value = false;
};
template <>
struct WindowFromSrc<LdsSrc> {
    static constexpr bool value = true;
};

// the parse of one stream by a 16-lane group from (i, done) with the table in htw.  The capped
// judgement compares 40 bytes forward (k1_lean: 24): the long parse is a latency chain (few streams
// per SIMD), and at C2 one accepted copy in nine is 24 - 39 bytes long, whose exact extension
// (gext_long) is a group-wide round trip that every stream of the wave waits for.
constexpr int32_t kLCap = 40;
// K1c's side outputs of a chunk's speculative parse (see kc_parse); NoEv: none (K1L)
struct NoEv {
    static constexpr bool kOn = false;
    int32_t stop, keep;
    uint32_t cnt;
    __device__ __forceinline__ void visit(int32_t, int32_t, bool, bool, int, int, int32_t, bool, int32_t) {}
};
template <class SRC, bool LW = false, class EV = NoEv>
__device__ __forceinline__ void long_loop(const SRC &P, const uint8_t *p, int32_t n, int32_t i, int32_t done, int64_t bs, int lj,
                                          int g, uint32_t *htw, uint32_t hsh, uint4 *rec, uint64_t rcap, const uint8_t *blo,
                                          const uint8_t *bhi, int32_t &nrec_out, int &err, uint8_t *wl = nullptr, EV *ev = nullptr) {
    constexpr int G = 16;
    int32_t nrec = 0;
    bool live = !err && i + 4 <= n && (!EV::kOn || i < ev->stop);
    int64_t guard = 4 * (int64_t)n + 64;
    V16 w0{0, 0}, w1{0, 0}, w2{0, 0};  // bytes x-8 .. x+7, x+8 .. x+23, x+24 .. x+39 of this lane's position x
    typename std::conditional<LW, WinLdsL, WinRollL>::type wr;
    if constexpr (LW) wr.wl = wl;
    if (!WindowFromSrc<SRC>::value) wr.init(p, i, lj, live, blo, bhi);
    constexpr bool kWinSrc = WindowFromSrc<SRC>::value;
#if (EZ_EXP & 4)
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_t = __builtin_amdgcn_s_memtime(), prof_it = 0, prof_acc = 0, prof_ef = 0, prof_eb = 0;
#endif
    while (__ballot(live) != 0) {
#if (EZ_EXP & 4)
        prof_it++;
#endif
        if constexpr (kWinSrc) {
            P.window48(live ? i + lj : 0, w0, w1, w2);
        } else {
            wr.bytes48(i, g, lj, w0, w1, w2);
        }
        EZ_PROF_MARK(0);
        if (live && --guard < 0) { err = EZ_ESTUCK; live = false; }
        const int32_t nvalid = n - 3 - i < G ? n - 3 - i : G;
        const int32_t x = i + lj;
        const bool valid = live && lj < nvalid;

        // ---- visit (writer.go:213-217): hash, table, nearest earlier lane with the same hash
        const uint32_t h = valid ? ((uint32_t)w0.hi * kHashMul) >> hsh : 0u;
        const int32_t tv = valid ? (int32_t)htw[h] : 0;
        const int32_t d = PredZ<G - 1>::get(valid ? h + 1 : 0u, 0);
        const int32_t cand = valid ? (d ? x - d : tv) : 0;
        const bool rl = cand >= done && cand < x;
        const bool far = !rl && (int64_t)done - cand > bs;  // writer.go:221-224
        EZ_PROF_MARK(1);
        V16 c0{0, 0}, c1{0, 0}, c2{0, 0};
        if (valid && !far) {
            P.bytes48(cand, c0, c1, c2);
            if (!rl && (int64_t)cand - 8 < (int64_t)done - bs) c0.lo = ring16(P, cand - 8, done, bs).lo;  // rare
        }
        EZ_PROF_MARK(2);

        // ---- capped judgement, writer.go:219-301 (window) and :441-473 (writeRunlen, cut)
        int32_t jf = first_diff40(w0.hi ^ c0.hi, w1.lo ^ c1.lo, w1.hi ^ c1.hi, w2.lo ^ c2.lo, w2.hi ^ c2.hi);
        jf = jf < n - x ? jf : n - x;
        int32_t bl = x - done;
        if (rl) bl = bl < cand ? bl : cand;
        int32_t jb = last_diff8(w0.lo ^ c0.lo);
        jb = jb < bl ? jb : bl;
        const bool zr = rl && c0.hi == 0 && cand + 8 < n;
        const int32_t fw = rl ? jf : (jf < done - cand ? jf : done - cand);
        const int64_t t1 = bs - (int64_t)(x - cand);  // trim 1: the copy ends within bs of x
        const int32_t len = rl ? fw + jb : (int32_t)((int64_t)(fw + jb) < t1 ? (int64_t)(fw + jb) : (t1 < 0 ? -1 : t1));
        const bool acc = valid && !far && (zr || len >= kMinCopyChunk);
        const bool cut = rl && !zr && (int64_t)(x - cand) >= bs - 8;

        // ---- this lane's action if it is the group's first acceptor
        int32_t lit, nx, dist, ext;
        bool force = false;
        if (zr) {  // writeZeros :407-439
            int32_t zf = first_diff40(0, c1.lo, c1.hi, c2.lo, c2.hi);
            zf = zf < n - cand ? zf : n - cand;
            int32_t zb = last_diff8(c0.lo);
            zb = zb < cand - done ? zb : cand - done;
            lit = cand - zb;
            nx = cand + zf;
            dist = 0;
            ext = (zf == kLCap && n - cand > kLCap ? 1 : 0) | (zb == 8 && cand - done > 8 ? 2 : 0);
        } else if (cut) {  // the cut branch: a literal to done + i - st, no copy (writer.go:464-473)
            lit = done + (x - cand);
            nx = lit;
            dist = 0;
            ext = 0;
        } else {  // writeRunlen :441-489 / window match :303-321
            lit = x - jb;
            nx = lit + len;
            dist = x - cand;
            force = rl;
            const int32_t room = rl ? n - x : (done - cand < n - x ? done - cand : n - x);
            ext = (jf == kLCap && room > kLCap && (rl || (int64_t)(jb + kLCap) < t1) ? 1 : 0) | (jb == 8 && bl > 8 ? 2 : 0);
        }
        const uint64_t am64 = __ballot(acc);
        const uint32_t am = (uint32_t)(am64 >> (G * g)) & 0xffffu;
        const int a = am ? __builtin_ctz(am) : -1;
        const bool act = live && a >= 0;
        const int al = G * g + (a < 0 ? 0 : a);
        int32_t nxt = bcast(nx, al);
        const int32_t ea = bcast(ext, al);
        EZ_PROF_MARK(3);
#if (EZ_EXP & 4)
        prof_acc += act ? 1 : 0;
        prof_ef += act && (ea & 1) ? 1 : 0;
        prof_eb += act && (ea & 2) ? 1 : 0;
#endif
        if (__ballot(act && ea != 0) != 0) {
            // rare: a saturated count; exact lengths by the whole group
            const int32_t xa = i + (a < 0 ? 0 : a);
            const int32_t ca = bcast(cand, al), jba = bcast(jb, al), fwa = bcast(zr ? nx - cand : fw, al);
            const int32_t fl = bcast((int32_t)rl | ((int32_t)zr << 1), al);
            const bool rla = fl & 1, zra = (fl >> 1) & 1;
            const bool need = act && ea != 0;
            const int mode = zra ? 0 : (rla ? 1 : 2);
            const int32_t fa = zra ? ca : xa;
            const int32_t blim = zra ? ca - done : (rla ? ((xa - done) < ca ? (xa - done) : ca) : xa - done);
            const int32_t flim = zra ? n - ca : (rla ? n - xa : ((done - ca) < n - xa ? done - ca : n - xa));
            int32_t fx, cx;
            gext_long<G, SRC>(P, need && (ea & 1), need && (ea & 2), g, lj, fa, ca, mode, done, bs, kLCap, flim, blim, fx, cx);
            if (need) {
                int32_t f = (ea & 1) ? fx : fwa;
                const int32_t c = (ea & 2) ? cx : (zra ? fa - bcast(lit, al) : jba);
                if (!zra && !rla) {  // trim 1 on the exact lengths
                    const int64_t t1a = bs - (int64_t)(xa - ca);
                    if ((int64_t)(f + c) > t1a) f = (int32_t)(t1a - c);
                }
                nxt = fa + f;
                if (lj == a) {
                    lit = fa - c;
                    nx = nxt;
                }
            }
        }
        EZ_PROF_MARK(4);
        // K1c: the window's visits (and the i+1 insert) into the chunk's log, in the parse's order
        bool keep = true;
        uint32_t logi = 0;
        if constexpr (EV::kOn) {
            const bool insb = bcast((int32_t)(act && lj == a && !rl && !zr && x + 1 + 4 <= n), al) != 0;
            ev->visit(x, cand, valid && (a < 0 || lj <= a), act && lj == a, g, lj, i, insb, i + (a < 0 ? 0 : a) + 1);
            logi = ev->cnt;
            keep = nxt >= ev->keep;
        }
        // ---- table: the visited lanes' positions (the last of a hash wins), then lane a's i+1
        if (valid && (a < 0 || lj <= a)) htw[h] = (uint32_t)x;
        if (act && lj == a) {
            if (!rl && !zr && x + 1 + 4 <= n) htw[((uint32_t)(w0.hi >> 8) * kHashMul) >> hsh] = (uint32_t)(x + 1);
        }
        // the record, stored after the next region's load is issued (as in lean_loop)
        const bool st_rec = act && lj == a && keep && (uint64_t)nrec < rcap;
        // (K1c: the log's length after this window in the flags word's bits 1..31; k1_emit reads bit 0)
        const u32x4 recv{(uint32_t)lit, (uint32_t)(nx - lit), (uint32_t)dist, (force ? 1u : 0u) | (logi << 1)};
        u32x4 *const recp = (u32x4 *)(rec + nrec);
        if (act) {
            if (keep) {
                if ((uint64_t)nrec >= rcap) { err = EZ_ESTUCK; live = false; }
                nrec++;
            }
            i = done = nxt;
        } else if (live) {
            i += nvalid;
        }
        if (live && (err || i + 4 > n || (EV::kOn && i >= ev->stop))) live = false;
        if (!kWinSrc) wr.advance(p, i, lj, live, blo, bhi);  // the next window's region
        __builtin_amdgcn_sched_barrier(0);
        if (st_rec) __builtin_nontemporal_store(recv, recp);
        EZ_PROF_MARK(5);
    }
#if (EZ_EXP & 4)
    if (blockIdx.x < 8 && lj == 0)
        printf("lprof blk %u g %d it %llu acc %llu ef %llu eb %llu: window %llu visit %llu cload %llu judge %llu ext %llu upd %llu\n", blockIdx.x, g,
               (unsigned long long)prof_it, (unsigned long long)prof_acc, (unsigned long long)prof_ef, (unsigned long long)prof_eb, (unsigned long long)prof[0], (unsigned long long)prof[1],
               (unsigned long long)prof[2], (unsigned long long)prof[3], (unsigned long long)prof[4], (unsigned long long)prof[5]);
#endif
    nrec_out = nrec;
}

// a group of 16 lanes per stream, 4 streams per wave; spec_mode 2: K1x's streams resume
// spw: streams per wave (1, 2 or 4; the other lane groups idle, with no table): a batch of few long
// streams runs more waves per SIMD, each a lone latency chain, instead of fewer waves of 4 streams
// only (K1c's fallback): the streams whose only[ostride s] is nonzero, the others untouched (nullptr: all)
template <bool LW = false>
__global__ __launch_bounds__(64) void k1_long(CompressArgs A, uint32_t table_words, uint4 *recs, uint64_t rcap, uint32_t spw,
                                              const uint32_t *only, uint32_t ostride) {
    constexpr int G = 16;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / G, lj = lane % G;
    const bool grp = (uint32_t)g < spw;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(A.hs - 1)));
    uint32_t *htw = (uint32_t *)smem + (uint32_t)(grp ? g : 0) * table_words;  // (an idle group never touches it)
    const uint64_t s = (uint64_t)blockIdx.x * spw + (uint32_t)g;
    const bool spec = A.spec_mode != 0;
    bool have = grp && s < A.count;
    if (have && spec && A.spec[s].flags != 0) have = false;  // finished by K1x
    if (have && only && only[(uint64_t)ostride * s] == 0) have = false;  // K1c took it
    const uint8_t *blo = A.in, *bhi = A.in + A.in_off[A.count];
    int32_t n = 0, i = 0, done = 0;
    const uint8_t *p = blo;
    if (have) {
        n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        p = A.in + A.in_off[s];
        if (spec) {
            i = (int32_t)A.spec[s].from;
            done = (int32_t)A.spec[s].done;
        }
    }
    if (grp)
        for (int32_t k = lj; k < (int32_t)A.hs; k += G) htw[k] = have && spec ? A.spec_tab[s * (uint64_t)A.hs + k] : 0u;
    int err = have && (uint64_t)n > A.max_len ? EZ_EINVAL : (have ? 0 : EZ_EINVAL);
    int32_t nrec = 0;
    // (LW: the groups' window buffers after the tables)
    uint8_t *wl = smem + (size_t)spw * table_words * 4 + (size_t)g * kWinLdsBytes;  // (idle groups too: their own buffers)
    long_loop<FreshSrc, LW>(FreshSrc{{p, blo, bhi}}, p, n, i, done, A.bs, lj, g, htw, hsh, recs + (have ? s * rcap : 0), rcap, blo, bhi,
                            nrec, err, wl);
    if (have && lj == 0) A.out_size[s] = (uint64_t)nrec | ((uint64_t)err << 48);
}

// ---------------------------------------------------------------- K1c: chunk-parallel long streams
// K1L runs one 16-lane group per stream: a batch of few long streams (C2's 4,096 x 256 KiB: one wave
// per SIMD; C4s's 64 streams after K1x) leaves the chip waiting on a few dependent chains.  K1c cuts
// each stream into chunks of C positions and parses all of them at once, then proves the result is
// Go's parse (writer.go:206-330) or hands the stream to K1L:
//   kc_parse   chunk k's speculative parse (long_loop): from W positions before its start b_k with
//              done there and a zero table, to O positions past the next chunk's start.  It keeps the
//              records ending at or after b_k and logs its visits in the order it makes them -- the
//              position and the table entry it read (bit 31: it accepted there), an i+1 insert as a
//              marker -- each record carrying the log's length after its window.  Chunk 0 starts where
//              the stream does (or at K1x's state), so its parse is Go's up to where it stops.
//   kc_stitch  per stream: the path is chunk 0's parse up to the first copy end it shares with chunk
//              1's parse (i == done == that position in both: from there the two make the same
//              choices as long as they read the same table entries), then chunk 1's, and so on (past
//              a copy over the next chunk's start: the first later chunk that ends a copy at one of
//              this one's copy ends).  A segment = (chunk, its records and its log range).
//   kc_gather  the path's records into the stream's record slot (K1L's layout, for k1_emit<true>).
//   kc_v1/v2   every logged read against the table of the stitched path itself (Go's table at that
//              visit: the last position of that hash visited or inserted before it in the path's
//              order; 0 at the stream start, K1x's table after its rounds): kc_v1 per segment with an
//              LDS table, kc_v2 per hash across segments for each segment's first read of it.  A visit
//              that read another entry is judged again with the right one and the path's pending
//              literal start (kc_accepts, long_loop's judgement): still a reject, the path stands (the
//              entry read decides only that visit; the table holds positions, not what was read); an
//              accept, or an acceptor that read another entry, fails the stream.
// Every choice of the stitched path is then Go's choice from Go's state, so it is Go's parse.
// Passes: a chunk's zero table at its warm-up misses entries older than the warm-up, and a visit that
// would have accepted with one fails the stream; the next pass parses again each chunk whose segment
// failed, from that segment's start (i == done there) with the stitched path's table at that point
// (kc_v2 writes both), which is Go's when the path before it is -- so each pass proves at least the
// first failed segment, and in practice most of them (the others keep their parses; every segment is
// checked again against the new path).  Streams still
// failed after the last pass, or that cannot be stitched (a chunk's error or log overflow, no shared
// copy end), take K1L from their start (k1_long's `only`).
struct KcBufs {
    uint4 *crec;      // per chunk: rcap_c records (K1L's; flags word bit 1..: the log length)
    uint2 *log;       // per chunk: logcap visits {position, entry read | accept << 31, or kKcIns}
    uint4 *meta;      // per chunk: {records kept, flags kKc*, log length, 0}
    uint32_t *seg;    // per stream: kmax segments of 8 words {chunk, from, to, rec lo, rec hi, rec dst, log lo, log hi}
    uint32_t *sinfo;  // per stream: kKcInfo words {segments, fail, chunks, first failed segment, pass}
    uint32_t *ft;     // per segment: first read's log index [hs], last position [hs]
    int32_t *cstart;  // per chunk: the next pass's start (a segment's start; -1: the warm-up start)
    uint32_t *t0;     // per chunk: the next pass's table at that start [hs]
    uint32_t *cfail;  // per chunk: its segment failed a check this pass (the next pass parses it again)
    int guess;        // the first pass starts from kc_guess's tables (else zero tables)
    int32_t C, W, O, kmax, logcap;
    uint32_t rcap_c;
};
constexpr uint32_t kKcHave = 1, kKcErr = 2, kKcBad = 4, kKcLast = 8;
constexpr uint32_t kKcIns = 0xfffffffeu, kKcNone = 0xffffffffu;
// fail codes (sinfo[3 s + 1]): a chunk's error or log overflow, no shared copy end, a judgement
// changed, the record slot
constexpr uint32_t kKcFailChunk = 1, kKcFailSync = 2, kKcFailJudge = 4, kKcFailCap = 8;
constexpr int kKcSegWords = 8, kKcInfo = 5;

struct ChunkEv {
    static constexpr bool kOn = true;
    int32_t stop, keep;
    uint32_t cnt;
    int bad;
    int32_t base;
    uint32_t cap;
    uint2 *log;
    // the window's visits (lanes 0 .. a, or all valid lanes) and the acceptor's i+1 insert
    // (group-uniform); windows wholly before the chunk are not logged (no segment reaches them)
    __device__ __forceinline__ void visit(int32_t x, int32_t cand, bool vis, bool acc, int g, int lj, int32_t i, bool insb,
                                          int32_t x1) {
        if (i + 16 <= base || bad) return;
        const uint32_t vm = gball<16>(vis, g);
        const uint32_t nv = (uint32_t)__builtin_popcount(vm);
        if (cnt + nv + 1 > cap) {
            bad = 1;
            return;
        }
        if (vis) log[cnt + (uint32_t)lj] = make_uint2((uint32_t)x, (uint32_t)cand | (acc ? 0x80000000u : 0u));
        if (insb && lj == 0) log[cnt + nv] = make_uint2((uint32_t)x1, kKcIns);
        cnt += nv + (insb ? 1u : 0u);
    }
};

template <bool LW>
__global__ __launch_bounds__(64) void kc_parse(CompressArgs A, KcBufs B, int pass) {
    constexpr int G = 16;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / G, lj = lane % G;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(A.hs - 1)));
    uint32_t *htw = (uint32_t *)smem + (uint32_t)g * (uint32_t)A.hs;
    const uint64_t c = (uint64_t)blockIdx.x * 4 + (uint32_t)g;
    const uint64_t s = c / (uint64_t)B.kmax;
    const int32_t k = (int32_t)(c % (uint64_t)B.kmax);
    const bool spec = A.spec_mode != 0;
    bool have = s < A.count;
    if (have && spec && A.spec[s].flags != 0) have = false;
    const uint8_t *blo = A.in, *bhi = A.in + A.in_off[A.count];
    int32_t n = 0, from0 = 0, done0 = 0;
    const uint8_t *p = blo;
    if (have) {
        n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        p = A.in + A.in_off[s];
        if (spec) {
            from0 = (int32_t)A.spec[s].from;
            done0 = (int32_t)A.spec[s].done;
        }
    }
    const int64_t b = (int64_t)from0 + (int64_t)k * B.C;
    if (have && k > 0 && b + 4 > n) have = false;  // no such chunk
    // later passes: the streams the last one failed on a judgement, from the failed segment's chunk on
    bool touch = have;
    int32_t cs = -1;
    if (have && pass > 1) {
        if (B.sinfo[kKcInfo * s + 1] != kKcFailJudge || B.cfail[c] == 0) touch = have = false;
        else cs = B.cstart[c];
    }
    const bool last = have && b + B.C + 4 > n;
    int32_t i0 = k == 0 ? from0 : (int32_t)(b - B.W > from0 ? b - B.W : from0);
    int32_t d0 = k == 0 ? done0 : i0;
    const uint32_t *tsrc = nullptr;
    if (cs >= 0) {  // a segment's start in the last pass's path, with its table there
        i0 = d0 = cs;
        tsrc = B.t0 + c * (uint64_t)A.hs;
    } else if (have && k == 0 && spec) {
        tsrc = A.spec_tab + s * (uint64_t)A.hs;
    } else if (have && k > 0 && pass == 1 && B.guess) {  // the warm-up start's guessed table (kc_guess)
        tsrc = B.t0 + c * (uint64_t)A.hs;
    }
    for (int32_t t = lj; t < (int32_t)A.hs; t += G) htw[t] = tsrc ? tsrc[t] : 0u;
    ChunkEv ev;
    ev.stop = last ? n : (int32_t)(b + B.C + B.O < n ? b + B.C + B.O : n);
    ev.keep = k == 0 ? (int32_t)0x80000000 : (int32_t)b;
    ev.cnt = 0;
    ev.bad = 0;
    ev.base = (int32_t)b;
    ev.cap = (uint32_t)B.logcap;
    ev.log = B.log + (have ? c : 0) * (uint64_t)B.logcap;
    int err = have && (uint64_t)n > A.max_len ? EZ_EINVAL : (have ? 0 : EZ_EINVAL);
    int32_t nrec = 0;
    uint8_t *wl = smem + (size_t)4 * A.hs * 4 + (size_t)g * kWinLdsBytes;
    long_loop<FreshSrc, LW, ChunkEv>(FreshSrc{{p, blo, bhi}}, p, n, have ? i0 : 0, have ? d0 : 0, A.bs, lj, g, htw, hsh,
                                     B.crec + (have ? c : 0) * (uint64_t)B.rcap_c, B.rcap_c, blo, bhi, nrec, err, wl, &ev);
    // (a start at a segment's start is a copy end of this parse too: the stitch may switch there)
    if (lj == 0 && s < A.count && (pass == 1 || touch))
        B.meta[c] = make_uint4((uint32_t)nrec, have ? (kKcHave | (err ? kKcErr : 0u) | (ev.bad ? kKcBad : 0u) | (last ? kKcLast : 0u)) : 0u,
                               ev.cnt, cs >= 0 && cs >= b ? (uint32_t)cs : kKcNone);
}

// The first pass's tables: chunk k's parse starts at s_k = b_k - W with, for each hash, its last
// position before s_k among all positions (Go's entry when Go visited that position; a chunk's
// zero table instead left 339,784 of C4s's 349,222 failed reads wrong).  kc_last: a block per chunk
// region [b_r, b_r+1), each hash's last position in it and in its part before b_r+1 - W (+1; 0 none);
// kc_guess: per (stream, hash) the running maximum over the regions into t0 of each chunk.
__global__ __launch_bounds__(256) void kc_last(CompressArgs A, KcBufs B) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *L = (uint32_t *)smem, *L2 = L + A.hs;
    const uint64_t s = blockIdx.x / (uint32_t)B.kmax;
    const int32_t k = (int32_t)(blockIdx.x % (uint32_t)B.kmax);
    if (s >= A.count || (A.spec_mode != 0 && A.spec[s].flags != 0)) return;
    const int32_t n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int32_t from0 = A.spec_mode != 0 ? (int32_t)A.spec[s].from : 0;
    const int64_t rb = (int64_t)from0 + (int64_t)k * B.C;
    if (rb + 4 > n) return;
    for (int32_t t = threadIdx.x; t < (int32_t)A.hs; t += 256) L[t] = L2[t] = 0;
    __syncthreads();
    const uint8_t *p = A.in + A.in_off[s];
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(A.hs - 1)));
    const int64_t re = rb + B.C < (int64_t)n - 3 ? rb + B.C : (int64_t)n - 3, cut = rb + B.C - B.W;
    for (int64_t y = rb + threadIdx.x; y < re; y += 256) {
        const uint32_t h = ((*(const u32_ua *)(p + y)) * kHashMul) >> hsh;
        atomicMax(L + h, (uint32_t)y + 1);
        if (y < cut) atomicMax(L2 + h, (uint32_t)y + 1);
    }
    __syncthreads();
    uint32_t *o = B.ft + (s * (uint64_t)B.kmax + (uint32_t)k) * 2 * (uint64_t)A.hs;  // (ft is free before the passes)
    for (int32_t t = threadIdx.x; t < (int32_t)A.hs; t += 256) o[t] = L[t], o[A.hs + t] = L2[t];
}
__global__ __launch_bounds__(256) void kc_guess(CompressArgs A, KcBufs B) {
    const uint64_t gi = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t s = gi / (uint64_t)A.hs;
    const uint32_t h = (uint32_t)(gi % (uint64_t)A.hs);
    if (s >= A.count || (A.spec_mode != 0 && A.spec[s].flags != 0)) return;
    const int32_t n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int32_t from0 = A.spec_mode != 0 ? (int32_t)A.spec[s].from : 0;
    uint32_t run = A.spec_mode != 0 ? A.spec_tab[s * (uint64_t)A.hs + h] + 1 : 0u;  // (+1: 0 = none)
    for (int32_t k = 1; k < B.kmax && (int64_t)from0 + (int64_t)k * B.C + 4 <= n; k++) {
        const uint32_t *o = B.ft + (s * (uint64_t)B.kmax + (uint32_t)(k - 1)) * 2 * (uint64_t)A.hs;
        const uint32_t g = run > o[A.hs + h] ? run : o[A.hs + h];  // before s_k = b_k - W
        B.t0[(s * (uint64_t)B.kmax + (uint32_t)k) * (uint64_t)A.hs + h] = g > 0 ? g - 1 : 0u;
        run = run > o[h] ? run : o[h];
    }
}

__device__ __forceinline__ int32_t kc_nx(const uint4 &r) { return (int32_t)(r.x + r.y); }
__device__ __forceinline__ uint32_t kc_li(const uint4 &r) { return r.w >> 1; }

// the first record of r[lo, hi) ending at or after y (copy ends never decrease along a parse)
__device__ __forceinline__ uint32_t kc_lower(const uint4 *r, uint32_t lo, uint32_t hi, int32_t y) {
    while (lo < hi) {
        const uint32_t m = lo + (hi - lo) / 2;
        if (kc_nx(r[m]) < y) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// the sequential stitch of stream s (one thread): chunk o's path up to the first copy end it shares
// with a later chunk's parse (or that chunk's start), then that chunk's; returns the failure code
__device__ uint32_t kc_stitch_seq(const CompressArgs &A, const KcBufs &B, uint64_t s, int32_t K, int32_t from0, int32_t n,
                                  int32_t &nseg, uint32_t &tot) {
    const uint64_t c0 = s * (uint64_t)B.kmax;
    uint32_t *seg = B.seg + c0 * kKcSegWords;
    uint32_t ri = 0, li = 0;
    int32_t o = 0, q = from0;
    nseg = 0;
    tot = 0;
    for (;;) {
        const uint4 mo = B.meta[c0 + o];
        const uint32_t no = mo.x;
        const uint4 *ro = B.crec + (c0 + o) * (uint64_t)B.rcap_c;
        uint32_t *e = seg + kKcSegWords * nseg;
        if (o == K - 1) {
            e[0] = (uint32_t)o, e[1] = (uint32_t)q, e[2] = (uint32_t)n, e[3] = ri, e[4] = no, e[5] = tot, e[6] = li, e[7] = mo.z;
            nseg++;
            tot += no - ri;
            return 0;
        }
        const int32_t xl = no > ri ? kc_nx(ro[no - 1]) : -1;  // this parse's last copy end
        bool found = false, virt = false;
        uint32_t fa = 0, fb = 0;
        int32_t fj = 0, Q = 0;
        for (int32_t j = o + 1; j < K && !found && (int64_t)from0 + (int64_t)j * B.C <= xl; j++) {
            const int32_t bj = (int32_t)((int64_t)from0 + (int64_t)j * B.C);
            const uint4 mj = B.meta[c0 + j];
            const uint32_t nj = mj.x;
            const uint4 *rj = B.crec + (c0 + j) * (uint64_t)B.rcap_c;
            if (mj.w != kKcNone) {  // chunk j starts at a copy end of the last pass's path
                const uint32_t ia = kc_lower(ro, ri, no, (int32_t)mj.w);
                if (ia < no && kc_nx(ro[ia]) == (int32_t)mj.w) {
                    found = virt = true;
                    fa = ia, fj = j, Q = (int32_t)mj.w;
                    break;
                }
            }
            uint32_t ia = kc_lower(ro, ri, no, bj), ib = 0;
            while (ia < no && ib < nj) {
                const int32_t va = kc_nx(ro[ia]), vb = kc_nx(rj[ib]);
                if (va == vb) {
                    found = true;
                    fa = ia, fb = ib, fj = j, Q = va;
                    break;
                }
                if (va < vb) ia++;
                else ib++;
            }
        }
        if (!found) return kKcFailSync;
        e[0] = (uint32_t)o, e[1] = (uint32_t)q, e[2] = (uint32_t)Q, e[3] = ri, e[4] = fa + 1, e[5] = tot, e[6] = li, e[7] = kc_li(ro[fa]);
        nseg++;
        tot += fa + 1 - ri;
        const uint4 *rj = B.crec + (c0 + fj) * (uint64_t)B.rcap_c;
        li = virt ? 0u : kc_li(rj[fb]);
        o = fj, q = Q, ri = virt ? 0u : fb + 1;
    }
}

// a wave per stream.  Every boundary k -> k+1 at once: the first copy end at or after b_k+1 that
// chunk k's parse shares with chunk k+1's (or chunk k+1's start); when every boundary has one and
// they increase, the segments are the chunks themselves and their record offsets a scan; else (a
// copy across a whole chunk, no shared end) the sequential stitch decides (C4s: 0.62 ms a pass
// for 64 streams x 128 chunks with the sequential one alone)
constexpr int32_t kKcPar = 1024;  // chunks the parallel stitch takes
constexpr uint32_t kKcVirt = 0xfffffffdu, kKcNoJoin = 0xfffffffcu;
__global__ __launch_bounds__(64) void kc_stitch(CompressArgs A, KcBufs B, uint64_t rcap, int pass) {
    __shared__ int32_t sQ[kKcPar];
    __shared__ uint32_t sfa[kKcPar], sfb[kKcPar];
    const uint64_t s = blockIdx.x;
    const int lane = (int)threadIdx.x;
    if (s >= A.count) return;
    if (A.spec_mode != 0 && A.spec[s].flags != 0) return;
    uint32_t *si = B.sinfo + kKcInfo * s;
    if (pass > 1 && si[1] != kKcFailJudge) return;
    const uint64_t c0 = s * (uint64_t)B.kmax;
    const int32_t n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int32_t from0 = A.spec_mode != 0 ? (int32_t)A.spec[s].from : 0;
    // the stream's chunks (present from 0 on, up to the one marked last) and their errors
    int32_t K = B.kmax;
    bool cerr = false;
    for (int32_t k = lane; k < B.kmax; k += 64) {
        const uint32_t f = B.meta[c0 + k].y;
        const int32_t kk = !(f & kKcHave) ? k : ((f & kKcLast) ? k + 1 : B.kmax);
        K = kk < K ? kk : K;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const int32_t o = __shfl_xor(K, d, 64);
        K = o < K ? o : K;
    }
    for (int32_t k = lane; k < K; k += 64) cerr = cerr || (B.meta[c0 + k].y & (kKcErr | kKcBad)) != 0;
    uint32_t fail = __ballot(cerr) != 0 ? kKcFailChunk : 0u;
    int32_t nseg = 0;
    uint32_t tot = 0;
    bool par = !fail && K <= kKcPar;
    if (par) {
        for (int32_t k = lane; k < K - 1; k += 64) {  // boundary k -> k+1
            const uint32_t no = B.meta[c0 + k].x;
            const uint4 *ro = B.crec + (c0 + k) * (uint64_t)B.rcap_c;
            const int32_t bj = (int32_t)((int64_t)from0 + (int64_t)(k + 1) * B.C);
            const uint4 mj = B.meta[c0 + k + 1];
            const uint4 *rj = B.crec + (c0 + k + 1) * (uint64_t)B.rcap_c;
            uint32_t fa = 0, fb = kKcNoJoin;
            int32_t Q = 0;
            if (mj.w != kKcNone) {
                const uint32_t ia = kc_lower(ro, 0, no, (int32_t)mj.w);
                if (ia < no && kc_nx(ro[ia]) == (int32_t)mj.w) fa = ia, fb = kKcVirt, Q = (int32_t)mj.w;
            }
            if (fb == kKcNoJoin) {
                uint32_t ia = kc_lower(ro, 0, no, bj), ib = 0;
                while (ia < no && ib < mj.x) {
                    const int32_t va = kc_nx(ro[ia]), vb = kc_nx(rj[ib]);
                    if (va == vb) {
                        fa = ia, fb = ib, Q = va;
                        break;
                    }
                    if (va < vb) ia++;
                    else ib++;
                }
            }
            sQ[k] = Q, sfa[k] = fa, sfb[k] = fb;
        }
        __syncthreads();
        // every boundary joined, the joins increasing, each segment at least its start record
        bool bad = false;
        for (int32_t k = lane; k < K - 1; k += 64) {
            if (sfb[k] == kKcNoJoin) bad = true;
            else if (k > 0 && (sQ[k] <= sQ[k - 1] || sfb[k - 1] == kKcNoJoin ||
                               (sfb[k - 1] != kKcVirt && sfa[k] < sfb[k - 1] + 1)))
                bad = true;
        }
        par = __ballot(bad) == 0;
    }
    if (par) {
        // segment k = chunk k: [Q_k-1, Q_k), records [ri_k, fa_k + 1), log [li_k, li of fa_k)
        uint32_t *seg = B.seg + c0 * kKcSegWords;
        uint32_t carry = 0;
        for (int32_t k0 = 0; k0 < K; k0 += 64) {
            const int32_t k = k0 + lane;
            uint32_t cnt = 0, w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (k < K) {
                const uint4 mk = B.meta[c0 + k];
                const uint4 *rk = B.crec + (c0 + k) * (uint64_t)B.rcap_c;
                const bool first = k == 0, lastk = k == K - 1;
                const bool pv = !first && sfb[k - 1] == kKcVirt;
                const uint32_t ri = first || pv ? 0u : sfb[k - 1] + 1;
                const uint32_t li = first || pv ? 0u : kc_li(rk[sfb[k - 1]]);
                const uint32_t rhi = lastk ? mk.x : sfa[k] + 1;
                const uint32_t lhi = lastk ? mk.z : kc_li(rk[sfa[k]]);
                w[0] = (uint32_t)k, w[1] = first ? (uint32_t)from0 : (uint32_t)sQ[k - 1], w[2] = lastk ? (uint32_t)n : (uint32_t)sQ[k];
                w[3] = ri, w[4] = rhi, w[6] = li, w[7] = lhi;
                cnt = rhi - ri;
            }
            uint32_t incl = cnt;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t u = (uint32_t)__shfl_up((int)incl, d, 64);
                if (lane >= d) incl += u;
            }
            if (k < K) {
                w[5] = carry + incl - cnt;
                for (int t = 0; t < kKcSegWords; t++) seg[(uint64_t)k * kKcSegWords + t] = w[t];
            }
            carry += (uint32_t)__shfl((int)incl, 63, 64);
        }
        nseg = K;
        tot = carry;
    } else if (!fail && lane == 0) {
        fail = kc_stitch_seq(A, B, s, K, from0, n, nseg, tot);
    }
    fail = (uint32_t)__shfl((int)fail, 0, 64);
    if (!fail && tot > rcap) fail = kKcFailCap;
    for (int32_t k = lane; k < K; k += 64) B.cstart[c0 + k] = -1, B.cfail[c0 + k] = 0;  // (kc_v2 sets the segments' owners)
    if (lane == 0) {
        si[0] = (uint32_t)nseg;
        si[1] = fail;
        si[2] = (uint32_t)K;
        si[3] = kKcNone;
        si[4] = (uint32_t)pass;
        if (!fail) A.out_size[s] = tot;
    }
}

// streams still failed on a judgement after this pass (the host stops the passes at 0)
__global__ __launch_bounds__(256) void kc_count(CompressArgs A, KcBufs B, uint32_t *left) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool f = s < A.count && !(A.spec_mode != 0 && A.spec[s].flags != 0) && B.sinfo[kKcInfo * s + 1] == kKcFailJudge;
    const uint64_t m = __ballot(f);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(left, (uint32_t)__builtin_popcountll(m));
}

// this pass's path of stream s is to be checked (stitched now, not given up)
__device__ __forceinline__ bool kc_checking(const KcBufs &B, uint64_t s, int pass) {
    const uint32_t *si = B.sinfo + kKcInfo * s;
    return si[4] == (uint32_t)pass && (si[1] == 0 || si[1] == kKcFailJudge) && si[0] != 0;
}

// a block per (stream, segment): the segment's records into the stream's slot
__global__ __launch_bounds__(256) void kc_gather(CompressArgs A, KcBufs B, uint4 *recs, uint64_t rcap, int pass) {
    const uint64_t s = blockIdx.x / (uint32_t)B.kmax;
    const uint32_t t = blockIdx.x % (uint32_t)B.kmax;
    if (s >= A.count || (A.spec_mode != 0 && A.spec[s].flags != 0)) return;
    if (!kc_checking(B, s, pass) || t >= B.sinfo[kKcInfo * s]) return;
    const uint32_t *e = B.seg + (s * (uint64_t)B.kmax + t) * kKcSegWords;
    const uint4 *src = B.crec + (s * (uint64_t)B.kmax + e[0]) * (uint64_t)B.rcap_c;
    uint4 *dst = recs + s * rcap + e[5];
    for (uint32_t r = e[3] + threadIdx.x; r < e[4]; r += 256) dst[r - e[3]] = src[r];
}

// Go's acceptance of position x with candidate cand while the pending literal starts at done: the
// judgement of one lane of long_loop (writer.go:213-301, :441-473), from the stream's bytes
__device__ bool kc_accepts(const uint8_t *p, int32_t n, int32_t x, int32_t cand, int32_t done, int64_t bs, const uint8_t *blo,
                           const uint8_t *bhi) {
    const FreshSrc P{{p, blo, bhi}};
    const bool rl = cand >= done && cand < x;
    if (!rl && (int64_t)done - cand > bs) return false;  // the far skip
    V16 w0, w1, w2, c0, c1, c2;
    bytes48_chk(p, x, w0, w1, w2, blo, bhi);
    P.bytes48(cand, c0, c1, c2);
    if (!rl && (int64_t)cand - 8 < (int64_t)done - bs) c0.lo = ring16(P, cand - 8, done, bs).lo;
    int32_t jf = first_diff40(w0.hi ^ c0.hi, w1.lo ^ c1.lo, w1.hi ^ c1.hi, w2.lo ^ c2.lo, w2.hi ^ c2.hi);
    jf = jf < n - x ? jf : n - x;
    int32_t bl = x - done;
    if (rl) bl = bl < cand ? bl : cand;
    int32_t jb = last_diff8(w0.lo ^ c0.lo);
    jb = jb < bl ? jb : bl;
    const bool zr = rl && c0.hi == 0 && cand + 8 < n;
    const int32_t fw = rl ? jf : (jf < done - cand ? jf : done - cand);
    const int64_t t1 = bs - (int64_t)(x - cand);
    const int32_t len = rl ? fw + jb : (int32_t)((int64_t)(fw + jb) < t1 ? (int64_t)(fw + jb) : (t1 < 0 ? -1 : t1));
    return zr || len >= kMinCopyChunk;
}

// log entry li of segment e (stream s) read `got` (bit 31: it accepted) where the path's table held
// `exact`: the stream stands only if that visit rejects with `exact` too, from the path's pending
// literal start there (the last record of the segment logged before the visit, else the segment's start)
__device__ void kc_recheck(const CompressArgs &A, const KcBufs &B, uint64_t s, uint32_t t, const uint32_t *e, uint32_t li,
                           uint32_t got, uint32_t exact) {
    bool bad = (got >> 31) != 0;
    if (!bad) {
        const uint4 *r = B.crec + (s * (uint64_t)B.kmax + e[0]) * (uint64_t)B.rcap_c;
        uint32_t lo = e[3], hi = e[4];  // the first record logged after li
        while (lo < hi) {
            const uint32_t m = lo + (hi - lo) / 2;
            if (kc_li(r[m]) <= li) lo = m + 1;
            else hi = m;
        }
        const int32_t done = lo > e[3] ? kc_nx(r[lo - 1]) : (int32_t)e[1];
        const int32_t x = (int32_t)B.log[(s * (uint64_t)B.kmax + e[0]) * (uint64_t)B.logcap + li].x;
        const uint8_t *p = A.in + A.in_off[s];
        const int32_t n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        bad = kc_accepts(p, n, x, (int32_t)exact, done, A.bs, A.in, A.in + A.in_off[A.count]);
    }
#if (EZ_EXP & 65536)
    // (experiment builds) mismatched reads; failing ones by kind: the read was a zero entry, the
    // right entry older / newer than the one read, the right entry before the chunk's own start
    atomicAdd(&g_kc_diag[0], 1ull);
    if (bad) {
        atomicAdd(&g_kc_diag[1], 1ull);
        if ((got & 0x7fffffffu) == 0) atomicAdd(&g_kc_diag[2], 1ull);
        if (exact < (got & 0x7fffffffu)) atomicAdd(&g_kc_diag[3], 1ull);
        else atomicAdd(&g_kc_diag[4], 1ull);
        if ((got >> 31) != 0) atomicAdd(&g_kc_diag[5], 1ull);
        const int64_t ck = (int64_t)e[0] * B.C - B.W;
        if ((int64_t)exact < ck) atomicAdd(&g_kc_diag[6], 1ull);
    }
#endif
    if (bad) {
        B.sinfo[kKcInfo * s + 1] = kKcFailJudge;
        atomicMin(B.sinfo + kKcInfo * s + 3, t);
        B.cfail[s * (uint64_t)B.kmax + e[0]] = 1;
    }
}

// a wave per (stream, segment): the segment's log in order, 64 visits a step; a visit's right entry
// is the position of the nearest earlier same-hash event of the step (ballots over the hash bits)
// or the segment's table so far; a segment's first read of a hash is left to kc_v2
__global__ __launch_bounds__(64) void kc_v1(CompressArgs A, KcBufs B, int pass) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *T = (uint32_t *)smem, *F = T + A.hs;
    const int lane = (int)threadIdx.x;
    const uint64_t s = blockIdx.x / (uint32_t)B.kmax;
    const uint32_t t = blockIdx.x % (uint32_t)B.kmax;
    if (s >= A.count || (A.spec_mode != 0 && A.spec[s].flags != 0)) return;
    if (!kc_checking(B, s, pass) || t >= B.sinfo[kKcInfo * s]) return;
    const int32_t hs = (int32_t)A.hs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));
    const int hb = 32 - (int)hsh;
    for (int32_t u = lane; u < hs; u += 64) T[u] = F[u] = kKcNone;
    const uint8_t *p = A.in + A.in_off[s];
    const uint32_t *e = B.seg + (s * (uint64_t)B.kmax + t) * kKcSegWords;
    const uint2 *lg = B.log + (s * (uint64_t)B.kmax + e[0]) * (uint64_t)B.logcap;
    const uint32_t lhi = e[7];
    __syncthreads();
    for (uint32_t l0 = e[6]; l0 < lhi; l0 += 64) {
        const uint32_t li = l0 + (uint32_t)lane;
        const bool in = li < lhi;
        const uint2 v = in ? lg[li] : make_uint2(0, 0);
        const uint32_t h = in ? ((*(const u32_ua *)(p + v.x)) * kHashMul) >> hsh : 0u;
        uint64_t m = __ballot(in);
        for (int u = 0; u < hb; u++) {
            const uint64_t bb = __ballot(in && ((h >> u) & 1));
            m &= ((h >> u) & 1) ? bb : ~bb;
        }
        const uint64_t lower = lane == 0 ? 0ull : (m & (~0ull >> (64 - lane)));
        const int pl = lower ? 63 - (int)__builtin_clzll(lower) : 0;
        const uint32_t xp = (uint32_t)__shfl((int)v.x, pl, 64);
        const uint32_t tv = in ? T[h] : 0u;
        const uint32_t exact = lower ? xp : tv;
        if (in && v.y != kKcIns) {
            if (exact == kKcNone) F[h] = li;
            else if ((v.y & 0x7fffffffu) != exact) kc_recheck(A, B, s, t, e, li, v.y, exact);
        }
        const uint64_t above = lane == 63 ? 0ull : (m >> (lane + 1));
        if (in && above == 0) T[h] = v.x;
    }
    __syncthreads();
    uint32_t *ft = B.ft + (s * (uint64_t)B.kmax + t) * 2 * (uint64_t)hs;
    for (int32_t u = lane; u < hs; u += 64) {
        ft[u] = F[u];
        ft[hs + u] = T[u];
    }
}

// a thread per (stream, hash): each segment's first read of the hash against the entry the
// segments before it leave (0 at the stream start, K1x's table after its rounds); that entry is also
// the next pass's table at the segment's start
__global__ __launch_bounds__(256) void kc_v2(CompressArgs A, KcBufs B, int pass) {
    const uint64_t gi = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t s = gi / (uint64_t)A.hs;
    const uint32_t h = (uint32_t)(gi % (uint64_t)A.hs);
    if (s >= A.count || (A.spec_mode != 0 && A.spec[s].flags != 0)) return;
    if (!kc_checking(B, s, pass)) return;
    const uint32_t ns = B.sinfo[kKcInfo * s];
    uint32_t run = A.spec_mode != 0 ? A.spec_tab[s * (uint64_t)A.hs + h] : 0u;
    for (uint32_t t = 0; t < ns; t++) {
        const uint32_t *ft = B.ft + (s * (uint64_t)B.kmax + t) * 2 * (uint64_t)A.hs;
        const uint32_t f = ft[h], w = ft[A.hs + h];
        const uint32_t *e = B.seg + (s * (uint64_t)B.kmax + t) * kKcSegWords;
        if (t > 0) {
            const uint64_t c = s * (uint64_t)B.kmax + e[0];
            B.t0[c * (uint64_t)A.hs + h] = run;
            if (h == 0) B.cstart[c] = (int32_t)e[1];
        }
        if (f != kKcNone) {
            const uint32_t got = B.log[(s * (uint64_t)B.kmax + e[0]) * (uint64_t)B.logcap + f].y;
            if ((got & 0x7fffffffu) != run) kc_recheck(A, B, s, t, e, f, got, run);
        }
        if (w != kKcNone) run = w;
    }
}

// K1L on a Writer handle (Writer.Write writer.go:206-337 on a stream at position start): one 16-lane
// group, the handle's table (uint32 stream positions) in LDS as positions relative to the Write (far
// ones clamped: the far skip, writer.go:219-221, still sees them as far), the history before the Write
// from the handle's ring (RingSrc).  The table goes back to the handle, converted back, at the end.
constexpr int32_t kRelFar = 1 << 28;  // |relative position| clamp (bs <= 2^26, Writes < 2^27 bytes)
template <bool WIDE>
__device__ __forceinline__ void emit_stream(const CompressArgs &A, const uint64_t *recs, uint64_t rcap, const uint64_t s, const int lane,
                                            uint64_t *stage = nullptr, uint8_t *sin = nullptr);
// the staged ring bytes for a Write of n bytes: 16 n, at least kRingMin, at most kLdsRing
#ifndef EZ_K1R_RL
#define EZ_K1R_RL 32768
#endif
__device__ __forceinline__ int32_t knob_dev_rl(int32_t n) {
    const int32_t r = 16 * n < EZ_K1R_RL ? EZ_K1R_RL : (16 * n > kLdsRing ? kLdsRing : ((16 * n + 15) & ~15));
    return r > kLdsRing ? kLdsRing : r;
}
template <bool LDS>
__global__ __launch_bounds__(256) void k1_long_ring(CompressArgs A, uint4 *recs, uint64_t rcap) {
    constexpr int G = 16;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = (int)threadIdx.x, lane = tid & 63;  // 4 waves stage; wave 0's first group parses
    const int g = lane / G + 4 * (tid >> 6), lj = lane % G;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(A.hs - 1)));
    uint32_t *htw = (uint32_t *)smem;
    const uint8_t *p = A.in + A.in_off[0];
    const int32_t n = (int32_t)(A.in_off[1] - A.in_off[0]);
    uint8_t *lds = smem + (size_t)A.hs * 4;
    // the ring's last rl bytes staged before the Write (older candidates read the ring in HBM; staging
    // less for small Writes measured no faster: 100-byte Writes 26.2 / 27.2 against 26.8 / 25.2 us at
    // 4 KiB and 32 KiB, two alternating runs; -DEZ_K1R_RL=<bytes> builds for A/B)
    static_assert(kLdsRing % 16 == 0, "");
    const int32_t want = knob_dev_rl(n);
    const int32_t rl = A.bs < want ? (int32_t)A.bs : want;
    const uint32_t mask = (uint32_t)(A.bs - 1);
    if (LDS) {  // the ring's last rl bytes, the Write, 64 zeros: 16 bytes per lane and step, 4 loads in flight
        const RingSrc R{p, p, p + n, A.ring, A.start, mask};
        for (int32_t y0 = -rl + 16 * tid; y0 < n + 64; y0 += 4 * 16 * 256) {
            V16 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int32_t y = y0 + u * 16 * 256;
                if (y < 0) v[u] = R.ring_at(y);  // (rl is a multiple of 16: no piece straddles the Write's start)
                else v[u] = p + y + 16 <= p + n ? ld16v(p + y) : (y < n ? ld_clamped(p + y, p, p + n) : V16{0, 0});
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int32_t y = y0 + u * 16 * 256;
                if (y < n + 64) {
                    *(u64_ua *)(lds + kLdsRing + y) = v[u].lo;
                    *(u64_ua *)(lds + kLdsRing + y + 8) = v[u].hi;
                }
            }
        }
    }
    // the table by the whole block (the parse below is one group's)
#pragma unroll 4
    for (int32_t k = tid; k < (int32_t)A.hs; k += 256) {
        int64_t r = (int64_t)A.ht_global[k] - A.start;
        r = r < -kRelFar ? -kRelFar : (r > kRelFar ? kRelFar : r);
        htw[k] = (uint32_t)(int32_t)r;
    }
    __syncthreads();
    int err = 0;
    int32_t nrec = 0;
    if (g == 0) {  // one group (the other lanes idle)
        const RingSrc P{p, p, p + n, A.ring, A.start, mask};
        if (LDS) long_loop(LdsSrc{lds, rl, n, P}, p, n, 0, 0, A.bs, lj, 0, htw, hsh, recs, rcap, p, p + n, nrec, err);
        else long_loop(P, p, n, 0, 0, A.bs, lj, 0, htw, hsh, recs, rcap, p, p + n, nrec, err);
    }
    __syncthreads();
    for (int32_t k = tid; k < (int32_t)A.hs; k += 256) {
        const int32_t r = (int32_t)htw[k];
        if (r != -kRelFar && r != kRelFar) A.ht_global[k] = (uint32_t)(A.start + r);
    }
    if (LDS) {  // the Write into the handle's ring (k1_ring_store's work; the parse has read the ring)
        const int32_t from = (int64_t)n > A.bs ? (int32_t)(n - A.bs) : 0;
        for (int32_t k = from + 16 * tid; k < n; k += 16 * 256) {
            const uint32_t r = (uint32_t)((A.start + k) & mask);
            const uint8_t *q = lds + kLdsRing + k;
            if (k + 16 <= n && r + 16 <= mask + 1) {
                *(u64_ua *)(A.ring + r) = *(const u64_ua *)q;
                *(u64_ua *)(A.ring + r + 8) = *(const u64_ua *)(q + 8);
            } else {
                for (int32_t t = 0; t < 16 && k + t < n; t++) A.ring[(r + (uint32_t)t) & mask] = q[t];
            }
        }
    }
    if (tid == 0) A.out_size[0] = (uint64_t)nrec | ((uint64_t)err << 48);
    if (LDS) {
        // the token writer (k1_emit's emit_stream) by wave 0 of the same block: one launch per Write
        __threadfence();
        __syncthreads();
        if (tid < 64) emit_stream<true>(A, (const uint64_t *)recs, rcap, 0, lane);
        if (A.done_flag) {
            __syncthreads();
            if (tid == 0) {
                __threadfence_system();
                __hip_atomic_store(A.done_flag, A.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// the Write's last min(n, bs) bytes into the handle's ring (block[(start + k) & mask], copyData)
__global__ __launch_bounds__(256) void k1_ring_store(CompressArgs A) {
    const uint8_t *p = A.in + A.in_off[0];
    const int64_t n = (int64_t)(A.in_off[1] - A.in_off[0]);
    const int64_t from = n > A.bs ? n - A.bs : 0;
    const uint64_t mask = (uint64_t)A.bs - 1;
    for (int64_t k = from + (int64_t)(blockIdx.x * 256 + threadIdx.x); k < n; k += (int64_t)gridDim.x * 256)
        A.ring[(uint64_t)(A.start + k) & mask] = p[k];
}

// Edge slots (after the records in the K1 scratch): a zeroed 128-byte dummy region for lane groups
// without a stream, then kEdgeSlots slots of edge_slot_bytes, then the slot counter (zeroed by the
// launcher).  A live stream (n >= 4) lacks the 64 bytes before or the 64 after it only if it starts
// in the batch's first 64 bytes (at most 16 such streams, each >= 4 bytes) or ends in its last 64
// (at most 16): 32 slots always suffice.

// waves per SIMD the VGPR budget is cut for: 8-lane groups are held to ~2 by their tables' LDS, so
// they keep VGPRs (no spills); (EZ_EXP & 8192 builds: 16-lane groups at 4, A/B)
#if (EZ_EXP & 8192)
constexpr int kLeanWaves16 = 4;
#else
constexpr int kLeanWaves16 = 5;
#endif
#if (EZ_EXP & 2097152)
constexpr uint32_t kLeanTMax = 1u << 18;
__device__ uint64_t g_lean_t[2 * kLeanTMax];
#endif
template <int TB, bool LW = false, int FW = 24, bool PERSIST = false, int G = 16>
__global__ __launch_bounds__(64, G == 8 ? 2 : (TB == 12 ? 6 : kLeanWaves16)) void k1_lean(CompressArgs A, uint32_t stride_words, uint32_t table_words, uint64_t *recs,
                                                 uint64_t rcap, int prio, uint8_t *edge) {
    constexpr int S = 64 / G;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / G, lj = lane % G;
    const int32_t hs = (int32_t)A.hs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));
    uint16_t *hth = (uint16_t *)((uint32_t *)smem + (uint32_t)g * stride_words);
    // (LW: the groups' window buffers after the S tables)
    uint8_t *wl = smem + (size_t)4 * stride_words * S + (size_t)g * kWinLdsBytes;
#if (EZ_EXP & 2097152)
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    lean_run<TB, LW, FW, PERSIST, G>(A, lj, g, hth, table_words, hsh, recs, rcap, prio, edge, wl);
#if (EZ_EXP & 2097152)
    {  // (timing builds) the wave's start and end (100 MHz), its XCC and CU
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        uint32_t hw = 0, xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        if (lane == 0 && blockIdx.x < kLeanTMax) {
            g_lean_t[2 * blockIdx.x] = t_start;
            g_lean_t[2 * blockIdx.x + 1] = (t_end & 0xffffffffffull) | ((uint64_t)((hw >> 8) & 15) << 40) | ((uint64_t)((hw >> 13) & 7) << 44) |
                                           ((uint64_t)((hw >> 12) & 1) << 47) | ((uint64_t)(xcc & 15) << 48) | ((uint64_t)((hw >> 4) & 3) << 52);
        }
    }
#endif
}

// ---------------------------------------------------------------- K1e
// 16 bytes at y of the batch [lo, hi) (bytes outside read as 0)
__device__ __forceinline__ V16 ld16_in(const uint8_t *y, const uint8_t *lo, const uint8_t *hi) {
    return y + 16 <= hi ? ld16v(y) : ld_clamped(y, lo, hi);
}

// copy L bytes src -> dst, one lane
__device__ __forceinline__ void copy_lane(uint8_t *dst, const uint8_t *src, int32_t L, const uint8_t *lo, const uint8_t *hi) {
    int32_t q = 0;
    for (; q + 16 <= L; q += 16) st16v(dst + q, ld16_in(src + q, lo, hi));
    if (q < L) put_small(dst + q, ld16_in(src + q, lo, hi), (uint32_t)(L - q));
}

constexpr int32_t kLongLit = 96;  // literals this long are copied by the whole wave
constexpr int kEmitStage = 320;    // records of a stream staged in LDS by k1_emit (C1: ~220 per stream)
constexpr int32_t kEmitIn = 4096;  // streams this short have their bytes staged in LDS by k1_emit too
typedef uint64_t __attribute__((aligned(1))) u64_lds_ua;
// copy L bytes from LDS (src) -> dst, one lane
__device__ __forceinline__ void copy_lane_lds(uint8_t *dst, const uint8_t *src, int32_t L) {
    int32_t q = 0;
    for (; q + 16 <= L; q += 16) st16v(dst + q, V16{*(const u64_lds_ua *)(src + q), *(const u64_lds_ua *)(src + q + 8)});
    if (q < L) put_small(dst + q, V16{*(const u64_lds_ua *)(src + q), *(const u64_lds_ua *)(src + q + 8)}, (uint32_t)(L - q));
}

// WIDE: k1_long's 16-byte records, and (spec_mode) the streams K1x hands over: their header and
// first tokens are written already, the output continues at spec[s].op with the pending literal
// from spec[s].done; streams K1x finished are skipped
// the token writer of stream s (wave-uniform) by one wave
template <bool WIDE>
__device__ __forceinline__ void emit_stream(const CompressArgs &A, const uint64_t *recs, uint64_t rcap, const uint64_t s, const int lane,
                                            uint64_t *stage, uint8_t *sin) {
    const bool spec = WIDE && A.spec_mode != 0;
    if (spec && A.spec[s].flags != 0) return;
    const uint8_t *lo = A.in, *hi = A.in + A.in_off[A.count];
    const uint8_t *p = A.in + A.in_off[s];
    const int32_t n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    uint8_t *out = A.out + A.out_off[s];
    const int64_t cap64 = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    const int32_t cap = cap64 > 0x7fffffff ? 0x7fffffff : (int32_t)cap64;
    const uint64_t pr = A.out_size[s];
    const uint64_t m64 = pr & 0xffffffffffffull;
    const int32_t m = (int32_t)(m64 < rcap ? m64 : rcap);
    int err = (int)(pr >> 48);
    const uint64_t *rec = recs + s * rcap;

    // header (writer.go:495-517): magic + reset, or reset alone
    const int32_t H = spec ? (int32_t)A.spec[s].op : (A.header ? (A.append_magic ? 9 : 3) : 0);
    if (!spec && H > cap) {
        if (lane == 0) {
            A.out_size[s] = 0;
            if (A.status) A.status[s] = EZ_ENOSPC;
        }
        return;
    }
    if (lane == 0 && !spec && H > 0) {
        const int32_t bsl = (int32_t)__builtin_ctzll((uint64_t)A.bs);
        const uint64_t hm = A.append_magic ? (0x141080797a616502ull << 8 | 0x80) : (0x80ull | 0x10ull << 8 | (uint64_t)bsl << 16);
        const V16 hv{hm, A.append_magic ? (uint64_t)bsl : 0ull};
        put_small(out, hv, (uint32_t)H);
    }
    int32_t op = H, done = spec ? (int32_t)A.spec[s].done : 0;
    bool full = false;
    // (stage: the stream's records in LDS, read with one round trip for all of them instead of one
    // per 64-record chunk, each of which waited for the previous chunk's stores -- vmcnt is in order)
    const bool staged = !WIDE && stage != nullptr && m <= kEmitStage;
    // (sin: the stream's bytes in LDS too, loaded with the records, so the literals' bytes are LDS
    // reads instead of a load round trip per 64 tokens: C1's 4 KiB streams)
    const bool inl = staged && sin != nullptr && n <= kEmitIn;
    if (!WIDE && staged) {
        uint64_t t[kEmitStage / 64];
        V16 u[kEmitIn / 1024];
#pragma unroll
        for (int q = 0; q < kEmitStage / 64; q++) t[q] = q * 64 + lane < m ? rec[q * 64 + lane] : 0ull;
        if (inl) {
#pragma unroll
            for (int q = 0; q < kEmitIn / 1024; q++) u[q] = 16 * (q * 64 + lane) < n ? ld16_in(p + 16 * (q * 64 + lane), lo, hi) : V16{0, 0};
        }
#pragma unroll
        for (int q = 0; q < kEmitStage / 64; q++) stage[q * 64 + lane] = t[q];
        if (inl) {
            typedef uint64_t __attribute__((aligned(8))) u64a8;
#pragma unroll
            for (int q = 0; q < kEmitIn / 1024; q++) {
                *(u64a8 *)(sin + 16 * (q * 64 + lane)) = u[q].lo;
                *(u64a8 *)(sin + 16 * (q * 64 + lane) + 8) = u[q].hi;
            }
        }
    }
    for (int32_t b0 = 0; b0 < m && !full; b0 += 64) {
        const int32_t k = b0 + lane;
        const bool here = k < m;
        int32_t lit_end, clen, dist;
        bool forced;
        if (WIDE) {
            const uint4 r4 = here ? ((const uint4 *)recs)[s * rcap + (uint64_t)k] : make_uint4(0, 0, 0, 0);
            lit_end = (int32_t)r4.x;
            clen = (int32_t)r4.y;
            dist = (int32_t)r4.z;
            forced = (r4.w & 1) != 0;
        } else {
            const uint64_t r = here ? (staged ? stage[k] : rec[k]) : 0ull;
            lit_end = (int32_t)(r & 0xfffff);
            clen = (int32_t)((r >> 20) & 0xfffff);
            dist = (int32_t)((r >> 40) & 0xfffff);
            forced = (r >> 60) != 0;
        }
        const int32_t end = lit_end + clen;
        const int32_t dk = wshr1(end, done);  // the previous record's end (lane 0: done)
        const int32_t L = lit_end - dk;
        const bool lit = here && (forced || L > 0);
        int32_t ln = 0, tn = 0, on = 0;
        const uint64_t lb = tag_bytes(0x00, L, &ln);
        if (!lit) ln = 0;
        uint64_t tb = tag_bytes(0x80, clen, &tn);
        uint64_t ob = off_bytes(dist, clen, &on);
        if (clen == 0) {  // a Write's end: its trailing literal only (writer.go:324-329)
            tb = ob = 0;
            tn = on = 0;
        }
        const int32_t T = here ? ln + (lit ? L : 0) + tn + on : 0;
        // inclusive prefix sum of T over the wave (DPP)
        const int32_t incl = wscan_add(T);
        const int32_t tok = op + incl - T;  // this token's output position
        const bool fits = here && tok + T <= cap;
        const uint64_t nofit = __ballot(here && !fits);
        const int lastok = nofit ? __builtin_ctzll(nofit) - 1 : 63;  // last lane whose token is written
        const bool wr = fits && lane <= lastok;
        bool longlit = false;
        if (wr) {
            uint8_t *d = out + tok;
            if (ln) put_small(d, V16{lb, 0}, (uint32_t)ln);
            if (lit) {
                if (L >= kLongLit) longlit = true;
                else if (inl) copy_lane_lds(d + ln, sin + dk, L);
                else copy_lane(d + ln, p + dk, L, lo, hi);
            }
            if (tn) {
                const uint64_t c0 = tb | (ob << (8 * tn));
                const uint64_t c1 = ob >> (64 - 8 * tn);
                put_small(d + T - tn - on, V16{c0, c1}, (uint32_t)(tn + on));
            }
        }
        // long literals: the whole wave, one at a time
        for (uint64_t lm = __ballot(longlit); lm; lm &= lm - 1) {
            const int src = __builtin_ctzll(lm);
            const int32_t Ls = rl32(L, src), ds = rl32(dk, src), ts = rl32(tok, src) + rl32(ln, src);
            for (int32_t q = 16 * lane; q < Ls; q += 16 * 64) {
                const V16 v = ld16_in(p + ds + q, lo, hi);
                if (q + 16 <= Ls) st16v(out + ts + q, v);
                else put_small(out + ts + q, v, (uint32_t)(Ls - q));
            }
        }
        if (nofit) {
            full = true;
            err = err ? err : EZ_ENOSPC;
            op = rl32(tok, lastok + 1);
        } else {
            op = rl32(op + incl, 63);
            done = rl32(end, m - b0 >= 64 ? 63 : m - b0 - 1);
        }
    }
    // trailing literal (writer.go:324-329)
    if (!full && !err && done < n) {
        const int32_t L = n - done;
        int32_t ln = 0;
        const uint64_t lb = tag_bytes(0x00, L, &ln);
        if (op + ln + L > cap) {
            err = EZ_ENOSPC;
        } else {
            if (lane == 0) put_small(out + op, V16{lb, 0}, (uint32_t)ln);
            const int32_t ts = op + ln;
            for (int32_t q = 16 * lane; q < L; q += 16 * 64) {
                const V16 v = ld16_in(p + done + q, lo, hi);
                if (q + 16 <= L) st16v(out + ts + q, v);
                else put_small(out + ts + q, v, (uint32_t)(L - q));
            }
            op += ln + L;
        }
    }
    if (lane == 0) {
        A.out_size[s] = (uint64_t)op;
        if (A.status) A.status[s] = err;
    }
}

template <bool WIDE>
__global__ __launch_bounds__(256, 8) void k1_emit(CompressArgs A, const uint64_t *recs, uint64_t rcap) {
    __shared__ uint64_t stage[WIDE ? 1 : 4][WIDE ? 1 : kEmitStage];
    __shared__ __attribute__((aligned(16))) uint8_t sin[WIDE ? 1 : 4][WIDE ? 16 : kEmitIn + 32];
    const int lane = (int)(threadIdx.x & 63);
    // the wave's stream, wave-uniform (readfirstlane: its per-stream values live in SGPRs)
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t s = (uint64_t)blockIdx.x * 4 + (uint32_t)w;
    if (s >= A.count) return;
    emit_stream<WIDE>(A, recs, rcap, s, lane, WIDE ? nullptr : &stage[WIDE ? 0 : w][0], WIDE ? nullptr : &sin[WIDE ? 0 : w][0]);
}

// The token writer for 16-byte records (K1L, K1c) across the chip: k1_emit<true> walks a stream's
// records with one wave, 64 at a time (C4s: 64 waves over ~180 k records each, 6.6 ms).  Here blocks
// of kEwRec records each sum their tokens' sizes (ke_size), one wave per stream scans the block sums
// after the header (ke_scan, which also decides the stream's size and status as emit_stream does),
// and every block writes its tokens at their offsets (ke_write).  Tokens, literal bytes and the
// trailing literal are emit_stream's; a token is written when it ends within the slot, and a slot
// too small ends the output at the first token that does not fit (ENOSPC), as emit_stream's does.
constexpr int32_t kEwRec = 2048, kEwPer = kEwRec / 256;
struct EwBufs {
    uint64_t *bsum;   // per (stream, block): the block's token bytes, then (ke_scan) its offset
    uint64_t *info;   // per stream: {records, tail literal start, out end of the records, flags}
    uint32_t nb;      // blocks per stream
};
// the size of record r's tokens (literal tag + bytes, copy tag + offset) and its literal (start, length)
__device__ __forceinline__ int32_t ew_token(const uint4 *rec, int32_t r, int32_t done0, int32_t &lit_at, int32_t &L) {
    const uint4 v = rec[r];
    const int32_t dk = r == 0 ? done0 : (int32_t)(rec[r - 1].x + rec[r - 1].y);
    L = (int32_t)v.x - dk;
    lit_at = dk;
    const bool lit = (v.w & 1) != 0 || L > 0;
    int32_t ln = 0, tn = 0, on = 0;
    (void)tag_bytes(0x00, L, &ln);
    (void)tag_bytes(0x80, (int32_t)v.y, &tn);
    (void)off_bytes((int32_t)v.z, (int32_t)v.y, &on);
    if (v.y == 0) tn = on = 0;
    return (lit ? ln + L : 0) + tn + on;
}
__device__ __forceinline__ void ew_stream(const CompressArgs &A, uint64_t s, int32_t &H, int32_t &done0, bool &skip) {
    const bool spec = A.spec_mode != 0;
    skip = spec && A.spec[s].flags != 0;
    H = spec ? (int32_t)A.spec[s].op : (A.header ? (A.append_magic ? 9 : 3) : 0);
    done0 = spec ? (int32_t)A.spec[s].done : 0;
}

__global__ __launch_bounds__(256) void ke_size(CompressArgs A, const uint4 *recs, uint64_t rcap, EwBufs E) {
    __shared__ uint64_t part[4];
    const uint64_t s = blockIdx.x / E.nb;
    const uint32_t b = blockIdx.x % E.nb;
    int32_t H, done0;
    bool skip;
    ew_stream(A, s, H, done0, skip);
    const int32_t m = (int32_t)((A.out_size[s] & 0xffffffffffffull) < rcap ? (A.out_size[s] & 0xffffffffffffull) : rcap);
    if (skip || (int64_t)b * kEwRec >= m) return;
    const uint4 *rec = recs + s * rcap;
    uint64_t sum = 0;
    for (int32_t t = 0; t < kEwPer; t++) {
        const int32_t r = (int32_t)b * kEwRec + t * 256 + (int32_t)threadIdx.x;
        int32_t la, L;
        if (r < m) sum += (uint64_t)ew_token(rec, r, done0, la, L);
    }
    for (int d = 32; d >= 1; d >>= 1) sum += (uint64_t)__shfl_xor((long long)sum, d, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) E.bsum[s * E.nb + b] = part[0] + part[1] + part[2] + part[3];
}

// a wave per stream: block offsets, the header, the stream's size and status (emit_stream's rules)
__global__ __launch_bounds__(64) void ke_scan(CompressArgs A, const uint4 *recs, uint64_t rcap, EwBufs E) {
    const uint64_t s = blockIdx.x;
    const int lane = (int)threadIdx.x;
    int32_t H, done0;
    bool skip;
    ew_stream(A, s, H, done0, skip);
    if (skip) return;
    const int32_t n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    uint8_t *out = A.out + A.out_off[s];
    const int64_t cap = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    const uint64_t pr = A.out_size[s];
    const int32_t m = (int32_t)((pr & 0xffffffffffffull) < rcap ? (pr & 0xffffffffffffull) : rcap);
    int err = (int)(pr >> 48);
    const bool spec = A.spec_mode != 0;
    uint64_t *inf = E.info + 4 * s;
    if (!spec && H > cap) {  // not even the header
        if (lane == 0) {
            inf[0] = 0, inf[3] = 1;
            A.out_size[s] = 0;
            if (A.status) A.status[s] = EZ_ENOSPC;
        }
        return;
    }
    if (lane == 0 && !spec && H > 0) {
        const int32_t bsl = (int32_t)__builtin_ctzll((uint64_t)A.bs);
        const uint64_t hm = A.append_magic ? (0x141080797a616502ull << 8 | 0x80) : (0x80ull | 0x10ull << 8 | (uint64_t)bsl << 16);
        put_small(out, V16{hm, A.append_magic ? (uint64_t)bsl : 0ull}, (uint32_t)H);
    }
    const uint32_t nb = (uint32_t)((m + kEwRec - 1) / kEwRec);
    uint64_t run = (uint64_t)H;
    for (uint32_t b0 = 0; b0 < nb; b0 += 64) {
        const uint32_t b = b0 + (uint32_t)lane;
        const uint64_t v = b < nb ? E.bsum[s * E.nb + b] : 0;
        uint64_t incl = v;
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t u = (uint64_t)__shfl_up((long long)incl, d, 64);
            if (lane >= d) incl += u;
        }
        if (b < nb) E.bsum[s * E.nb + b] = run + incl - v;
        run += (uint64_t)__shfl((long long)incl, 63, 64);
    }
    if (lane != 0) return;
    const int32_t tail_at = m > 0 ? (int32_t)(recs[s * rcap + m - 1].x + recs[s * rcap + m - 1].y) : done0;
    inf[0] = (uint64_t)m, inf[1] = (uint64_t)tail_at, inf[2] = run, inf[3] = 0;
    if ((int64_t)run > cap) {  // ke_write's block at the crossing sets the size
        if (A.status) A.status[s] = err ? err : EZ_ENOSPC;
        inf[3] = 2;
        return;
    }
    uint64_t op = run;
    if (!err && tail_at < n) {  // the trailing literal (writer.go:324-329): its tag here, its bytes in ke_write
        const int32_t L = n - tail_at;
        int32_t ln = 0;
        const uint64_t lb = tag_bytes(0x00, L, &ln);
        if ((int64_t)op + ln + L > cap) {
            err = EZ_ENOSPC;
        } else {
            put_small(out + op, V16{lb, 0}, (uint32_t)ln);
            inf[3] = 4 | ((uint64_t)(op + ln) << 8);  // (the tail's bytes go to op + ln)
            op += ln + L;
        }
    }
    A.out_size[s] = op;
    if (A.status) A.status[s] = err;
}

__global__ __launch_bounds__(256) void ke_write(CompressArgs A, const uint4 *recs, uint64_t rcap, EwBufs E) {
    __shared__ uint64_t wsum[4];
    const uint64_t s = blockIdx.x / E.nb;
    const uint32_t b = blockIdx.x % E.nb;
    int32_t H, done0;
    bool skip;
    ew_stream(A, s, H, done0, skip);
    if (skip) return;
    const uint64_t *inf = E.info + 4 * s;
    if (inf[3] == 1) return;
    const int32_t m = (int32_t)inf[0];
    const uint8_t *lo = A.in, *hi = A.in + A.in_off[A.count];
    const uint8_t *p = A.in + A.in_off[s];
    uint8_t *out = A.out + A.out_off[s];
    const uint64_t cap = A.out_off[s + 1] - A.out_off[s];
    const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
    if ((int64_t)b * kEwRec < m) {
        const uint4 *rec = recs + s * rcap;
        // this thread's kEwPer consecutive records: sizes, then offsets by a block scan
        const int32_t r0 = (int32_t)b * kEwRec + (int32_t)threadIdx.x * kEwPer;
        uint64_t mine = 0;
        for (int32_t t = 0; t < kEwPer; t++) {
            int32_t la, L;
            if (r0 + t < m) mine += (uint64_t)ew_token(rec, r0 + t, done0, la, L);
        }
        uint64_t incl = mine;
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t u = (uint64_t)__shfl_up((long long)incl, d, 64);
            if (lane >= d) incl += u;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint64_t at = E.bsum[s * E.nb + b] + incl - mine;
        for (int v = 0; v < w; v++) at += wsum[v];
        for (int32_t t = 0; t < kEwPer; t++) {
            const int32_t r = r0 + t;
            const bool here = r < m;
            int32_t dk = 0, L = 0, T = 0;
            uint64_t lpos = 0;  // a long literal's output position
            bool longlit = false;
            if (here) {
                T = ew_token(rec, r, done0, dk, L);
                const uint4 v = rec[r];
                if (at + (uint64_t)T <= cap) {
                    uint8_t *d = out + at;
                    const bool lit = (v.w & 1) != 0 || L > 0;
                    int32_t ln = 0, tn = 0, on = 0;
                    const uint64_t lb = tag_bytes(0x00, L, &ln);
                    uint64_t tb = tag_bytes(0x80, (int32_t)v.y, &tn);
                    uint64_t ob = off_bytes((int32_t)v.z, (int32_t)v.y, &on);
                    if (v.y == 0) tb = ob = 0, tn = on = 0;
                    if (lit) {
                        put_small(d, V16{lb, 0}, (uint32_t)ln);
                        if (L >= kLongLit) {
                            longlit = true;
                            lpos = at + (uint64_t)ln;
                        } else {
                            copy_lane(d + ln, p + dk, L, lo, hi);
                        }
                    }
                    if (tn) {
                        const uint64_t c0 = tb | (ob << (8 * tn));
                        const uint64_t c1 = ob >> (64 - 8 * tn);
                        put_small(d + T - tn - on, V16{c0, c1}, (uint32_t)(tn + on));
                    }
                } else if (at <= cap) {  // the first token that does not fit: the output ends before it
                    A.out_size[s] = at;
                }
            }
            // long literals: the whole wave, one at a time (as emit_stream)
            for (uint64_t lm = __ballot(longlit); lm; lm &= lm - 1) {
                const int src = __builtin_ctzll(lm);
                const int32_t Ls = __shfl(L, src, 64), ds = __shfl(dk, src, 64);
                const uint64_t ts = (uint64_t)__shfl((long long)lpos, src, 64);
                for (int32_t q = 16 * lane; q < Ls; q += 16 * 64) {
                    const V16 v = ld16_in(p + ds + q, lo, hi);
                    if (q + 16 <= Ls) st16v(out + ts + q, v);
                    else put_small(out + ts + q, v, (uint32_t)(Ls - q));
                }
            }
            if (here) at += (uint64_t)T;
        }
    }
    // the trailing literal's bytes, by the stream's blocks in turn
    if (inf[3] & 4) {
        const int32_t n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        const int32_t ta = (int32_t)inf[1];
        const int32_t L = n - ta;
        const uint64_t ts = inf[3] >> 8;
        for (int64_t q = ((int64_t)b * 256 + threadIdx.x) * 16; q < L; q += (int64_t)E.nb * 256 * 16) {
            const V16 v = ld16_in(p + ta + q, lo, hi);
            if (q + 16 <= L) st16v(out + ts + q, v);
            else put_small(out + ts + q, v, (uint32_t)(L - q));
        }
    }
}

// LDS words of a stream's table (0 = this variant cannot take the batch)
template <bool T16>
uint32_t split_table_words(const CompressArgs &a) {
    if (a.ring || a.max_len == 0 || 2 * (int64_t)a.max_len > a.bs || a.hs > 4096 || a.hs < 4) return 0;
    if ((int64_t)a.max_len > (T16 ? kMaxT16 : kMaxT32)) return 0;
    const uint64_t words = T16 ? ((uint64_t)a.hs + 1) / 2 : (uint64_t)a.hs;
    return (uint32_t)((words + 3) & ~3ull);
}
template <int G, bool T16>
uint32_t split_stride(const CompressArgs &a) {
    const uint64_t tw = split_table_words<T16>(a);
    if (tw == 0) return 0;
    const uint64_t w = tw;
    if (w * 4 * (64 / G) > 160 * 1024) return 0;
    return (uint32_t)w;
}

// lanes per stream for T32: 32 when the batch has few streams (long Writes, C2: two
// waves per SIMD instead of one, 33.3 vs 34.3 ms); EZ_K1S_G32=16|32 overrides
int split_g32(uint64_t count) {
    static const int g = knob("EZ_K1S_G32", 0);
    if (g == 32 || g == 16) return g;
    return count <= 8192 ? 32 : 16;
}
std::atomic<bool> g_split_t32{false};  // ez_select_compress_kernel('S')
bool split_t32_forced() {
    static const bool v = knob("EZ_K1S_T", 0) == 32;
    return v || g_split_t32;
}

template <int G, bool T16, bool MW>
hipError_t launch_split_g(const CompressArgs &a, uint64_t *recs, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_parse<G, T16, MW>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    constexpr int S = 64 / G;
    const uint32_t stride = split_stride<G, T16>(a), tw = split_table_words<T16>(a);
    const uint64_t rcap = rec_cap(a);
    const unsigned grid = (unsigned)((a.count + S - 1) / S);
    // EZ_K1S_LDSPAD (experiments): extra LDS per block, to cap the streams resident per CU
    static const size_t pad = (size_t)knob("EZ_K1S_LDSPAD", 0);
    // wave priority (s_setprio 3) on the chain up to the candidate loads' issue: bit 0 (default),
    // bit 1 around the next window's load; EZ_K1S_PRIO=0|1|2|3 (A/B, same box: 3.58 / 3.52 /
    // 3.58 / 3.53 ms at C1)
    static const int prio = knob("EZ_K1S_PRIO", 1);
    hipLaunchKernelGGL((k1_parse<G, T16, MW>), dim3(grid), dim3(64), (size_t)stride * 4 * S + pad, st, a, stride, tw, recs, rcap,
                       prio);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const unsigned egrid = (unsigned)((a.count + 3) / 4);
    hipLaunchKernelGGL(k1_emit<false>, dim3(egrid), dim3(256), 0, st, a, (const uint64_t *)recs, rcap);
    return hipGetLastError();
}

// the lean single-Write parse (k1_lean) + the token writer; EZ_K1S_LEAN=0 takes k1_parse (A/B)
bool split_lean() {
    static const bool v = knob("EZ_K1S_LEAN", 1) != 0;
    return v;
}
// resident blocks of a k1_lean variant on the device (per process; the persistent grid)
template <int TB, bool LW, int FW, bool PERSIST, int G>
unsigned lean_resident(size_t lds) {
    static unsigned cached = 0;
    static size_t cached_lds = 0;
    if (cached == 0 || cached_lds != lds) {
        int dev = 0, cus = 0, per = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)k1_lean<TB, LW, FW, PERSIST, G>, 64, lds) != hipSuccess || per <= 0 ||
            cus <= 0)
            return 0;
        cached = (unsigned)(per * cus);
        cached_lds = lds;
    }
    return cached;
}

template <int TB, bool LW, int FW, int G = 16>
hipError_t launch_lean_v(const CompressArgs &a, uint64_t *recs, uint32_t stride, uint32_t tw, size_t lds, int prio, uint8_t *edge,
                         bool persist, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_lean<TB, LW, FW, false, G>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k1_lean<TB, LW, FW, true, G>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    constexpr uint64_t S = 64 / G;
    const uint64_t rcap = rec_cap(a);
    const uint64_t blocks = (a.count + S - 1) / S;
    const unsigned res = persist ? lean_resident<TB, LW, FW, true, G>(lds) : 0;
    if (res != 0 && blocks > res)
        hipLaunchKernelGGL((k1_lean<TB, LW, FW, true, G>), dim3(res), dim3(64), lds, st, a, stride, tw, recs, rcap, prio, edge);
    else
        hipLaunchKernelGGL((k1_lean<TB, LW, FW, false, G>), dim3((unsigned)blocks), dim3(64), lds, st, a, stride, tw, recs, rcap, prio, edge);
    return hipGetLastError();
}

static uint32_t w12_words(const CompressArgs &a) { return (uint32_t)((2 * ((a.hs + 4) / 5) + 3) & ~3ll); }  // u32 words of a 12-bit table
hipError_t launch_lean(const CompressArgs &a, uint64_t *recs, hipStream_t st) {
    // the visit by one ds_mskor (when its lane order holds); EZ_K1S_MSK=0 takes the DPP search (A/B).
    // EZ_K1S_T12=1 (A/B) puts streams of <= 4099 bytes on 12-bit tables: 6 waves per SIMD instead of
    // 5 measured the same at C1 (k1_lean 2,100 against 2,095 us), so the u16 tables stay
    static const bool msk = knob("EZ_K1S_MSK", 1) != 0 && lds_mskor_in_lane_order();
    static const bool m12 = msk && knob("EZ_K1S_T12", 0) != 0 && lds_mskor64_in_lane_order();
    const bool t12 = m12 && a.max_len <= 4099 && a.hs <= 4096;
    // 8-lane groups (8 streams per wave) for streams over 4 KiB: a window's acceptor is one of lanes
    // 0..7 in 74 % of C1's windows (6.3 of 16 lanes are visits on average), so half-width windows
    // take ~37 % fewer wave iterations; with the same streams per CU (the tables bound them) but half
    // the waves, C1 measured 2.01 -> 2.14 ms, 8 KiB streams 8.58 -> 8.11, 16 KiB 11.06 -> 9.49 (with
    // the 40-byte judgement), 64 KiB 14.10 -> 11.67.  EZ_K1S_G=8 / 16 (A/B) forces one
    static const int gw = knob("EZ_K1S_G", 0);
    const bool g8 = (gw == 8 || (gw == 0 && a.max_len > 4096)) && msk && knob("EZ_K1S_LW", 1) != 0 &&
                    (t12 ? (uint64_t)w12_words(a) * 4 * 8 <= 160 * 1024 : split_stride<8, true>(a) != 0);
    const int S = g8 ? 8 : 4;
    const uint32_t w12 = (uint32_t)((2 * ((a.hs + 4) / 5) + 3) & ~3ll);  // u32 words of a 12-bit table
    const uint32_t stride = t12 ? w12 : split_stride<16, true>(a), tw = t12 ? w12 : split_table_words<true>(a);
    const uint64_t rcap = rec_cap(a);
    // bit 0: s_setprio 3 on the chain up to the candidate loads; bit 2: the i+1 insert by lane a+1
    // (EZ_K1S_NEXT1=0 (A/B): by the acceptor, with its own hash)
    static const int prio = knob("EZ_K1S_PRIO", 1) | (knob("EZ_K1S_NEXT1", 1) ? 4 : 0);
    uint8_t *edge = (uint8_t *)(recs + a.count * rcap);
    // (the edge area's first 128 bytes: the dummy region of idle groups; its last 16: the edge-slot
    // counter and the stream queue)
    hipError_t z = hipMemsetAsync(edge, 0, 128, st);
    if (z == hipSuccess) z = hipMemsetAsync(edge + 128 + kEdgeSlots * edge_slot_bytes(a), 0, 16, st);
    if (z != hipSuccess) return z;
    // EZ_K1S_LDSPAD (experiments): extra LDS per block, to cap the streams resident per CU
    static const size_t pad = (size_t)knob("EZ_K1S_LDSPAD", 0);
    // the window's region in LDS (WinLds; C1 K1 2.18 -> 2.08 ms, A/B on one box); EZ_K1S_LW=0 (A/B) keeps it in the lanes' registers
    static const bool lw = knob("EZ_K1S_LW", 1) != 0;
    // the judgement's forward cap: 40 bytes (48-byte windows and candidates; C1 K1 2.081 -> 2.012 ms,
    // A/B on one box) for streams up to 8 KiB (16 KiB with 8-lane groups: 9.79 -> 9.49 ms), else 24
    // (16-lane groups at 16 and 64 KiB ran 9-12 % slower with 40; 8-lane at 64 KiB 11.67 against
    // 11.77); EZ_K1S_FW=40 or 24 (A/B) forces one
    static const int fw = knob("EZ_K1S_FW", 0);
    const bool w40 = fw == 40 || (fw == 0 && a.max_len <= (g8 ? 16384u : 8192u));
    // persistent groups (a stream queue); EZ_K1S_PERSIST=0 (A/B): one launch block per 4 streams
    static const bool persist = knob("EZ_K1S_PERSIST", 0) != 0;
    const size_t lds = (size_t)stride * 4 * S + (lw && msk ? (size_t)kWinLdsBytes * S : 0) + pad;
    hipError_t e;
    if (g8) {
        if (t12) e = launch_lean_v<12, true, 40, 8>(a, recs, stride, tw, lds, prio, edge, persist, st);
        else if (w40) e = launch_lean_v<16, true, 40, 8>(a, recs, stride, tw, lds, prio, edge, persist, st);
        else e = launch_lean_v<16, true, 24, 8>(a, recs, stride, tw, lds, prio, edge, persist, st);
    } else if (lw && msk) {
        if (t12) e = launch_lean_v<12, true, 24>(a, recs, stride, tw, lds, prio, edge, persist, st);
        else if (w40) e = launch_lean_v<16, true, 40>(a, recs, stride, tw, lds, prio, edge, persist, st);
        else e = launch_lean_v<16, true, 24>(a, recs, stride, tw, lds, prio, edge, persist, st);
    } else if (t12)
        e = launch_lean_v<12, false, 24>(a, recs, stride, tw, lds, prio, edge, persist, st);
    else if (msk)
        e = launch_lean_v<16, false, 24>(a, recs, stride, tw, lds, prio, edge, persist, st);
    else
        e = launch_lean_v<0, false, 24>(a, recs, stride, tw, lds, prio, edge, persist, st);
    if (e != hipSuccess) return e;
#if (EZ_EXP & 2097152)
    {  // (timing builds) waves active over time, and when each XCC's last wave ends
        const uint64_t nb = (a.count + S - 1) / S < kLeanTMax ? (a.count + S - 1) / S : kLeanTMax;
        std::vector<uint64_t> t(2 * nb);
        (void)hipStreamSynchronize(st);
        (void)hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_lean_t), 16 * nb);
        uint64_t t0 = ~0ull, t1 = 0, xe[16] = {0}, xs[16], cnt[16] = {0};
        for (int k = 0; k < 16; k++) xs[k] = ~0ull;
        for (uint64_t b = 0; b < nb; b++) {
            const uint64_t st0 = t[2 * b] & 0xffffffffffull, en = t[2 * b + 1] & 0xffffffffffull;
            const int x = (int)((t[2 * b + 1] >> 48) & 15);
            t0 = st0 < t0 ? st0 : t0;
            t1 = en > t1 ? en : t1;
            xe[x] = en > xe[x] ? en : xe[x];
            xs[x] = st0 < xs[x] ? st0 : xs[x];
            cnt[x]++;
        }
        const int bins = 40;
        std::vector<double> act(bins, 0.0);
        std::vector<uint64_t> ends(nb), lens(nb);
        for (uint64_t b = 0; b < nb; b++) {
            const uint64_t st0 = (t[2 * b] & 0xffffffffffull) - t0, en = (t[2 * b + 1] & 0xffffffffffull) - t0;
            ends[b] = en;
            lens[b] = en - st0;
            for (int k = 0; k < bins; k++) {
                const double lo = (double)(t1 - t0) * k / bins, hi = (double)(t1 - t0) * (k + 1) / bins;
                const double ov = std::min((double)en, hi) - std::max((double)st0, lo);
                if (ov > 0) act[k] += ov / (hi - lo);
            }
        }
        std::sort(ends.begin(), ends.end());
        std::sort(lens.begin(), lens.end());
        fprintf(stderr, "lean waves %llu span %.1f us; wave life p10 %.1f p50 %.1f p90 %.1f max %.1f us; end p50 %.1f p90 %.1f p99 %.1f us\n",
                (unsigned long long)nb, (t1 - t0) / 100.0, lens[nb / 10] / 100.0, lens[nb / 2] / 100.0, lens[nb * 9 / 10] / 100.0, lens[nb - 1] / 100.0,
                ends[nb / 2] / 100.0, ends[nb * 9 / 10] / 100.0, ends[nb * 99 / 100] / 100.0);
        fprintf(stderr, "lean active waves per bin of %.1f us:", (t1 - t0) / 100.0 / bins);
        for (int k = 0; k < bins; k++) fprintf(stderr, " %.0f", act[k]);
        fprintf(stderr, "\nlean per xcc (waves, first start, last end, us):");
        for (int x = 0; x < 16; x++)
            if (cnt[x]) fprintf(stderr, " [%d %llu %.1f %.1f]", x, (unsigned long long)cnt[x], (xs[x] - t0) / 100.0, (xe[x] - t0) / 100.0);
        fprintf(stderr, "\n");
    }
#endif
#if (EZ_EXP & 65536)
    {  // (experiment builds) the acceptor-lane histogram of this launch
        unsigned long long hst[18];
        (void)hipStreamSynchronize(st);
        (void)hipMemcpyFromSymbol(hst, HIP_SYMBOL(g_lean_hist), sizeof hst);
        unsigned long long tot = 0, vis = 0;
        for (int t = 0; t < 18; t++) tot += hst[t];
        for (int t = 1; t < 17; t++) vis += hst[t] * (unsigned long long)t;
        vis += hst[0] * 16ull;
        fprintf(stderr, "lean windows %llu (no accept %llu); visited lanes %.3f of 16; by acceptor lane:", tot, hst[0], (double)vis / (double)tot);
        for (int t = 1; t < 17; t++) fprintf(stderr, " %.3f", (double)hst[t] / (double)tot);
        fprintf(stderr, "\n");
        memset(hst, 0, sizeof hst);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lean_hist), hst, sizeof hst);
    }
#endif
    const unsigned egrid = (unsigned)((a.count + 3) / 4);
    hipLaunchKernelGGL(k1_emit<false>, dim3(egrid), dim3(256), 0, st, a, (const uint64_t *)recs, rcap);
    return hipGetLastError();
}

// The property T16 relies on, checked once per process on the device:
// same-address ds_write_b16 of one wave instruction land in ascending lane
// order (the highest lane's value stays).
__global__ void k_lds_store_order(uint32_t *res) {
    __shared__ uint16_t t[8];
    const uint32_t l = threadIdx.x;
    if (l < 8) t[l] = 0;
    __syncthreads();
    t[l & 7] = (uint16_t)(l + 1);
    __syncthreads();
    if (l < 8 && t[l] != (uint16_t)(56 + l + 1)) atomicAdd(res, 1u);
}

// the same for 32-bit stores (k1_long's u32 table)
__global__ void k_lds_store_order32(uint32_t *res) {
    __shared__ uint32_t t[8];
    const uint32_t l = threadIdx.x;
    if (l < 8) t[l] = 0;
    __syncthreads();
    t[l & 7] = l + 1;
    __syncthreads();
    if (l < 8 && t[l] != 56 + l + 1) atomicAdd(res, 1u);
}

// The property k1_lean<16> relies on, checked once per process on the device: same-word
// ds_mskor_rtn_b32 of one wave instruction apply in ascending lane order (each lane reads the
// entry as the latest earlier lane on it left it), on both halves of a word.
__global__ void k_lds_mskor_order(uint32_t *res) {
    __shared__ uint16_t t[8];
    const uint32_t l = threadIdx.x;
    if (l < 8) t[l] = 0;
    __syncthreads();
    const uint32_t e = (l * 5 + (l >> 3)) & 7;
    const uint32_t got = lds_mskor16(t, e, l + 1);
    uint32_t want = 0, last = 0;
    for (uint32_t k = 0; k < 64; k++) {
        const uint32_t ek = (k * 5 + (k >> 3)) & 7;
        if (ek == e && k < l) want = k + 1;
        if (l < 8 && ek == l) last = k + 1;
    }
    __syncthreads();
    if (got != want || (l < 8 && t[l] != last)) atomicAdd(res, 1u);
}

// the same for ds_mskor_rtn_b64 on 12-bit fields (k1_lean<12>): five entries per word
__global__ void k_lds_mskor64_order(uint32_t *res) {
    __shared__ uint64_t t[2];
    const uint32_t l = threadIdx.x;
    if (l < 2) t[l] = 0;
    __syncthreads();
    const uint32_t e = (l * 7 + (l >> 3)) % 10;  // entries 0 - 9: both words, every field
    const uint32_t got = lds_mskor12(t, e, l + 1);
    uint32_t want = 0;
    for (uint32_t k = 0; k < l; k++)
        if ((k * 7 + (k >> 3)) % 10 == e) want = k + 1;
    __syncthreads();
    if (got != want) atomicAdd(res, 1u);
    if (l < 10) {  // the final entries, and a put without return after them
        uint32_t last = 0;
        for (uint32_t k = 0; k < 64; k++)
            if ((k * 7 + (k >> 3)) % 10 == l) last = k + 1;
        const uint32_t sh = 12u * (l % 5);
        if (((uint32_t)(t[l / 5] >> sh) & 0xfffu) != last) atomicAdd(res, 1u);
    }
    __syncthreads();
    if (l < 10) lds_put12(t, l, 100 + l);
    __syncthreads();
    if (l < 10 && ((uint32_t)(t[l / 5] >> (12u * (l % 5))) & 0xfffu) != 100 + l) atomicAdd(res, 1u);
}

// The property T32 relies on, checked once per process on the device: same-address LDS
// exchanges of one wave instruction apply in ascending lane order (lane l reads what lane l-4
// wrote).  If it ever fails, K1s-T32 is not used.
__global__ void k_lds_order(uint32_t *res) {
    __shared__ uint32_t t[4];
    const uint32_t l = threadIdx.x;
    if (l < 4) t[l] = 0;
    __syncthreads();
    const uint32_t old = atomicExch(&t[l & 3], l + 1);
    const uint32_t want = l < 4 ? 0 : l - 3;
    if (old != want) atomicAdd(res, 1u);
}

// one 64-lane probe kernel on a private stream; true when it reports no violation
bool lds_probe(void (*kern)(uint32_t *)) {
    uint32_t *d = nullptr, h = 1;
    hipStream_t st = nullptr;
    bool ok = false;
    if (hipMalloc(&d, sizeof(uint32_t)) != hipSuccess) return false;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) {
        if (hipMemsetAsync(d, 0, sizeof(uint32_t), st) == hipSuccess) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, st, d);
            if (hipGetLastError() == hipSuccess && hipMemcpyAsync(&h, d, sizeof(uint32_t), hipMemcpyDeviceToHost, st) == hipSuccess &&
                hipStreamSynchronize(st) == hipSuccess)
                ok = h == 0;
        }
        (void)hipStreamDestroy(st);
    }
    (void)hipFree(d);
    return ok;
}

}  // namespace

bool lds_exchange_in_lane_order() {
    static const bool ok = lds_probe(k_lds_order);
    return ok;
}

bool lds_store_in_lane_order() {
    static const bool ok = lds_probe(k_lds_store_order);
    return ok;
}

bool lds_mskor_in_lane_order() {
    static const bool ok = lds_probe(k_lds_mskor_order);
    return ok;
}

bool lds_mskor64_in_lane_order() {
    static const bool ok = lds_probe(k_lds_mskor64_order);
    return ok;
}

bool lds_store32_in_lane_order() {
    static const bool ok = lds_probe(k_lds_store_order32);
    return ok;
}

// K1L: long fresh single-Write streams (table <= 4096 entries, positions < 2^31, LDS lane order);
// EZ_K1L=0 turns it off (A/B: K1x's continuation on the general kernel)
bool long_applies(const CompressArgs &a) {
    static const bool off = knob("EZ_K1L", 1) == 0;
    return !off && !a.ring && !a.write_idx && a.start == 0 && a.header && a.hs <= 4096 && a.hs >= 4 && a.max_len > 0 &&
           a.max_len < (1ull << 31) && lds_store32_in_lane_order();
}
// K1c geometry: chunks of C positions, parses from W positions before a chunk to O past the next one's
// start (EZ_K1C_C / _W / _O, experiment builds); event words and records per chunk
struct KcGeom {
    int32_t C, W, O, kmax, logcap;
    uint32_t rcap_c;
};
static KcGeom kc_geom(const CompressArgs &a) {
    // (W: the chunk's warm-up before its start, parsed with a zero table and not kept.  8 KiB instead of
    // 1 KiB: fewer first-pass reads of entries older than the warm-up, so fewer streams need another
    // pass -- 1,024 x 1 MiB logs K1 73.0 -> 67.5 ms, 1,024 x 256 KiB 25.9 -> 22.6 ms, C4s unchanged)
    // (C: positions per chunk, the power of two that leaves about 8,192 chunks in the batch -- two
    // waves per SIMD -- within 32 .. 128 KiB: fewer chunk boundaries to stitch and prove where the
    // chunks still fill the chip.  1,024 x 1 MiB logs: 73.0 (32 KiB) / 60.8 (64) / 48.9 (128) /
    // 74.9 ms (256); 1,024 x 256 KiB: 22.4 (32) / 26.4 ms (64); C4s: 21.2 (32) / 28.9 ms (64))
    static const int32_t Ck = knob("EZ_K1C_C", 0), W = knob("EZ_K1C_W", 8192), O = knob("EZ_K1C_O", 1024);
    int32_t C = Ck;
    if (C <= 0) {
        const uint64_t per = (uint64_t)a.count * a.max_len / 8192;
        C = 32768;
        while (C < 131072 && (uint64_t)C * 2 <= per) C *= 2;
    }
    KcGeom g;
    g.C = C, g.W = W, g.O = O;
    g.kmax = (int32_t)((a.max_len + (uint64_t)C - 1) / (uint64_t)C);
    g.logcap = W + C + O + 2048;  // (re-visits: an accept short of x + 2 parses positions again)
    g.rcap_c = (uint32_t)((C + O + 64) / 6 + 4);
    return g;
}
static uint64_t up256(uint64_t x) { return (x + 255) & ~255ull; }
struct KcLay {
    uint64_t crec, log, meta, seg, sinfo, ft, cstart, t0, cfail, left, total;
};
static KcLay kc_layout(const CompressArgs &a, const KcGeom &g) {
    const uint64_t nc = a.count * (uint64_t)g.kmax;
    KcLay l;
    uint64_t o = 0;
    l.crec = o, o += up256(nc * g.rcap_c * sizeof(uint4));
    l.log = o, o += up256(nc * (uint64_t)g.logcap * sizeof(uint2));
    l.meta = o, o += up256(nc * sizeof(uint4));
    l.seg = o, o += up256(nc * kKcSegWords * 4);
    l.sinfo = o, o += up256(a.count * kKcInfo * 4);
    l.ft = o, o += up256(nc * 2 * (uint64_t)a.hs * 4);
    l.cstart = o, o += up256(nc * 4);
    l.t0 = o, o += up256(nc * (uint64_t)a.hs * 4);
    l.cfail = o, o += up256(nc * 4);
    l.left = o, o += 256;
    l.total = o;
    return l;
}

// the chip-wide token writer's workspace (after K1L's records) and its launch: batches of at most
// 1,024 streams (C4s 36.9 -> 30.9 ms; C2's 4,096 streams keep k1_emit<true>, one wave per stream:
// 25.0 against 28.0 ms); EZ_K1E_WIDE=0 / 1 (experiment builds) forces either
static uint32_t ew_blocks(const CompressArgs &a) { return (uint32_t)((rec_cap(a) + kEwRec - 1) / kEwRec); }
static uint64_t ew_bytes(const CompressArgs &a) { return up256(a.count * ew_blocks(a) * 8) + up256(a.count * 32); }
static hipError_t launch_emit_wide(const CompressArgs &a, const uint4 *recs, uint64_t rcap, uint8_t *ws, hipStream_t st) {
    static const int wk = knob("EZ_K1E_WIDE", -1);
    const bool wide = wk < 0 ? a.count <= 1024 : wk != 0;
    if (!wide) {
        hipLaunchKernelGGL(k1_emit<true>, dim3((unsigned)((a.count + 3) / 4)), dim3(256), 0, st, a, (const uint64_t *)recs, rcap);
        return hipGetLastError();
    }
    EwBufs E;
    E.nb = ew_blocks(a);
    E.bsum = (uint64_t *)ws;
    E.info = (uint64_t *)(ws + up256(a.count * E.nb * 8));
    const unsigned g = (unsigned)(a.count * E.nb);
    hipLaunchKernelGGL(ke_size, dim3(g), dim3(256), 0, st, a, recs, rcap, E);
    hipLaunchKernelGGL(ke_scan, dim3((unsigned)a.count), dim3(64), 0, st, a, recs, rcap, E);
    hipLaunchKernelGGL(ke_write, dim3(g), dim3(256), 0, st, a, recs, rcap, E);
    return hipGetLastError();
}

// K1c takes K1L's batches of at most 1,024 streams at least two chunks long: there K1L runs at most
// one wave per SIMD, each a latency chain over a whole stream (C4s, 64 x 4 MiB: K1 245 -> 31 ms;
// 1,024 x 1 MiB: 115 -> 103 ms); C2's 4,096 streams keep K1L (25 ms against 64 for K1c's passes,
// which are bound by the parse's instructions there).  EZ_K1C=0 / EZ_K1C_MAXCOUNT (experiment
// builds) or a forced 'l': K1L alone
// K1c's workspace is sized by the batch's longest stream (count x kmax chunks of about 400 KB: ~12 x
// count x max_len); a skewed batch (one long stream among many short ones) would ask for far more than
// its bytes, so above kK1cMaxBytes the batch takes K1L alone, as it does when the C-ABI cannot
// allocate it (no_k1c)
constexpr uint64_t kK1cMaxBytes = (uint64_t)24 << 30;
bool chunk_applies(const CompressArgs &a) {
    static const bool on = knob("EZ_K1C", 1) != 0;
    static const uint64_t most = (uint64_t)knob("EZ_K1C_MAXCOUNT", 1024);
    return on && !a.no_k1c && !compress_forced_long() && long_applies(a) && a.count <= most &&
           a.max_len >= 2 * (uint64_t)kc_geom(a).C && kc_layout(a, kc_geom(a)).total <= kK1cMaxBytes;
}

// verdict counts of K1c batches while counting is on (ez_compress_k1c_stats; the multi-device batches
// launch from several host threads)
static std::mutex g_kc_mu;
static bool g_kc_stats_on = false;
static uint64_t g_kc_stats[6] = {0, 0, 0, 0, 0, 0};
void k1c_stats(int enable, uint64_t *out) {
    std::lock_guard<std::mutex> lk(g_kc_mu);
    if (out)
        for (int t = 0; t < 6; t++) out[t] = g_kc_stats[t];
    if (enable)
        for (int t = 0; t < 6; t++) g_kc_stats[t] = 0;
    g_kc_stats_on = enable != 0;
}
static bool kc_stats_on() {
    std::lock_guard<std::mutex> lk(g_kc_mu);
    return g_kc_stats_on;
}

static hipError_t launch_chunk(const CompressArgs &a, uint8_t *recs, hipStream_t st) {
    const KcGeom g = kc_geom(a);
    const KcLay l = kc_layout(a, g);
    const uint64_t rcap = rec_cap(a);
    uint8_t *ews = recs + up256(a.count * rcap * sizeof(WideRec));
    uint8_t *base = ews + ew_bytes(a);
    KcBufs B;
    B.crec = (uint4 *)(base + l.crec);
    B.log = (uint2 *)(base + l.log);
    B.meta = (uint4 *)(base + l.meta);
    B.seg = (uint32_t *)(base + l.seg);
    B.sinfo = (uint32_t *)(base + l.sinfo);
    B.ft = (uint32_t *)(base + l.ft);
    B.cstart = (int32_t *)(base + l.cstart);
    B.t0 = (uint32_t *)(base + l.t0);
    B.cfail = (uint32_t *)(base + l.cfail);
    B.C = g.C, B.W = g.W, B.O = g.O, B.kmax = g.kmax, B.logcap = g.logcap, B.rcap_c = g.rcap_c;
    const uint64_t nc = a.count * (uint64_t)g.kmax;
    hipError_t e = hipSuccess;
    static const bool lw = knob("EZ_K1L_LW", 1) != 0;
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)kc_parse<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)kc_parse<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k1_long<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k1_long<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const size_t lds = (size_t)4 * (size_t)a.hs * 4 + (lw ? (size_t)4 * kWinLdsBytes : 0);
    const unsigned pgrid = (unsigned)((nc + 3) / 4);
    // the first pass's guessed tables (EZ_K1C_GUESS=1, experiment builds; off: C4s 31.5 against 30.9 ms,
    // 1,024 x 1 MiB 102.5 against 102.7 -- the reads it fixes are not the ones that fail a stream)
    static const bool guess = knob("EZ_K1C_GUESS", 0) != 0;
    B.guess = guess ? 1 : 0;
    if (guess) {
        hipLaunchKernelGGL(kc_last, dim3((unsigned)nc), dim3(256), (size_t)2 * (size_t)a.hs * 4, st, a, B);
        hipLaunchKernelGGL(kc_guess, dim3((unsigned)((a.count * (uint64_t)a.hs + 255) / 256)), dim3(256), 0, st, a, B);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // passes (EZ_K1C_PASSES, experiment builds; 1 = the speculative chunks alone): from the third on,
    // the host reads how many streams are still failed and stops at none (C2 / C4s: all proven after
    // 4 passes of 32 KiB chunks)
    static const int passes = knob("EZ_K1C_PASSES", 12);
    uint32_t *left = (uint32_t *)(base + l.left);
    static const bool diag = knob("EZ_K1C_DIAG", 0) != 0;
    const bool stats = kc_stats_on();
    for (int pass = 1; pass <= passes; pass++) {
        if (lw) hipLaunchKernelGGL(kc_parse<true>, dim3(pgrid), dim3(64), lds, st, a, B, pass);
        else hipLaunchKernelGGL(kc_parse<false>, dim3(pgrid), dim3(64), lds, st, a, B, pass);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(kc_stitch, dim3((unsigned)a.count), dim3(64), 0, st, a, B, rcap, pass);
        hipLaunchKernelGGL(kc_gather, dim3((unsigned)nc), dim3(256), 0, st, a, B, (uint4 *)recs, rcap, pass);
        hipLaunchKernelGGL(kc_v1, dim3((unsigned)nc), dim3(64), (size_t)2 * (size_t)a.hs * 4, st, a, B, pass);
        hipLaunchKernelGGL(kc_v2, dim3((unsigned)((a.count * (uint64_t)a.hs + 255) / 256)), dim3(256), 0, st, a, B, pass);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        bool stop = false;
        if (pass >= 3 && pass < passes) {
            uint32_t h_left = 0;
            if ((e = hipMemsetAsync(left, 0, 4, st)) != hipSuccess) return e;
            hipLaunchKernelGGL(kc_count, dim3((unsigned)((a.count + 255) / 256)), dim3(256), 0, st, a, B, left);
            if ((e = hipMemcpyAsync(&h_left, left, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            stop = h_left == 0;
        }
        const bool final = stop || pass == passes;
        if (!(diag || (stats && final))) {
            if (stop) break;
            continue;
        }
        // (tests, experiment builds) the verdicts: wait for them and count
        std::vector<uint32_t> si(a.count * kKcInfo);
        std::vector<SpecState> sp(a.spec_mode != 0 ? a.count : 0);
        if ((e = hipMemcpyAsync(si.data(), B.sinfo, si.size() * 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if (!sp.empty() && (e = hipMemcpyAsync(sp.data(), a.spec, sp.size() * sizeof(SpecState), hipMemcpyDeviceToHost, st)) != hipSuccess)
            return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        uint64_t f[16] = {0}, segs = 0;
        for (uint64_t s = 0; s < a.count; s++) {
            if (!sp.empty() && sp[s].flags != 0) continue;  // (finished by K1x)
            f[si[kKcInfo * s + 1] & 15]++;
            segs += si[kKcInfo * s];
        }
        const uint64_t v[6] = {f[0], f[kKcFailChunk], f[kKcFailSync], f[kKcFailJudge], f[kKcFailCap], segs};
        if (stats && final) {
            std::lock_guard<std::mutex> lk(g_kc_mu);
            for (int t = 0; t < 6; t++) g_kc_stats[t] += v[t];
        }
        if (diag)
            fprintf(stderr, "K1c pass %d: %llu streams x %d chunks; proven %llu, chunk %llu, sync %llu, judge %llu, cap %llu; segments %llu\n",
                    pass, (unsigned long long)a.count, g.kmax, (unsigned long long)v[0], (unsigned long long)v[1], (unsigned long long)v[2],
                    (unsigned long long)v[3], (unsigned long long)v[4], (unsigned long long)v[5]);
#if (EZ_EXP & 65536)
        if (diag) {
            unsigned long long d[8];
            (void)hipMemcpyFromSymbol(d, HIP_SYMBOL(g_kc_diag), sizeof d);
            fprintf(stderr, "  reads rechecked %llu, failing %llu: zero read %llu, right older %llu, right newer %llu, at an accept %llu, right before the chunk's warm-up %llu\n",
                    d[0], d[1], d[2], d[3], d[4], d[5], d[6]);
            memset(d, 0, sizeof d);
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kc_diag), d, sizeof d);
        }
#endif
        if (stop) break;
    }
    // the fallback: K1L from the start (or K1x's state) for the streams K1c could not prove
    const uint32_t S = a.count <= 256 ? 1u : 4u;
    const size_t llds = (size_t)S * (size_t)a.hs * 4 + (lw ? (size_t)4 * kWinLdsBytes : 0);
    const unsigned lgrid = (unsigned)((a.count + S - 1) / S);
    if (lw) hipLaunchKernelGGL(k1_long<true>, dim3(lgrid), dim3(64), llds, st, a, (uint32_t)a.hs, (uint4 *)recs, rcap, S, B.sinfo + 1, kKcInfo);
    else hipLaunchKernelGGL(k1_long<false>, dim3(lgrid), dim3(64), llds, st, a, (uint32_t)a.hs, (uint4 *)recs, rcap, S, B.sinfo + 1, kKcInfo);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return launch_emit_wide(a, (const uint4 *)recs, rcap, ews, st);
}

// [K1L's records][the token writer's workspace][K1c's workspace]
uint64_t long_scratch_bytes(const CompressArgs &a) {
    const uint64_t r = up256(a.count * rec_cap(a) * sizeof(WideRec)) + ew_bytes(a);
    return chunk_applies(a) ? r + kc_layout(a, kc_geom(a)).total : r;
}

hipError_t launch_long(const CompressArgs &a, uint8_t *recs, hipStream_t st) {
    if (chunk_applies(a)) return launch_chunk(a, recs, st);
    // streams per wave: one for batches of a few hundred streams (C4s' 64: K1 361 -> 291 ms), else 4
    // (each wave's instructions serve 4 streams; C2's 4,096 streams: 32.3 ms at 4, 33.5 at 2, 38.2 at
    // 1; 1,024 x 1 MiB compressed at 7.3 GiB/s at 1 against 7.6 at 4); EZ_K1L_SPW=1|2|4 overrides
    static const uint32_t spw_env = (uint32_t)knob("EZ_K1L_SPW", 0);
    const uint32_t S = spw_env == 1 || spw_env == 2 || spw_env == 4 ? spw_env : (a.count <= 256 ? 1u : 4u);
    const uint64_t rcap = rec_cap(a);
    // the window's region in LDS (WinLdsL; C2 K1 25.8 -> 24.9 ms, C4s 254 -> 246); EZ_K1L_LW=0 (A/B) keeps it in registers
    static const bool lw = knob("EZ_K1L_LW", 1) != 0;
    const size_t lds = (size_t)S * (size_t)a.hs * 4 + (lw ? (size_t)4 * kWinLdsBytes : 0);
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_long<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k1_long<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const unsigned grid = (unsigned)((a.count + S - 1) / S);
    if (lw) hipLaunchKernelGGL(k1_long<true>, dim3(grid), dim3(64), lds, st, a, (uint32_t)a.hs, (uint4 *)recs, rcap, S, nullptr, 0u);
    else hipLaunchKernelGGL(k1_long<false>, dim3(grid), dim3(64), lds, st, a, (uint32_t)a.hs, (uint4 *)recs, rcap, S, nullptr, 0u);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_emit_wide(a, (const uint4 *)recs, rcap, recs + up256(a.count * rcap * sizeof(WideRec)), st);
}

// K1L for one Write on a Writer handle (writer_run): single Writes of 16 bytes .. 64 MiB on
// handles with version 0, a table of at most 4096 entries, bs <= 2^26, positions below 2^32
// (the uint32 table values stay exact: a Write across 2^32 takes the general kernel)
bool long_ring_applies(const CompressArgs &a) {
    return a.count == 1 && a.ring && !a.write_idx && a.ver == 0 && a.hs <= 4096 && a.hs >= 4 && a.bs <= (1ll << 26) &&
           a.max_len >= 16 && a.max_len < (1ull << 26) && a.start >= 0 && (uint64_t)a.start + a.max_len <= (1ull << 32) &&
           lds_store32_in_lane_order();
}
uint64_t long_ring_scratch_bytes(const CompressArgs &a) { return rec_cap(a) * sizeof(WideRec); }
hipError_t launch_long_ring(const CompressArgs &a, uint8_t *recs, hipStream_t st) {
    const uint64_t rcap = rec_cap(a);
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_long_ring<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    // Writes of up to kLdsWrite bytes: the Write and the ring's last bytes in LDS, the token writer in
    // the same kernel
    if (a.max_len <= (uint64_t)kLdsWrite) {
        hipLaunchKernelGGL(k1_long_ring<true>, dim3(1), dim3(256), (size_t)a.hs * 4 + kLdsRing + kLdsWrite + 64, st, a, (uint4 *)recs,
                           rcap);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k1_long_ring<false>, dim3(1), dim3(256), (size_t)a.hs * 4, st, a, (uint4 *)recs, rcap);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k1_emit<true>, dim3(1), dim3(256), 0, st, a, (const uint64_t *)recs, rcap);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (a.max_len <= (uint64_t)kLdsWrite) return hipSuccess;  // (k1_long_ring<true> stored the ring)
    const uint64_t n = a.max_len;
    const uint64_t blocks = (n < (uint64_t)a.bs ? n : (uint64_t)a.bs) / 256 / 16 + 1;
    hipLaunchKernelGGL(k1_ring_store, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), 0, st, a);
    return hipGetLastError();
}

// the table the batch takes: 16 (T16), 32 (T32) or 0 (K1s cannot take it)
static int split_table(const CompressArgs &a) {
    if (a.count > (1ull << 31)) return 0;
    if (!split_t32_forced() && split_stride<16, true>(a) != 0 && lds_store_in_lane_order()) return 16;
    if (split_stride<16, false>(a) != 0 && lds_exchange_in_lane_order()) return 32;
    return 0;
}

void select_split_table(bool t32) { g_split_t32 = t32; }

uint32_t split_stride_words(const CompressArgs &a) { return split_table(a) != 0 ? 1u : 0u; }

// records (8 bytes per record slot entry), then k1_lean's edge area
static bool split_takes_long(const CompressArgs &a) {
    return !a.write_idx && !split_t32_forced() && split_table(a) != 16 && long_applies(a);
}
uint64_t split_scratch_words(const CompressArgs &a) {
    if (split_takes_long(a)) return (long_scratch_bytes(a) + 3) / 4;
    return a.count * rec_cap(a) * 2 + (edge_area_bytes(a) + 3) / 4;
}

// K1s routing: one Write per stream on the u16 table -> k1_lean (EZ_K1S_LEAN=0: k1_parse, the
// previous form, kept for A/B); one Write per stream on the u32 table (streams over 64 KiB) -> K1L;
// multi-Write streams and forced T32 -> k1_parse, 32 lanes per stream for batches of few streams
hipError_t launch_compress_split(const CompressArgs &a, uint32_t *scratch, hipStream_t st) {
    uint64_t *recs = (uint64_t *)scratch;
    const int T = split_table(a);
    if (a.write_idx) {
        if (T == 16) return launch_split_g<16, true, true>(a, recs, st);
        if (split_g32(a.count) == 32) return launch_split_g<32, false, true>(a, recs, st);
        return launch_split_g<16, false, true>(a, recs, st);
    }
    if (T == 16) return split_lean() ? launch_lean(a, recs, st) : launch_split_g<16, true, false>(a, recs, st);
    // single Writes on the u32 table (streams over 64 KiB, C2): K1L, the lean parse (C2 31.5 vs 33.7 ms)
    if (split_takes_long(a)) return launch_long(a, (uint8_t *)scratch, st);
    if (split_g32(a.count) == 32) return launch_split_g<32, false, false>(a, recs, st);
    return launch_split_g<16, false, false>(a, recs, st);
}

}  // namespace ez
