// ez_compress_tile.hip — K1t: batch compression of fresh streams, G lanes per
// stream, 64/G streams per wave, hash table and input staged in LDS.
//
// Writer.Write (writer.go:206-337) for a fresh stream (SURVEY §8 unit of work;
// 2n <= block, so the ring is the linear history with zeros from `done` on:
// no far skip, no cut, no trim 1), judged G positions at a time like K1grp,
// with the table traffic cut to one instruction per window:
//
//   * Visit = `pos := ht[h]; ht[h] = start+i` (writer.go:214-217) for the G
//     positions of the window is ONE `ds_wrxchg_rtn_b32`: same-address LDS
//     atomics of one wave instruction are applied in ascending lane order
//     (measured on gfx950, tools/mb_ldsatomic.hip; guarded by a GPU test), so
//     lane j receives exactly what Go's sequential visits would read — the
//     latest earlier position of the window with its hash, else the table.
//   * Positions after the window's first accepting lane are not visited in
//     Go; their inserts are undone with one `ds_min_u32` of the values they
//     read (in a window whose start lies above every position in the table,
//     the smallest value read per hash is the one before the first undone
//     insert).  Windows that start at or below the highest inserted position
//     (after a zero run ends before the visiting position and `i` moves back,
//     writeZeros :407-439) are judged one position at a time, where the
//     exchange alone is exact.
//   * Acceptance is judged with 8-byte capped match lengths (exact: the
//     threshold minCopyChunk = 6 is below the cap, writer.go:119, 301); only
//     an accepted match whose capped count saturates is extended cooperatively.
//   * Tokens are written as 4-byte chunks per lane: literal bytes from LDS
//     with the tag and copy bytes merged in (Encoder.Tag/Offset :537-597).
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_k1_common.h"

#include <type_traits>

#ifndef EZ_EXP
#define EZ_EXP 0  // timing experiments only: bit 0 no token stores, bit 1 no exact extension
#endif

namespace ez {
namespace {
using namespace k1;

// EZ_EXP bit 2: cycle profile of the window loop (s_memtime between section
// marks, printed by lane 0 of the first blocks); diagnostic builds only
#if (EZ_EXP & 4)
#define EZ_PROF_MARK(k)                                            \
    do {                                                           \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();          \
        prof[(k) == 0 ? 7 : (k) - 1] += t_ - prof_t;               \
        prof_t = t_;                                               \
        if ((k) == 0) prof_it++;                                   \
    } while (0)
#define EZ_PROF_DUMP()                                                                                         \
    do {                                                                                                       \
        if (blockIdx.x < 3 && lane == 0)                                                                       \
            printf("prof blk %u it %llu: visit %llu judge %llu ballot %llu ext %llu enc %llu emit %llu fin %llu loop %llu\n", \
                   blockIdx.x, (unsigned long long)prof_it, (unsigned long long)prof[0], (unsigned long long)prof[1], \
                   (unsigned long long)prof[2], (unsigned long long)prof[3], (unsigned long long)prof[4],            \
                   (unsigned long long)prof[5], (unsigned long long)prof[6], (unsigned long long)prof[7]);           \
    } while (0)
#else
#define EZ_PROF_MARK(k) do {} while (0)
#define EZ_PROF_DUMP() do {} while (0)
#endif

typedef uint32_t __attribute__((aligned(1))) u32_ua;

// bytes [k, k+4) of the 16-byte little-endian value (lo, hi), 0 <= k <= 12
__device__ __forceinline__ uint32_t bytes4_at(uint64_t lo, uint64_t hi, int32_t k) {
    const uint64_t w = k < 8 ? ((lo >> (8 * k)) | (k == 0 ? 0ull : hi << (64 - 8 * k))) : (hi >> (8 * (k - 8)));
    return (uint32_t)w;
}

// The group writes T token bytes at out + op: bytes [0, e1) are the literal
// tag (lb), [e1, e2) the literal p[lit0 ...], [e2, T) the copy token
// (cb, ch2).  4 bytes per lane per step; a chunk's bytes past T are
// overwritten by the next emission (or lie past the stream's end inside its
// slot), never past cap.
template <int G, class SRC>
__device__ __forceinline__ void emit(const SRC &P, uint8_t *out, int32_t op, int32_t cap, bool act, int lj, int32_t T,
                                     int32_t e1, int32_t e2, uint64_t lb, int32_t lit0, uint64_t cb, uint64_t ch2) {
    for (int32_t q0 = 4 * lj; __ballot(act && q0 < T) != 0; q0 += 4 * G) {
        if (act && q0 < T) {
            uint32_t v = P.u32(lit0 + q0 - e1);  // the literal's bytes (lit0 - 5 >= -8: staging pads)
            if (q0 < e1) {
                const int32_t k = e1 - q0;
                const uint32_t m = k >= 4 ? 0xffffffffu : ((1u << (8 * k)) - 1);
                v = (v & ~m) | ((uint32_t)(lb >> (8 * q0)) & m);
            }
            if (q0 + 4 > e2) {
                const int32_t d = q0 - e2;
                const uint32_t tv = d >= 0 ? bytes4_at(cb, ch2, d) : (uint32_t)(cb << (8 * -d));
                const uint32_t m = d >= 0 ? 0xffffffffu : ~((1u << (8 * -d)) - 1);
                v = (v & ~m) | (tv & m);
            }
            uint8_t *d = out + op + q0;
            if (op + q0 + 4 <= cap) {
                *(u32_ua *)d = v;
            } else {
                for (int32_t t = 0; t < 4 && op + q0 + t < cap; t++) d[t] = (uint8_t)(v >> (8 * t));
            }
        }
    }
}

// GIN: the input is read from HBM through the caches (LDS holds only the
// tables, 2.5 waves per SIMD at hs = 1024); else it is staged in LDS too.
template <int G, bool GIN>
__global__ __launch_bounds__(64) void k1_tile(CompressArgs A, uint32_t stride_words) {
    using SRC = typename std::conditional<GIN, GW, PW>::type;
    constexpr int S = 64 / G;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / G, lj = lane % G;
    const int32_t hs = (int32_t)A.hs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));

    // per-stream LDS: [ht u32 x hs][input words: 2 zero words, the stream, 5 zero words (!GIN)]
    uint32_t *base = (uint32_t *)smem + (uint32_t)g * stride_words;
    uint32_t *ht = base;
    uint32_t *pw = base + hs;

    const uint64_t s = (uint64_t)blockIdx.x * S + g;
    const bool have = s < A.count;
    int32_t n = 0;
    const uint8_t *gp = A.in;
    if (have) {
        n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
        gp = A.in + A.in_off[s];
    }
    SRC P;
    if constexpr (GIN) {
        P.p = gp;
        P.blo = A.in;
        P.bhi = A.in + A.in_off[A.count];
    } else {
        const uint32_t r = (uint32_t)((uintptr_t)gp & 3);
        const uint32_t *gw = (const uint32_t *)(gp - r);
        const int32_t nw = have ? (int32_t)((r + (uint32_t)n + 3) >> 2) : 0;
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
    }
    // ht zero = stream position 0 (writer.go:183, A.2)
    for (int32_t k = 4 * lj; k < hs; k += 4 * G) *(uint4 *)(ht + k) = make_uint4(0, 0, 0, 0);

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

    int32_t i = 0, done = 0, hiw = -1;  // hiw: highest position in the table
    bool live = have && n >= 4 && !err;
    int32_t guard = 4 * n + 64;
#if (EZ_EXP & 4)
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prof_t = __builtin_amdgcn_s_memtime(), prof_it = 0;
#endif
    while (__ballot(live) != 0) {
        if (live && --guard < 0) { err = EZ_ESTUCK; live = false; }
        int32_t nvalid = n - 3 - i < G ? n - 3 - i : G;
        if (i <= hiw) nvalid = 1;  // not monotone: one position per window
        const int32_t x = i + lj;
        const bool valid = live && lj < nvalid;

        EZ_PROF_MARK(0);
        // ---- 1. visit: hash, exchange (lookup + insert in lane order)
        uint64_t pxb = 0, pxf = 0;
        uint32_t h = 0;
        int32_t cand = 0;
        if (valid) {
            P.around(x, pxb, pxf);
            h = ((uint32_t)pxf * kHashMul) >> hsh;
            cand = (int32_t)atomicExch(&ht[h], (uint32_t)x);
        }

        EZ_PROF_MARK(1);
        // ---- 2. capped judgement (exact decision)
        bool acc = false;
        int32_t info = 0;  // cand | forward count << 16 | backward count << 20 | rl << 24 | zr << 25
        if (valid) {
            uint64_t pcb, pcf;
            P.around(cand, pcb, pcf);
            const bool rl = cand >= done && cand < x;
            const bool zr = rl && cand + 8 < n && pcf == 0;
            const int32_t bl = rl ? ((x - done) < cand ? (x - done) : cand) : x - done;
            int32_t jb = clz_bytes(pxb ^ pcb);
            jb = jb < bl ? jb : bl;
            int32_t jf = ctz_bytes(pxf ^ (rl ? pcf : low_bytes(pcf, done - cand)));
            jf = jf < n - x ? jf : n - x;
            acc = rl ? (zr || jf + jb >= kMinCopyChunk) : ((jf < done - cand ? jf : done - cand) + jb >= kMinCopyChunk);
            int32_t zb = clz_bytes(pcb);
            zb = zb < cand - done ? zb : cand - done;
            const int32_t fk = zr ? 8 : jf, bk = zr ? zb : jb;
            info = cand | (fk << 16) | (bk << 20) | ((int32_t)rl << 24) | ((int32_t)zr << 25);
        }
        EZ_PROF_MARK(2);
        const uint32_t am = gball<G>(acc, g);
        const int a = am ? __builtin_ctz(am) : -1;  // the group's first accepting lane

        // ---- 3. undo the inserts of the lanes Go does not visit
        if (valid && a >= 0 && lj > a) atomicMin(&ht[h], (uint32_t)cand);

        // ---- 4. the accepted match: exact lengths, tokens
        const int32_t ib = bcast(info, G * g + (a < 0 ? 0 : a));
        const bool act = live && a >= 0;
        const int32_t xa = i + a;
        const int32_t ca = ib & 0xffff, fk = (ib >> 16) & 0xf, bk8 = (ib >> 20) & 0xf;
        const bool rl = (ib >> 24) & 1, zr = (ib >> 25) & 1;
        const int mode = zr ? 0 : (rl ? 1 : 2);
        const int32_t fa = zr ? ca : xa;
        constexpr bool kExt = (EZ_EXP & 2) == 0;
        EZ_PROF_MARK(3);
        const int32_t fx = gcount<G, true>(P, kExt && act && fk == 8, g, lj, fa, ca, mode, done, 8, n - fa);
        const int32_t f = fk == 8 ? fx : fk;
        const int32_t blim = zr ? ca - done : (rl ? ((xa - done) < ca ? (xa - done) : ca) : xa - done);
        const int32_t cx = gcount<G, false>(P, kExt && act && bk8 == 8, g, lj, fa, ca, mode, done, 8, blim);
        const int32_t c = bk8 == 8 ? cx : bk8;
        EZ_PROF_MARK(4);
        int32_t lit_end = 0, nxt = 0, clen = 0, T = 0, e1 = 0, e2 = 0;
        uint64_t lb = 0, cb = 0, ch2 = 0;
        if (act) {
            if (zr) {  // writeZeros :407-439
                lit_end = ca - c;
                nxt = ca + f;
                clen = nxt - lit_end;
            } else if (rl) {  // writeRunlen :441-489
                lit_end = xa - c;
                nxt = xa + f;
                clen = f + c;
            } else {  // window match, trim 2 (:292-296)
                const int32_t over = ca + f - done;
                lit_end = xa - c;
                nxt = xa + f - (over > 0 ? over : 0);
                clen = nxt - lit_end;
            }
            const bool lit = (rl && !zr) || lit_end > done;  // run-length: unconditional
            const int32_t L = lit_end - done;
            int32_t ln = 0;
            lb = tag_bytes(0x00, L, &ln);
            if (!lit) ln = 0;
            int32_t tn, on;
            const uint64_t tb = tag_bytes(0x80, clen, &tn);
            uint64_t ob;
            if (zr) { ob = 0x00ffull; on = 2; }  // OffLong, 0: zero region
            else ob = off_bytes(xa - ca, clen, &on);
            cb = tb | (ob << (8 * tn));
            ch2 = ob >> (64 - 8 * tn);
            e1 = ln;
            e2 = ln + (lit ? L : 0);
            T = e2 + tn + on;
            if (op + T > cap) err = EZ_ENOSPC;
        }
        EZ_PROF_MARK(5);
        const bool wr = act && !err && (EZ_EXP & 1) == 0;
        emit<G, SRC>(P, out, op, cap, wr, lj, T, e1, e2, lb, done, cb, ch2);
        EZ_PROF_MARK(6);
        if (act) {
            // the extra insert of i+1 after a window match (writer.go:315-318)
            if (!rl && xa + 1 + 4 <= n && lj == 0) {
                const uint32_t h1 = (P.u32(xa + 1) * kHashMul) >> hsh;
                ht[h1] = (uint32_t)(xa + 1);
            }
            const int32_t top = rl ? xa : xa + 1;
            hiw = hiw > top ? hiw : top;
            if (!err) op += T;
            i = done = nxt;
        } else if (live) {
            const int32_t top = i + nvalid - 1;
            hiw = hiw > top ? hiw : top;
            i += nvalid;
        }
        if (live && (err || i + 4 > n)) live = false;
        EZ_PROF_MARK(7);

    }
    // trailing literal (writer.go:324-329)
    {
        const bool tail = have && !err && done < n;
        int32_t ln = 0, T = 0;
        uint64_t lb = 0;
        if (tail) {
            lb = tag_bytes(0x00, n - done, &ln);
            T = ln + n - done;
            if (op + T > cap) err = EZ_ENOSPC;
        }
        emit<G, SRC>(P, out, op, cap, tail && !err && (EZ_EXP & 1) == 0, lj, T, ln, T, lb, done, 0, 0);
        if (tail && !err) op += T;
    }
    EZ_PROF_DUMP();
    if (have && lj == 0) {
        A.out_size[s] = (uint64_t)op;
        if (A.status) A.status[s] = err;
    }
}

int tile_g() {
    static const int g = getenv("EZ_K1T_G") ? atoi(getenv("EZ_K1T_G")) : 16;
    return g == 8 || g == 32 ? g : 16;
}
bool tile_gin() {
    static const bool v = !(getenv("EZ_K1T_GIN") && atoi(getenv("EZ_K1T_GIN")) == 0);
    return v;
}

template <int G>
uint32_t tile_stride(const CompressArgs &a) {
    if (a.ring || a.max_len == 0 || 2 * (int64_t)a.max_len > a.bs || a.max_len > 16384 || a.hs > 4096 || a.hs < 4) return 0;
    const uint64_t pwords = tile_gin() ? 0 : 2 + (a.max_len + 3) / 4 + 1 + 5;
    uint64_t w = (uint64_t)a.hs + pwords;
    w = (w + 3) & ~3ull;
    if (w * 4 * (64 / G) > 160 * 1024) return 0;
    return (uint32_t)w;
}

template <int G, bool GIN>
hipError_t launch_tile(const CompressArgs &a, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k1_tile<G, GIN>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    constexpr int S = 64 / G;
    const uint32_t stride = tile_stride<G>(a);
    const unsigned grid = (unsigned)((a.count + S - 1) / S);
    hipLaunchKernelGGL((k1_tile<G, GIN>), dim3(grid), dim3(64), (size_t)stride * 4 * S, st, a, stride);
    return hipGetLastError();
}

}  // namespace

// The property the visit relies on, checked once per process on the device:
// same-address LDS exchanges of one wave instruction apply in ascending lane
// order (lane l reads what lane l-4 wrote).  If it ever fails, K1t is not used.
__global__ void k_lds_order(uint32_t *res) {
    __shared__ uint32_t t[4];
    const uint32_t l = threadIdx.x;
    if (l < 4) t[l] = 0;
    __syncthreads();
    const uint32_t old = atomicExch(&t[l & 3], l + 1);
    const uint32_t want = l < 4 ? 0 : l - 3;
    if (old != want) atomicAdd(res, 1u);
}

bool lds_exchange_in_lane_order() {
    static int ok = -1;
    if (ok >= 0) return ok == 1;
    ok = 0;
    uint32_t *d = nullptr, h = 1;
    hipStream_t st = nullptr;
    if (hipMalloc(&d, sizeof(uint32_t)) != hipSuccess) return false;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess) {
        if (hipMemsetAsync(d, 0, sizeof(uint32_t), st) == hipSuccess) {
            hipLaunchKernelGGL(k_lds_order, dim3(1), dim3(64), 0, st, d);
            if (hipGetLastError() == hipSuccess && hipMemcpyAsync(&h, d, sizeof(uint32_t), hipMemcpyDeviceToHost, st) == hipSuccess &&
                hipStreamSynchronize(st) == hipSuccess)
                ok = h == 0 ? 1 : 0;
        }
        (void)hipStreamDestroy(st);
    }
    (void)hipFree(d);
    return ok == 1;
}

uint32_t tile_stride_words(const CompressArgs &a) {
    if (!lds_exchange_in_lane_order()) return 0;
    const int G = tile_g();
    return G == 8 ? tile_stride<8>(a) : (G == 32 ? tile_stride<32>(a) : tile_stride<16>(a));
}

hipError_t launch_compress_tile(const CompressArgs &a, hipStream_t st) {
    const int G = tile_g();
    if (tile_gin()) return G == 8 ? launch_tile<8, true>(a, st) : (G == 32 ? launch_tile<32, true>(a, st) : launch_tile<16, true>(a, st));
    return G == 8 ? launch_tile<8, false>(a, st) : (G == 32 ? launch_tile<32, false>(a, st) : launch_tile<16, false>(a, st));
}

}  // namespace ez
