// ez_compress_lane.hip — K1l: batch compression, one lane per stream.
//
// For batches of many small fresh streams (the BASELINE C1/C3 shape:
// 64 Ki x 4 KiB) the window-per-wave kernels pay a large fixed cost per
// window.  Here every lane runs the reference loop of Writer.Write
// (writer.go:206-337, writeRunlen :441-489, writeZeros :407-439) on its own
// stream, so each wave instruction serves 64 streams:
//   * the hash table is per stream in HBM scratch (u16 entries: fresh
//     streams with n < 64 Ki positions), zeroed by the lane;
//   * the ring is the fresh-stream image (start = 0, 2n <= block):
//     block[y] = p[y] for 0 <= y < done, else 0;
//   * matches are judged 8 bytes at a time from 16-byte unaligned global
//     loads around the position and the candidate (xor + ctz/clz), and
//     extended 8 bytes at a time only when the first 8 bytes all match;
//   * tokens are written with 16-byte stores (the slot's slack absorbs the
//     overshoot, which the next token overwrites).
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_bytes.h"

namespace ez {
namespace {

typedef uint64_t __attribute__((aligned(1))) u64_u;

constexpr int kWin = 8;  // positions judged per speculative window

struct Lane {
    const uint8_t *p;
    int32_t n;
    const uint8_t *lo_lim, *hi_lim;  // [batch start, batch end - 16]: every load stays inside the batch
    // 16 bytes y..y+15 of the stream, zero outside [0, n).  One unaligned load
    // at the exact address (neighbouring streams' bytes are masked off); only
    // the batch's first/last bytes need the clamp-and-shift fix-up.
    EZ_HD void ld16(int32_t y, uint64_t &lo, uint64_t &hi) const {
        const uint8_t *a = p + y;
        const uint8_t *ac = a < lo_lim ? lo_lim : (a > hi_lim ? hi_lim : a);
        V16 v = ld16v(ac);
        if (ac != a) v = a > ac ? shr16(v, (uint32_t)(a - ac)) : shl16(v, (uint32_t)(ac - a));
        if (y < 0 || y + 16 > n) {  // keep bytes j with 0 <= y + j < n
            const int32_t za = y < 0 ? -y : 0, kb = n - y;  // za bytes cut in front, kb bytes kept from the start
            const uint64_t l1 = za >= 8 ? 0 : ~0ull << (8 * za);
            const uint64_t h1 = za >= 16 ? 0 : (za <= 8 ? ~0ull : ~0ull << (8 * (za - 8)));
            const uint64_t l2 = kb >= 8 ? ~0ull : (kb <= 0 ? 0 : (1ull << (8 * kb)) - 1);
            const uint64_t h2 = kb >= 16 ? ~0ull : (kb <= 8 ? 0 : (1ull << (8 * (kb - 8))) - 1);
            v.lo &= l1 & l2;
            v.hi &= h1 & h2;
        }
        lo = v.lo;
        hi = v.hi;
    }
    EZ_HD uint64_t ld8(int32_t y) const {
        uint64_t lo, hi;
        ld16(y, lo, hi);
        return lo;
    }
};

EZ_HD uint64_t low_bytes(uint64_t x, int32_t k) {
    return k >= 8 ? x : (k <= 0 ? 0ull : (x & ((1ull << (8 * k)) - 1)));
}
EZ_HD int32_t ctz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_ctzll(d) >> 3) : 8; }
EZ_HD int32_t clz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_clzll(d) >> 3) : 8; }

// Encoder.Tag / Encoder.Offset (writer.go:537-597), branch-free
EZ_HD uint64_t tag_bytes(uint32_t tag, int32_t l, int32_t *n) {
    const bool a = l < 124, b = l < 380, c = l < 65916;
    *n = a ? 1 : (b ? 2 : (c ? 3 : 5));
    const uint32_t b0 = tag | (uint32_t)(a ? l : (b ? 124 : (c ? 125 : 126)));
    const uint64_t v = (uint64_t)(uint32_t)(b ? l - 124 : (c ? l - 380 : l - 65916));
    return a ? (uint64_t)b0 : ((uint64_t)b0 | (v << 8));
}
EZ_HD uint64_t off_bytes(int32_t off, int32_t l, int32_t *n) {
    const bool lg = off < l;
    const int32_t o = lg ? off : off - l;
    const bool a = o < 252, b = o < 508, c = o < 66044;
    int32_t k = a ? 1 : (b ? 2 : (c ? 3 : 5));
    const uint32_t b0 = (uint32_t)(a ? o : (b ? 252 : (c ? 253 : 254)));
    const uint64_t v = (uint64_t)(uint32_t)(b ? o - 252 : (c ? o - 508 : o - 66044));
    uint64_t r = a ? (uint64_t)b0 : ((uint64_t)b0 | (v << 8));
    if (lg) { r = 0xff | (r << 8); k += 1; }
    *n = k;
    return r;
}

EZ_HD void st16(uint8_t *d, uint64_t lo, uint64_t hi) {
    *(uint4_u *)d = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

struct Out {
    uint8_t *o;
    int32_t op, cap;
    int err;
    // `k` bytes of (lo, hi); the 16-byte store overshoots when the slot has room
    EZ_HD void put(uint64_t lo, uint64_t hi, int32_t k) {
        if (err) return;
        if (op + k > cap) { err = EZ_ENOSPC; return; }
        if (op + 16 <= cap) {
            st16(o + op, lo, hi);
        } else {
            for (int32_t j = 0; j < k; j++) o[op + j] = (uint8_t)(j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8)));
        }
        op += k;
    }
    // literal header + p[src..src+L)
    EZ_HD void literal(const Lane &P, int32_t src, int32_t L) {
        int32_t ln;
        const uint64_t tb = tag_bytes(0x00, L, &ln);
        put(tb, 0, ln);
        if (err) return;
        if (op + L > cap) { err = EZ_ENOSPC; return; }
        int32_t k = 0;
        for (; k + 16 <= L; k += 16) {
            uint64_t lo, hi;
            P.ld16(src + k, lo, hi);
            st16(o + op + k, lo, hi);
        }
        if (k < L) {
            uint64_t lo, hi;
            P.ld16(src + k, lo, hi);
            if (op + k + 16 <= cap) st16(o + op + k, lo, hi);
            else for (int32_t j = 0; k + j < L; j++) o[op + k + j] = (uint8_t)(j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8)));
        }
        op += L;
    }
    // Tag(Copy, l) + Offset(off, l); zero region: Tag(Copy, l) + OffLong 0
    EZ_HD void copy(int32_t l, int32_t off, bool zero) {
        int32_t tn, on;
        const uint64_t tb = tag_bytes(0x80, l, &tn);
        uint64_t ob;
        if (zero) { ob = 0x00ffull; on = 2; }
        else ob = off_bytes(off, l, &on);
        put(tb | (ob << (8 * tn)), ob >> (64 - 8 * tn), tn + on);
    }
};

// HT_LDS: the lane's hash table lives in LDS (64 lanes x hs u16 per block,
// one 64-lane block per CU at hs = 1024); else in HBM scratch.
EZ_HD void lane_one(const CompressArgs &A, uint16_t *ht, const uint64_t s) {
    const int32_t hs = (int32_t)A.hs;
    const int64_t bs = A.bs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));
    Lane P;
    P.p = A.in + A.in_off[s];
    P.n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    P.lo_lim = A.in;
    P.hi_lim = A.in + A.in_off[A.count] - 16;  // the launcher guarantees >= 16 batch bytes (max_len >= 16)
    const int32_t n = P.n;
    for (int32_t k = 0; k < hs; k += 8) *(uint4 *)(ht + k) = make_uint4(0, 0, 0, 0);
    Out O;
    O.o = A.out + A.out_off[s];
    O.cap = (int32_t)(A.out_off[s + 1] - A.out_off[s]);
    O.op = 0;
    O.err = 0;
    {  // header (writer.go:495-517)
        const uint64_t bsl = (uint64_t)__builtin_ctzll((uint64_t)bs);
        if (A.append_magic) O.put(0x1080797a61650280ull, bsl, 9);  // 80 02 'e' 'a' 'z' 'y' 80 10 | bsl
        else O.put(0x1080ull | (bsl << 16), 0, 3);
    }
    int32_t i = 0, done = 0;
    int32_t guard = 16 * n + 4096;
    while (i + 4 <= n && !O.err) {
        if (--guard < 0) { O.err = EZ_ESTUCK; break; }
        // ---- speculative window: positions i .. i+kn-1 judged together ----
        uint64_t w0, w1, w2, w3;  // p[i-8 .. i+23]
        P.ld16(i - 8, w0, w1);
        P.ld16(i + 8, w2, w3);
        const int32_t kn = n - 3 - i < kWin ? n - 3 - i : kWin;  // positions with p + 4 <= n
        uint64_t X[kWin], B[kWin], CB[kWin], CF[kWin];
        uint32_t H[kWin];
        int32_t C[kWin];
#pragma unroll
        for (int k = 0; k < kWin; k++) {
            X[k] = k ? (w1 >> (8 * k)) | (w2 << (64 - 8 * k)) : w1;  // p[i+k .. i+k+7]
            B[k] = k ? (w0 >> (8 * k)) | (w1 << (64 - 8 * k)) : w0;  // p[i+k-8 .. i+k-1]
            H[k] = ((uint32_t)X[k] * kHashMul) >> hsh;
        }
#pragma unroll
        for (int k = 0; k < kWin; k++) C[k] = k < kn ? (int32_t)ht[H[k]] : 0;
        // positions of this window visited before i+k shadow the table entry
#pragma unroll
        for (int k = 1; k < kWin; k++)
#pragma unroll
            for (int j = 0; j < k; j++)
                if (H[j] == H[k]) C[k] = i + j;
#pragma unroll
        for (int k = 0; k < kWin; k++) P.ld16(C[k] - 8, CB[k], CF[k]);
        // acceptance with 8-byte capped lengths is exact: the threshold
        // kMinCopyChunk (6) is below the cap (8)
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < kWin; k++) {
            const int32_t p = i + k, c = C[k];
            const bool rl = c >= done && c < p;  // c == p only at p == 0 (empty table)
            const int32_t bl = rl ? ((p - done) < c ? (p - done) : c) : p - done;
            int32_t jb = clz_bytes(B[k] ^ CB[k]);
            jb = jb < bl ? jb : bl;
            int32_t jf = ctz_bytes(X[k] ^ (rl ? CF[k] : low_bytes(CF[k], done - c)));
            jf = jf < n - p ? jf : n - p;
            const bool ok = rl ? ((c + 8 < n && CF[k] == 0) || jf + jb >= kMinCopyChunk)
                               : ((jf < done - c ? jf : done - c) + jb >= kMinCopyChunk);
            acc |= (uint32_t)(k < kn && ok) << k;
        }
        const int32_t kk = acc ? (int32_t)__builtin_ctz(acc) : kn;
        const int32_t kv = acc ? kk + 1 : kn;  // positions visited (and inserted)
#pragma unroll
        for (int k = 0; k < kWin; k++)
            if (k < kv) ht[H[k]] = (uint16_t)(i + k);
        if (!acc) { i += kn; continue; }
        uint64_t xb = 0, xf = 0, cb = 0, cf = 0;
        int32_t cand = 0;
#pragma unroll
        for (int k = 0; k < kWin; k++)
            if (k == kk) { xb = B[k]; xf = X[k]; cb = CB[k]; cf = CF[k]; cand = C[k]; }
        i += kk;
        // ---- the accepted position: one code path for the three match kinds ----
        // run-length (writeRunlen writer.go:441-489, candidate inside the unemitted part),
        // its zero-region form (writeZeros :407-439) and the window match (:233-321;
        // ring image: p[y] for 0 <= y < done, else 0).  No cut / trim 1 / far
        // reference: impossible for fresh streams with 2n <= block (dispatch checks).
        const bool rl = cand >= done && cand < i;
        const bool zr = rl && cand + 8 < n && cf == 0;
        // forward count from fa against the candidate (or against zeros)
        const int32_t fa = zr ? cand : i;
        int32_t f = zr ? 8 : ctz_bytes(xf ^ (rl ? cf : low_bytes(cf, done - cand)));
        while (f >= 8 && fa + f < n) {
            const int32_t y = cand + f;
            const uint64_t w = zr ? 0ull : (rl ? P.ld8(y) : low_bytes(P.ld8(y), done - y));
            const int32_t t = ctz_bytes(P.ld8(fa + f) ^ w);
            f += t;
            if (t < 8) break;
        }
        if (f > n - fa) f = n - fa;
        // backward count before fa (zeros: back to done; run-length: st + jb >= 0, i + jb >= done)
        const int32_t blim = zr ? cand - done : (rl ? ((i - done) < cand ? (i - done) : cand) : i - done);
        int32_t c = clz_bytes(zr ? cb : (xb ^ cb));  // window: bytes before cand < done, no ring mask
        while (c >= 8 && c < blim) {
            const int32_t y = cand - c - 8;
            const uint64_t w = zr ? 0ull : (rl ? P.ld8(y) : low_bytes(P.ld8(y), done - y));
            const int32_t t = clz_bytes(P.ld8(fa - c - 8) ^ w);
            c += t;
            if (t < 8) break;
        }
        if (c > blim) c = blim;
        int32_t lit_end, next, clen;
        if (zr) {
            lit_end = cand - c;
            next = cand + f;
            clen = next - lit_end;
        } else if (rl) {
            lit_end = i - c;
            next = i + f;
            clen = f + c;
        } else {
            // trim 2 (writer.go:292-296): the copy source may not pass done
            const int32_t over = cand + f - done;
            lit_end = i - c;
            next = i + f - (over > 0 ? over : 0);
            clen = next - lit_end;
        }
        if (rl && !zr ? true : lit_end > done) O.literal(P, done, lit_end - done);  // run-length: unconditional
        O.copy(clen, i - cand, zr);
        if (!rl && i + 1 + 4 <= n) {  // the extra insert of i+1 after a window match (writer.go:315-318)
            const uint32_t h1 = ((uint32_t)(xf >> 8) * kHashMul) >> hsh;
            ht[h1] = (uint16_t)(i + 1);
        }
        i = done = next;
    }
    if (!O.err && done < n) O.literal(P, done, n - done);  // writer.go:324-329
    A.out_size[s] = (uint64_t)O.op;
    if (A.status) A.status[s] = O.err;
}

// grid-stride over streams; a lane's table is reused for each of its streams
// (the launcher may run fewer lanes than streams to keep tables cache-resident)
template <bool HT_LDS>
__global__ __launch_bounds__(256) void k1_lane(CompressArgs A, uint16_t *htbase) {
    extern __shared__ uint16_t lds_ht[];
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint16_t *ht = HT_LDS ? lds_ht + threadIdx.x * A.hs : htbase + t * A.hs;
    for (uint64_t s = t; s < A.count; s += (uint64_t)gridDim.x * blockDim.x) lane_one(A, ht, s);
}

}  // namespace

constexpr int32_t kLaneLdsHs = 1024;  // largest table kept in LDS (64 x 2 KiB = 128 KiB per block)

static unsigned lane_block() {
    static const unsigned blk = getenv("EZ_K1_BLOCK") ? (unsigned)atoi(getenv("EZ_K1_BLOCK")) : 256u;
    return blk;
}
// threads launched = lanes in flight, a whole number of blocks (EZ_K1_WAVES caps them, experiments);
// the scratch holds one table per launched thread
static uint64_t lane_threads(const CompressArgs &a) {
    static const uint64_t maxw = getenv("EZ_K1_WAVES") ? (uint64_t)atoll(getenv("EZ_K1_WAVES")) : 0;
    uint64_t t = a.count;
    if (maxw && t > maxw * 64) t = maxw * 64;
    return (t + lane_block() - 1) / lane_block() * lane_block();
}

uint64_t lane_scratch_halves(const CompressArgs &a) {
    if (a.ring || a.max_len < 16 || a.max_len > 65535 || 2 * (int64_t)a.max_len > a.bs || a.hs < 8) return 0;
    if (a.hs <= kLaneLdsHs && getenv("EZ_K1_HTL")) return 1;  // LDS tables (experiment): no scratch
    return lane_threads(a) * (uint64_t)a.hs;
}

hipError_t launch_compress_lane(const CompressArgs &a, uint16_t *scratch, hipStream_t st) {
    if (a.hs <= kLaneLdsHs && getenv("EZ_K1_HTL")) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void *)k1_lane<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr = true;
        }
        const unsigned grid = (unsigned)((a.count + 63) / 64);
        hipLaunchKernelGGL(k1_lane<true>, dim3(grid), dim3(64), (size_t)64 * a.hs * 2, st, a, scratch);
        return hipGetLastError();
    }
    const unsigned blk = lane_block();
    const unsigned grid = (unsigned)(lane_threads(a) / blk);
    hipLaunchKernelGGL(k1_lane<false>, dim3(grid), dim3(blk), 0, st, a, scratch);
    return hipGetLastError();
}

}  // namespace ez
