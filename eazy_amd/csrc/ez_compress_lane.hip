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

namespace ez {
namespace {

typedef uint4 __attribute__((aligned(1))) uint4_u;
typedef uint64_t __attribute__((aligned(1))) u64_u;

constexpr int kWin = 8;  // positions judged per speculative window

struct Lane {
    const uint8_t *p;
    int32_t n;
    // 16 bytes y..y+15 of the stream, zero outside [0, n): one clamped
    // unaligned load shifted into place (bytes before 0 / from n on are 0)
    __device__ __forceinline__ void ld16(int32_t y, uint64_t &lo, uint64_t &hi) const {
        if (n >= 16) {
            const int32_t y0 = y < 0 ? 0 : (y > n - 16 ? n - 16 : y);
            const uint4 v = *(const uint4_u *)(p + y0);
            unsigned __int128 x = ((unsigned __int128)((uint64_t)v.z | ((uint64_t)v.w << 32)) << 64) |
                                  (uint64_t)v.x | ((uint64_t)v.y << 32);
            const int32_t d = y - y0;
            if (d < 0) x = d <= -16 ? 0 : x << (8 * -d);
            else if (d > 0) x = d >= 16 ? 0 : x >> (8 * d);
            lo = (uint64_t)x;
            hi = (uint64_t)(x >> 64);
            return;
        }
        lo = hi = 0;
        for (int k = 0; k < 16; k++) {
            const int32_t q = y + k;
            const uint64_t b = (q >= 0 && q < n) ? (uint64_t)p[q] : 0ull;
            if (k < 8) lo |= b << (8 * k);
            else hi |= b << (8 * (k - 8));
        }
    }
    __device__ __forceinline__ uint64_t ld8(int32_t y) const {
        uint64_t lo, hi;
        ld16(y, lo, hi);
        return lo;
    }
};

__device__ __forceinline__ uint64_t low_bytes(uint64_t x, int32_t k) {
    return k >= 8 ? x : (k <= 0 ? 0ull : (x & ((1ull << (8 * k)) - 1)));
}
__device__ __forceinline__ uint64_t high_bytes(uint64_t x, int32_t k) {
    return k >= 8 ? x : (k <= 0 ? 0ull : (x & ~((1ull << (8 * (8 - k))) - 1)));
}
__device__ __forceinline__ int32_t ctz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_ctzll(d) >> 3) : 8; }
__device__ __forceinline__ int32_t clz_bytes(uint64_t d) { return d ? (int32_t)(__builtin_clzll(d) >> 3) : 8; }

// Encoder.Tag / Encoder.Offset (writer.go:537-597), branch-free
__device__ __forceinline__ uint64_t tag_bytes(uint32_t tag, int32_t l, int32_t *n) {
    const bool a = l < 124, b = l < 380, c = l < 65916;
    *n = a ? 1 : (b ? 2 : (c ? 3 : 5));
    const uint32_t b0 = tag | (uint32_t)(a ? l : (b ? 124 : (c ? 125 : 126)));
    const uint64_t v = (uint64_t)(uint32_t)(b ? l - 124 : (c ? l - 380 : l - 65916));
    return a ? (uint64_t)b0 : ((uint64_t)b0 | (v << 8));
}
__device__ __forceinline__ uint64_t off_bytes(int32_t off, int32_t l, int32_t *n) {
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

__device__ __forceinline__ void st16(uint8_t *d, uint64_t lo, uint64_t hi) {
    *(uint4_u *)d = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

struct Out {
    uint8_t *o;
    int32_t op, cap;
    int err;
    // `k` bytes of (lo, hi); the 16-byte store overshoots when the slot has room
    __device__ __forceinline__ void put(uint64_t lo, uint64_t hi, int32_t k) {
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
    __device__ __forceinline__ void literal(const Lane &P, int32_t src, int32_t L) {
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
    __device__ __forceinline__ void copy(int32_t l, int32_t off, bool zero) {
        int32_t tn, on;
        const uint64_t tb = tag_bytes(0x80, l, &tn);
        uint64_t ob;
        if (zero) { ob = 0x00ffull; on = 2; }
        else ob = off_bytes(off, l, &on);
        put(tb | (ob << (8 * tn)), ob >> (64 - 8 * tn), tn + on);
    }
};

__global__ __launch_bounds__(256) void k1_lane(CompressArgs A, uint16_t *htbase) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= A.count) return;
    const int32_t hs = (int32_t)A.hs;
    const int64_t bs = A.bs;
    const uint32_t hsh = 32u - (uint32_t)(64 - __builtin_clzll((uint64_t)(hs - 1)));
    Lane P;
    P.p = A.in + A.in_off[s];
    P.n = (int32_t)(A.in_off[s + 1] - A.in_off[s]);
    const int32_t n = P.n;
    uint16_t *ht = htbase + s * (uint64_t)hs;
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
            const bool rl = c >= done;
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
        if (cand >= done && cand < i) {
            // writeRunlen writer.go:441-489, st = cand
            const int32_t st = cand;
            if (st + 8 < n && cf == 0) {
                // writeZeros writer.go:407-439
                int32_t ze = st + 8;
                while (ze < n) {
                    const int32_t z = ctz_bytes(P.ld8(ze));
                    ze += z;
                    if (z < 8) break;
                }
                if (ze > n) ze = n;
                int32_t zs = st;
                while (zs > done) {
                    const int32_t back = zs - done < 8 ? zs - done : 8;
                    const int32_t z = clz_bytes(high_bytes(P.ld8(zs - 8), back) | (back < 8 ? ((1ull << (8 * (8 - back))) - 1) : 0));
                    zs -= z < back ? z : back;
                    if (z < back) break;
                }
                if (ze - zs < kMinCopyChunk) { i = zs + 1; continue; }  // unreachable
                if (done != zs) O.literal(P, done, zs - done);
                O.copy(ze - zs, 0, true);
                i = done = ze;
                continue;
            }
            // jf forward, jb backward (st + jb >= 0, i + jb >= done)
            int32_t jf = ctz_bytes(xf ^ cf);
            while (jf >= 8 && i + jf < n) {
                const int32_t t = ctz_bytes(P.ld8(i + jf) ^ P.ld8(st + jf));
                jf += t;
                if (t < 8) break;
            }
            if (jf > n - i) jf = n - i;
            const int32_t blim = (i - done) < st ? (i - done) : st;
            int32_t jb = clz_bytes(xb ^ cb);
            while (jb >= 8 && jb < blim) {
                const int32_t t = clz_bytes(P.ld8(i - jb - 8) ^ P.ld8(st - jb - 8));
                jb += t;
                if (t < 8) break;
            }
            if (jb > blim) jb = blim;
            if (jf + jb < kMinCopyChunk) { i++; continue; }  // unreachable (judged above)
            if ((int64_t)(i - st) >= bs - 8) {  // cut writer.go:464-473
                const int32_t iend = done + i - st;
                O.literal(P, done, iend - done);
                i = done = iend;
                continue;
            }
            O.literal(P, done, i - jb - done);  // unconditional
            O.copy(jf + jb, i - st, false);
            i = done = i + jf;
            continue;
        }
        // window match writer.go:233-321; ring: p[y] for 0 <= y < done, else 0
        int32_t f = ctz_bytes(xf ^ low_bytes(cf, done - cand));
        while (f >= 8 && i + f < n) {
            const int32_t t = ctz_bytes(P.ld8(i + f) ^ low_bytes(P.ld8(cand + f), done - cand - f));
            f += t;
            if (t < 8) break;
        }
        if (f > n - i) f = n - i;
        const int32_t blim = i - done;
        int32_t c = clz_bytes(xb ^ low_bytes(cb, done - cand + 8));
        while (c >= 8 && c < blim) {
            const int32_t y = cand - c - 8;
            const int32_t t = clz_bytes(P.ld8(i - c - 8) ^ low_bytes(P.ld8(y), done - y));
            c += t;
            if (t < 8) break;
        }
        if (c > blim) c = blim;
        const int32_t ist = i - c;
        int32_t iend = i + f;
        const int64_t st = (int64_t)cand - c;
        int64_t end = (int64_t)cand + f;
        int64_t dd = ((int64_t)done - bs + (iend - done)) - st;
        if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
        dd = end - done;
        if (dd > 0) { end -= dd; iend -= (int32_t)dd; }
        if (end - st < kMinCopyChunk) { i++; continue; }  // unreachable (judged above)
        if (done < ist) O.literal(P, done, ist - done);
        if ((int64_t)(i - cand) > bs) { O.err = EZ_EINVAL; break; }
        O.copy(iend - ist, i - cand, false);
        if (i + 1 + 4 <= n) {
            const uint32_t h1 = ((uint32_t)(xf >> 8) * kHashMul) >> hsh;
            ht[h1] = (uint16_t)(i + 1);
        }
        i = done = iend;
    }
    if (!O.err && done < n) O.literal(P, done, n - done);  // writer.go:324-329
    A.out_size[s] = (uint64_t)O.op;
    if (A.status) A.status[s] = O.err;
}

}  // namespace

uint64_t lane_scratch_halves(const CompressArgs &a) {
    if (a.ring || a.max_len == 0 || a.max_len > 65535 || 2 * (int64_t)a.max_len > a.bs || a.hs < 8) return 0;
    return a.count * (uint64_t)a.hs;
}

hipError_t launch_compress_lane(const CompressArgs &a, uint16_t *scratch, hipStream_t st) {
    static const unsigned blk = getenv("EZ_K1_BLOCK") ? (unsigned)atoi(getenv("EZ_K1_BLOCK")) : 256u;
    const unsigned grid = (unsigned)((a.count + blk - 1) / blk);
    hipLaunchKernelGGL(k1_lane, dim3(grid), dim3(blk), 0, st, a, scratch);
    return hipGetLastError();
}

}  // namespace ez
