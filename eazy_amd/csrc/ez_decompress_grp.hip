// ez_decompress_grp.hip — K2p + K2x: two-phase batch decompression of small
// streams, the decoded history resident in LDS.
//
// Restates Reader.Read to EOF for NewReaderBytes (reader.go:116-216 read,
// readTag :218-270, continueMetaTag :272-325, reset :327-344, Decoder
// :346-514) for the common case; any other stream goes to the exact decoder
// through the slow list, as with k2_fast.
//
// Why two phases.  A token's header depends only on the compressed bytes, its
// bytes on earlier output.  k2_fast does both per lane and pays an HBM
// read-back of recently written output per token; a group-per-stream decoder
// with the output in LDS avoids that but repeats the serial parse in every lane
// of the group.  Here:
//   K2p (one lane per stream) parses the stream into 4-byte token records —
//       literal: L << 16 | input offset, copy: 1 << 31 | L << 16 | distance —
//       written into the stream's own output slot (the slot is free until the
//       end of K2x), validates everything (errors, metas, slot and LDS fits),
//       and leaves the record count in out_size (or hands the stream over);
//   K2x (G lanes per stream) stages the compressed stream at the top of an LDS
//       region, reads the records 16 at a time (one coalesced load per group,
//       broadcast token by token with DPP row_newbcast: no LDS), builds the
//       output from the bottom of the region one byte per lane per step, and
//       writes it to the slot with 16-byte stores at the end.
// K2p checks the region invariant for every token (output position <= unread
// input position), so K2x needs no checks.  A back-reference of distance
// D >= G is read forward in G-byte steps (every source byte precedes the
// step); D < G uses out[pos - D + (k mod D)]; sources before the stream start
// read zeros (the fresh ring).
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"

namespace ez {
namespace {

constexpr uint64_t kHandOver = ~0ull;  // out_size mark of a stream K2p handed to the exact decoder
constexpr int kXG = 16;                // K2x lanes per stream (one DPP row)

// the LDS region layout both phases agree on: input words at the top, 16 bytes
// of pad after them; returns the region byte of input byte 0 (< 0: no fit)
__host__ __device__ __forceinline__ int32_t region_ib(uint32_t R, uint32_t r, int32_t nb) {
    const int32_t nw = (int32_t)((r + (uint32_t)nb + 3) >> 2);
    const int32_t wb = (int32_t)(R >> 2) - 4 - nw;
    return wb < 0 ? -1 : 4 * wb + (int32_t)r;
}

// ---------------------------------------------------------------- K2p
__device__ __forceinline__ void parse_one(const DecompressArgs &A, uint32_t R, uint64_t s) {
    const uint8_t *b = A.in + A.in_off[s];
    const int64_t nb64 = (int64_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint8_t *in_end = A.in + A.in_off[A.count];
    uint8_t *out = A.out + A.out_off[s];
    const int64_t cap64 = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    const int64_t limit = A.block_size_limit;
    const int32_t nb = nb64 > (int64_t)R ? (int32_t)R + 1 : (int32_t)nb64;
    const int32_t cap = cap64 > (1ll << 30) ? (1 << 30) : (int32_t)cap64;
    const int32_t ib = region_ib(R, (uint32_t)((uintptr_t)b & 3), nb);
    bool slow = in_end - A.in < 16 || ib < 0;
    const int32_t rcap = cap / 4;  // records the slot holds
    int32_t i = 0, pos = 0, bsl = -1, nt = 0;
    while (!slow && i < nb) {
        const V16 h = b + i + 16 <= in_end ? ld16v(b + i) : ld_clamped(b + i, A.in, in_end);
        const uint32_t w0 = (uint32_t)h.lo, w1 = (uint32_t)(h.lo >> 32);
        const uint32_t t0 = w0 & 0xff, l7 = t0 & 0x7f;
        if (t0 == 0) {  // padding (reader.go:221-224): the zero bytes of the window at once
            i += h.lo ? (int32_t)(__builtin_ctzll(h.lo) >> 3) : (h.hi ? 8 + (int32_t)(__builtin_ctzll(h.hi) >> 3) : 16);
            continue;
        }
        if (t0 == 0x80) {  // meta (continueMetaTag reader.go:272-325): header metas and breaks only
            const uint32_t mb = (w0 >> 8) & 0xff, mt = mb & 0xf8, ml = mb & 7;
            const int32_t mln = ml == 7 ? 0 : (1 << ml);
            const uint32_t marg = (w0 >> 16) & 0xff;
            const bool m_brk = mt == kMetaBreak && mln == 0;
            const bool m_rst = mt == kMetaReset && mln == 1 && marg <= 32 && pos == 0 && (limit == 0 || (1ll << marg) <= limit);
            const bool m_ver = mt == kMetaVer && mln == 1 && marg == 0;
            const bool m_mag = mt == kMetaMagic && mln == 4 && ((w0 >> 16) | (w1 << 16)) == 0x797a6165u;
            if (ml == 6 || i + 2 + mln > nb || !(m_brk || m_rst || m_ver || m_mag)) { slow = true; break; }
            if (m_rst) bsl = (int32_t)marg;
            i += 2 + mln;
            continue;
        }
        // Decoder.Tag reader.go:346-392, Decoder.Offset :394-420 (1-3 byte forms)
        const uint32_t lx = (w0 >> 8) | (w1 << 24);
        const int32_t L = l7 < 124 ? (int32_t)l7 : (l7 == 124 ? 124 + (int32_t)(lx & 0xff) : 380 + (int32_t)(lx & 0xffff));
        const uint32_t j = l7 < 124 ? 1 : (l7 == 124 ? 2 : 3);
        const bool cp = (t0 & 0x80) != 0;
        const uint32_t x = (uint32_t)(h.lo >> (8 * j));
        const bool lng = (x & 0xff) == 0xff;
        const uint32_t y = lng ? (uint32_t)(h.lo >> (8 * j + 8)) : x;
        const uint32_t o = y & 0xff, ox = y >> 8;
        const int32_t D0 = o < 252 ? (int32_t)o : (o == 252 ? 252 + (int32_t)(ox & 0xff) : 508 + (int32_t)(ox & 0xffff));
        const uint32_t k = o < 252 ? 1 : (o == 252 ? 2 : 3);
        const int32_t D = lng ? D0 : D0 + L;
        const int32_t adv = cp ? (int32_t)(j + (lng ? 1 : 0) + k) : (int32_t)j + L;
        const int64_t bs = bsl < 0 ? 0 : (1ll << bsl);
        // 5-byte forms, LenAlt/OffAlt, BlockSizeLimit, missed meta, truncation, the
        // slot, distance > window, the record list, the LDS region invariant
        const bool bad = l7 >= 126 || (cp && o >= 254) || (limit != 0 && L > limit) || bs == 0 || pos + L > cap ||
                         i + adv > nb || (cp && D > bs) || nt + 1 > rcap || L >= 32768 ||
                         (cp ? pos + L > ib + i + adv : pos > ib + i + (int32_t)j);
        if (bad) { slow = true; break; }
        const uint32_t rec = cp ? (0x80000000u | ((uint32_t)L << 16) | (uint32_t)D) : (((uint32_t)L << 16) | (uint32_t)(i + (int32_t)j));
        *(uint32_t __attribute__((aligned(1))) *)(out + 4 * nt) = rec;
        nt++;
        pos += L;
        i += adv;
    }
    if (slow) {
        A.out_size[s] = kHandOver;
        const uint32_t at = atomicAdd(&A.slow[0], 1u);
        A.slow[1 + at] = (uint32_t)s;
    } else {
        A.out_size[s] = (uint64_t)nt;
    }
}

__global__ __launch_bounds__(256) void k2_parse(DecompressArgs A, uint32_t R) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < A.count; s += (uint64_t)gridDim.x * blockDim.x)
        parse_one(A, R, s);
}

// ---------------------------------------------------------------- K2x
template <int TT>
__device__ __forceinline__ uint32_t row_bcast(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + TT, 0xf, 0xf, false);  // row_newbcast:TT
}

template <int TT>
__device__ __forceinline__ void exec_token(uint8_t *reg, uint32_t recs, int32_t t0, int32_t nt, int32_t ib, int lj, int32_t &pos) {
    const uint32_t rec = row_bcast<TT>(recs);
    const bool here = t0 + TT < nt;
    const int32_t L = here ? (int32_t)((rec >> 16) & 0x7fff) : 0;
    const bool cp = (rec >> 31) != 0;
    const int32_t v = (int32_t)(rec & 0xffff);
    const int32_t src = cp ? pos - v : ib + v;
    const bool run = cp && v < kXG;  // short-period run or zero region
    for (int32_t base = 0; __ballot(base < L) != 0; base += kXG) {
        const int32_t k = base + lj;
        if (k < L) {
            int32_t yy = src + k;
            if (run) yy = v == 0 ? -1 : src + (int32_t)((uint32_t)k % (uint32_t)v);
            const uint32_t c = reg[yy < 0 ? 0 : yy];
            reg[pos + k] = (uint8_t)(yy < 0 ? 0u : c);
        }
    }
    pos += L;
}

__global__ __launch_bounds__(64) void k2_exec(DecompressArgs A, uint32_t R) {
    constexpr int S = 64 / kXG;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / kXG, lj = lane % kXG;
    const uint64_t s = (uint64_t)blockIdx.x * S + g;
    uint64_t nt64 = kHandOver;
    if (s < A.count) nt64 = A.out_size[s];
    const bool go = nt64 != kHandOver;
    const int32_t nt = go ? (int32_t)nt64 : 0;
    uint8_t *reg = smem + (uint32_t)g * R;
    const uint8_t *gb = go ? A.in + A.in_off[s] : A.in;
    const int32_t nb = go ? (int32_t)(A.in_off[s + 1] - A.in_off[s]) : 0;
    const uint32_t r = (uint32_t)((uintptr_t)gb & 3);
    const int32_t ib = go ? region_ib(R, r, nb) : 0;
    uint8_t *out = go ? A.out + A.out_off[s] : A.out;
    if (go) {  // stage the compressed stream's words at the region's top
        const uint32_t *gw = (const uint32_t *)(gb - r);
        uint32_t *lw = (uint32_t *)(reg + (ib - (int32_t)r));
        const int32_t nw = (int32_t)((r + (uint32_t)nb + 3) >> 2);
        for (int32_t k = lj; k < nw; k += kXG) lw[k] = gw[k];
    }
    typedef uint32_t __attribute__((aligned(1))) u32_ua;
    const u32_ua *rp = (const u32_ua *)out;  // the records K2p left in the slot
    uint32_t recs = 0;
    if (go && lj < nt) recs = rp[lj];
    __syncthreads();  // one wave: orders the staging before the reads
    int32_t pos = 0;
    for (int32_t t0 = 0; __ballot(t0 < nt) != 0; t0 += kXG) {
        const uint32_t cur = recs;
        if (go && t0 + kXG + lj < nt) recs = rp[t0 + kXG + lj];  // the next 16, loaded beside these
        exec_token<0>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<1>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<2>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<3>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<4>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<5>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<6>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<7>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<8>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<9>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<10>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<11>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<12>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<13>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<14>(reg, cur, t0, nt, ib, lj, pos);
        exec_token<15>(reg, cur, t0, nt, ib, lj, pos);
    }
    if (!go) return;
    // the decoded bytes to the slot (over the records): 16 bytes per lane per step
    for (int32_t k = 16 * lj; k < pos; k += 16 * kXG) {
        const uint4 v = *(const uint4 *)(reg + k);
        const V16 x{(uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z | ((uint64_t)v.w << 32)};
        if (k + 16 <= pos) st16v(out + k, x);
        else put_small(out + k, x, (uint32_t)(pos - k));
    }
    if (lj == 0) {
        A.out_size[s] = (uint64_t)pos;
        if (A.status) A.status[s] = EZ_OK;
    }
}

}  // namespace

// LDS region per stream for a batch whose largest output slot is max_out
// (0 = not usable: unknown or too large for LDS residency)
uint32_t grp_decode_region(uint64_t max_out) {
    if (max_out == 0 || max_out > 32768) return 0;
    const uint64_t R = (max_out + 64 + 64 + 15) & ~15ull;
    if (R * (64 / kXG) + 16 > 160 * 1024) return 0;
    return (uint32_t)R;
}

hipError_t launch_decompress_grp(const DecompressArgs &a, uint32_t R, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k2_exec, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const uint64_t pgrid = (a.count + 255) / 256;
    hipLaunchKernelGGL(k2_parse, dim3((unsigned)pgrid), dim3(256), 0, st, a, R);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    constexpr int S = 64 / kXG;
    const uint64_t grid = (a.count + S - 1) / S;
    hipLaunchKernelGGL(k2_exec, dim3((unsigned)grid), dim3(64), (size_t)R * S + 16, st, a, R);
    return hipGetLastError();
}

}  // namespace ez
