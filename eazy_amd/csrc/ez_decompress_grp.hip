// ez_decompress_grp.hip — K2grp: batch decompression of small streams with the
// whole stream resident in LDS.
//
// Restates Reader.Read to EOF for NewReaderBytes (reader.go:116-216 read /
// readTag :218-270 / continueMetaTag :272-325 / reset :327-344, Decoder
// :346-514) for the common case, like k2_fast, but the decoded history lives
// in LDS instead of HBM: a back-reference reads bytes this stream produced a
// few tokens earlier, and from LDS that costs ~60 cycles where the HBM slot
// read-back of k2_fast costs a cache miss (PMC: 2.4 GB fetched per launch).
//
// Mapping: G lanes per stream, 64/G streams per wave (one wave per
// workgroup).  Each stream owns an LDS region of R bytes: the compressed
// stream is staged at its top end, the output grows from its bottom.  The
// output position never passes the unread input (checked per token:
// pos <= input position for literals, which are copied forward, and
// pos + L <= next token for copies), so both fit in max_out + a small margin.
// The G lanes of a stream parse every token redundantly (group-uniform
// values, no shuffles) and move its bytes one byte per lane per step;
// a back-reference of distance D >= G is read forward in G-byte steps
// (every source byte is < the step's first destination byte or was written
// by an earlier step), D < G uses out[pos - D + (k mod D)].
// At the end the group writes the region's output to the slot with 16-byte
// stores.  Anything unusual (errors, mid-stream MetaReset, wide metas, long
// lengths/offsets, a full slot or region) hands the stream to the exact
// decoder through the slow list, as k2_fast does.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"

namespace ez {
namespace {

// 8 bytes at byte address a of LDS (any alignment): three dword reads
__device__ __forceinline__ uint64_t lds_u64(const uint32_t *w, uint32_t a) {
    const uint32_t k = a >> 2, sh = a & 3;
    const uint32_t w0 = w[k], w1 = w[k + 1], w2 = w[k + 2];
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}

template <int G>
__global__ __launch_bounds__(64) void k2_grp(DecompressArgs A, uint32_t R) {
    constexpr int S = 64 / G;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)(threadIdx.x & 63);
    const int g = lane / G, lj = lane % G;
    const uint64_t s = (uint64_t)blockIdx.x * S + g;
    const bool have = s < A.count;

    uint8_t *reg = smem + (uint32_t)g * R;  // this stream's region (16-byte aligned)
    const uint32_t *regw = (const uint32_t *)reg;
    int32_t nb = 0, cap = 0;
    const uint8_t *gb = A.in;
    if (have) {
        const uint64_t n64 = A.in_off[s + 1] - A.in_off[s];
        const uint64_t c64 = A.out_off[s + 1] - A.out_off[s];
        gb = A.in + A.in_off[s];
        nb = n64 > (uint64_t)R ? (int32_t)R + 1 : (int32_t)n64;
        cap = c64 > (uint64_t)(1u << 30) ? (int32_t)(1u << 30) : (int32_t)c64;
    }
    // staging: the aligned words of the stream at the region's top, 16 bytes of pad after
    const uint32_t r = (uint32_t)((uintptr_t)gb & 3);
    const uint32_t *gw = (const uint32_t *)(gb - r);
    const int32_t nw = (int32_t)((r + (uint32_t)nb + 3) >> 2);
    const int32_t wb = (int32_t)(R >> 2) - 4 - nw;  // first staged word
    bool slow = have && wb < 0;
    const bool go = have && !slow && nb > 0;
    if (go) {
        uint32_t *lw = (uint32_t *)reg + wb;
        for (int32_t k = lj; k < nw; k += G) lw[k] = gw[k];
    }
    __syncthreads();  // one wave: orders the staging before the parse's reads
    const uint32_t ib = 4u * (uint32_t)(wb < 0 ? 0 : wb) + r;  // region byte of input byte 0
    const int64_t limit = A.block_size_limit;

    int32_t i = 0, pos = 0, bsl = -1;
    bool live = go;
    uint64_t lo = live ? lds_u64(regw, ib) : 0;
    while (__ballot(live) != 0) {
        // ---- parse one token (every lane of the group computes the same values, by selects)
        int32_t L = 0, D = 0, src = 0;
        bool cp = false;
        if (live) {
            const uint32_t w0 = (uint32_t)lo, w1 = (uint32_t)(lo >> 32);
            const uint32_t t0 = w0 & 0xff, l7 = t0 & 0x7f;
            const bool pad = t0 == 0, meta = t0 == 0x80;
            // padding (reader.go:221-224): the zero bytes of the window at once
            const int32_t pad_adv = w0 ? (int32_t)(__builtin_ctz(w0) >> 3) : (w1 ? 4 + (int32_t)(__builtin_ctz(w1) >> 3) : 8);
            // meta (continueMetaTag reader.go:272-325): header metas and breaks only
            const uint32_t mb = (w0 >> 8) & 0xff, mt = mb & 0xf8, ml = mb & 7;
            const int32_t mln = ml == 7 ? 0 : (1 << ml);
            const uint32_t marg = (w0 >> 16) & 0xff;
            const bool m_brk = mt == kMetaBreak && mln == 0;
            const bool m_rst = mt == kMetaReset && mln == 1 && marg <= 32 && pos == 0 &&
                               (limit == 0 || (1ll << marg) <= limit);
            const bool m_ver = mt == kMetaVer && mln == 1 && marg == 0;
            const bool m_mag = mt == kMetaMagic && mln == 4 && ((w0 >> 16) | (w1 << 16)) == 0x797a6165u;
            const bool m_bad = ml == 6 || i + 2 + mln > nb || !(m_brk || m_rst || m_ver || m_mag);
            // Decoder.Tag reader.go:346-392, Decoder.Offset :394-420 (1-3 byte forms)
            const uint32_t lx = (w0 >> 8) | (w1 << 24);
            const int32_t Lt = l7 < 124 ? (int32_t)l7 : (l7 == 124 ? 124 + (int32_t)(lx & 0xff) : 380 + (int32_t)(lx & 0xffff));
            const uint32_t j = l7 < 124 ? 1 : (l7 == 124 ? 2 : 3);
            const bool c = (t0 & 0x80) != 0;
            const uint32_t x = (uint32_t)(lo >> (8 * j));  // the offset's bytes (<= 4 needed)
            const bool lng = (x & 0xff) == 0xff;
            const uint32_t y = lng ? (uint32_t)(lo >> (8 * j + 8)) : x;
            const uint32_t o = y & 0xff, ox = y >> 8;
            const int32_t D0 = o < 252 ? (int32_t)o : (o == 252 ? 252 + (int32_t)(ox & 0xff) : 508 + (int32_t)(ox & 0xffff));
            const uint32_t k = o < 252 ? 1 : (o == 252 ? 2 : 3);
            const int32_t Dt = lng ? D0 : D0 + Lt;
            const int32_t tadv = c ? (int32_t)(j + (lng ? 1 : 0) + k) : (int32_t)j + Lt;
            const int32_t bs = bsl < 0 ? 0 : (bsl >= 31 ? 0x7fffffff : (1 << bsl));
            const int32_t ip = (int32_t)ib + i;  // region byte of this token
            // 5-byte lengths / offsets, LenAlt/OffAlt, BlockSizeLimit, missed meta,
            // truncation, the slot, the region, distance > window: the exact decoder
            const bool t_bad = l7 >= 126 || (c && o >= 254) || (limit != 0 && Lt > limit) || bs == 0 ||
                               pos + Lt > cap || i + (c ? tadv : (int32_t)j + Lt) > nb || (c && Dt > bs) ||
                               (c ? pos + Lt > ip + tadv : pos > ip + (int32_t)j);
            const bool bad = meta ? m_bad : (!pad && t_bad);
            const bool tok = !pad && !meta && !bad;
            bsl = meta && m_rst ? (int32_t)marg : bsl;
            L = tok ? Lt : 0;
            cp = tok && c;
            D = Dt;
            src = c ? pos - Dt : ip + (int32_t)j;
            const int32_t adv = pad ? pad_adv : (meta ? 2 + mln : tadv);
            slow = bad;
            i += adv;
            live = !bad && i < nb;
            if (live) lo = lds_u64(regw, ib + (uint32_t)i);  // the next header, read beside this move
        }
        // ---- move L bytes, one byte per lane per step
        const bool run = cp && D < G;  // short-period run or zero region
        for (int32_t base = 0; __ballot(base < L) != 0; base += G) {
            const int32_t k = base + lj;
            if (k < L) {
                int32_t y = src + k;
                if (run) y = D == 0 ? -1 : src + (int32_t)((uint32_t)k % (uint32_t)D);
                const uint32_t v = reg[y < 0 ? 0 : y];
                reg[pos + k] = (uint8_t)(y < 0 ? 0u : v);  // before the stream start: the fresh ring's zeros
            }
        }
        pos += L;
    }
    if (!have) return;
    if (slow) {
        if (lj == 0) {
            const uint32_t at = atomicAdd(&A.slow[0], 1u);
            A.slow[1 + at] = (uint32_t)s;
        }
        return;
    }
    // ---- the decoded bytes to the slot: 16 bytes per lane per step
    uint8_t *out = A.out + A.out_off[s];
    for (int32_t k = 16 * lj; k < pos; k += 16 * G) {
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

int grp_g() {
    static const int g = getenv("EZ_K2_G") ? atoi(getenv("EZ_K2_G")) : 16;
    return g == 8 || g == 32 ? g : 16;
}

template <int G>
hipError_t launch_g(const DecompressArgs &a, uint32_t R, hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        (void)hipFuncSetAttribute((const void *)k2_grp<G>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    constexpr int S = 64 / G;
    const uint64_t grid = (a.count + S - 1) / S;
    hipLaunchKernelGGL(k2_grp<G>, dim3((unsigned)grid), dim3(64), (size_t)R * S + 16, st, a, R);
    return hipGetLastError();
}

}  // namespace

// LDS region per stream for a batch whose largest output slot is max_out
// (0 = not usable: unknown or too large for LDS residency)
uint32_t grp_decode_region(uint64_t max_out) {
    if (max_out == 0 || max_out > 32768) return 0;
    const uint64_t R = (max_out + 64 + 64 + 15) & ~15ull;
    if (R * (64 / grp_g()) + 16 > 160 * 1024) return 0;
    return (uint32_t)R;
}

hipError_t launch_decompress_grp(const DecompressArgs &a, uint32_t R, hipStream_t st) {
    const int G = grp_g();
    return G == 8 ? launch_g<8>(a, R, st) : (G == 32 ? launch_g<32>(a, R, st) : launch_g<16>(a, R, st));
}

}  // namespace ez
