// ez_decompress.hip — K2: eazy decompression on gfx950.
//
// Restates Reader.Read's inner loop (reader.go:116-141 without more()),
// read (:143-216), readTag (:218-270), continueMetaTag (:272-325),
// reset (:327-344) and the Decoder (:346-514).  One wave64 per stream: the
// token parse is wave-uniform (scalar control flow, every lane agrees); the
// bytes of each token are produced by all 64 lanes.
//
// The window ring is not materialised: output is linear, so block[x & mask]
// is the output byte at block position x (0 for x < 0: a fresh ring,
// SURVEY A.12).  A back-reference of distance D produces
// out[pos+k] = out[pos - D + (k mod D)], always reading bytes written by
// earlier tokens, so every token is one hazard-free parallel pass.
#include "ez_format.h"
#include "ez_internal.h"
#include "ez_wave.h"
#include "ez_bytes.h"

#include <string.h>

namespace ez {
namespace {

struct Dec {
    // decoder state (reader.go:23-34)
    int64_t bs, mask, pos, off, len;
    int state, ver;
    int64_t detail;
    uint8_t *blk;  // blk[y] = byte at block position y (y >= max(0, pos - bs))
    // input (reader.go:36-39)
    const uint8_t *b;
    int64_t nb, boff;
    // config (reader.go:27-30)
    int64_t limit;
    bool req_magic, skip_meta;
};

// Reader.reset reader.go:327-344 (the ring is the linear output from here on)
__device__ __forceinline__ void d_reset(Dec &d, int64_t bsl) {
    d.bs = (int64_t)1 << bsl;
    d.blk = d.blk + d.pos;  // next output byte is block position 0
    d.pos = 0;
    d.mask = d.bs - 1;
    d.state = 0;
}

// continueMetaTag reader.go:272-325 -> err, *io = i
__device__ int d_continue_meta(Dec &d, int64_t st, int64_t *io) {
    int64_t i = st;
    st--;
    int64_t meta, l;
    int err = dec_meta(d.b, d.nb, i, &meta, &l, &i);
    if (err) { *io = i; return err; }
    if (d.boff == 0 && st == 0 && meta != kMetaMagic && d.req_magic) { *io = st; return EZ_ENOMAGIC; }
    if (i + l > d.nb) { *io = st; return EZ_ESHORTBUF; }
    const int64_t j = meta >> 3;
    if (j < 4) {
        const int64_t want = j == 0 ? 4 : (j == 3 ? 0 : 1);  // tagLen {4,1,1,0}
        if (l != want) { *io = st; return EZ_EUNSUPMETA; }
    }
    if (meta == kMetaMagic) {
        if (d.b[i] != 'e' || d.b[i + 1] != 'a' || d.b[i + 2] != 'z' || d.b[i + 3] != 'y') { *io = st; return EZ_EBADMAGIC; }
    } else if (meta == kMetaVer) {
        d.ver = d.b[i];
        if (d.ver > EZ_VERSION) { d.detail = d.ver; *io = st; return EZ_EUNSUPVER; }
    } else if (meta == kMetaReset) {
        const int64_t bsl = d.b[i];
        if (bsl > 32 || l != 1 || (d.limit != 0 && ((int64_t)1 << bsl) > d.limit)) { *io = st; return EZ_EOVERFLOW; }
        d_reset(d, bsl);
    } else if (meta == kMetaBreak) {
        *io = i + l;
        return EZ_EBREAK;
    } else if (!d.skip_meta) {
        d.detail = meta;
        *io = st;
        return EZ_EUNSUPMETA;
    }
    *io = i + l;
    return EZ_OK;
}

// readTag reader.go:218-270
__device__ int d_read_tag(Dec &d, int64_t st, int64_t *io) {
    int64_t i = st;
    while (i < d.nb && d.b[i] == 0) i++;  // skip zero padding
    st = i;
    int tag;
    int64_t l;
    int err = dec_tag(d.b, d.nb, st, &tag, &l, &i);
    if (err) { *io = st; return err; }
    if (d.boff == 0 && st == 0 && d.b[st] != kMeta && d.req_magic) { *io = st; return EZ_ENOMAGIC; }
    if (tag == kMeta && l == 0) return d_continue_meta(d, i, io);
    if (d.limit != 0 && l > d.limit) { *io = st; return EZ_EBLOCKLIMIT; }
    if (tag == kLiteral) {
        d.state = 'l';
        d.off = 0;
    } else {
        int64_t off;
        err = dec_offset(d.b, d.nb, i, l, &off, &i);
        if (err) { *io = st; return err; }
        if (off > d.bs) { *io = st; return EZ_EOVERFLOW; }
        d.off = d.pos - off;
        d.state = 'c';
    }
    d.len = l;
    *io = i;
    return EZ_OK;
}

// Reader.read reader.go:143-216; produces at most plen bytes at blk+pos.
// dry: compute but store nothing (capacity probe).
__device__ int d_read(Dec &d, int64_t plen, int64_t st, int64_t *nout, int64_t *io, bool dry, int lane) {
    int64_t i = st;
    *nout = 0;
    while (d.state == 0) {
        const int err = d_read_tag(d, i, &i);
        if (err) { *io = i; return err; }
    }
    if (d.bs == 0) { *io = st; return EZ_EMISSEDMETA; }
    if (d.state == 'l' && i == d.nb) { *io = i; return EZ_ESHORTBUF; }
    int64_t end = d.len < plen ? d.len : plen;
    uint8_t *p = d.blk + d.pos;
    if (d.state == 'l') {
        const int64_t avail = d.nb - i;
        if (end > avail) end = avail;
        if (!dry) {
            const uint8_t *src = d.b + i;
            for (int64_t k = lane; k < end; k += kWave) p[k] = src[k];
        }
        i += end;
    } else if (d.off == d.pos) {  // zero region (off+len <= pos is impossible here for len > 0)
        if (!dry) for (int64_t k = lane; k < end; k += kWave) p[k] = 0;
    } else {
        // back-reference: non-overlapping (off+len <= pos) or runlen
        const int64_t D = d.pos - d.off;
        if (!dry) {
            const uint8_t *blk = d.blk;
            const int64_t off = d.off;
            if (D >= end) {
                for (int64_t k = lane; k < end; k += kWave) {
                    const int64_t y = off + k;
                    p[k] = y < 0 ? 0 : blk[y];
                }
            } else {
                int64_t m = lane % D;
                const int64_t step = kWave % D;
                for (int64_t k = lane; k < end; k += kWave) {
                    const int64_t y = off + m;
                    p[k] = y < 0 ? 0 : blk[y];
                    m += step;
                    if (m >= D) m -= D;
                }
            }
        }
        d.off += end;
    }
    d.len -= end;
    d.pos += end;
    if (d.len == 0) d.state = 0;
    *nout = end;
    *io = i;
    return EZ_OK;
}

// Reader.Read reader.go:116-133 minus more(): until p is full, the input
// runs short (EZ_ESHORTBUF) or another error.
__device__ int d_read_loop(Dec &d, int64_t plen, int64_t *i, int64_t *nout, bool dry, int lane) {
    int64_t n = 0;
    int err = EZ_OK;
    while (n < plen && err == EZ_OK) {
        int64_t m;
        err = d_read(d, plen - n, *i, &m, i, dry, lane);
        n += m;
        if (n == plen) break;
        if (err == EZ_ESHORTBUF) break;
    }
    *nout = n;
    return err;
}


// ---------------------------------------------------------------------------
// K2-fast: one lane per stream (batch mode).  A lane parses its stream's
// tokens serially and expands them with 16-byte moves; 64 streams advance in
// parallel per wave, so the per-token parse cost is shared by 64 tokens.
// It restates the same reader.go semantics for the common case only: header
// metas (magic / version 0 / reset before any output), padding, breaks
// (skipped), literal and copy tokens.  Any other condition — an error of any
// kind, a mid-stream MetaReset, an unsupported or wide meta, a length over
// BlockSizeLimit, a full output slot, a truncated token — hands the stream to
// the exact wave-per-stream decoder (k2_decompress over A.slow), which
// recomputes it from scratch.
//
// Lanes of a wave sit at different points of different streams, so the loop
// body is written to be uniform: every lane runs the same instruction
// sequence each iteration (parse by selects, one predicated 16-byte load,
// one 16-byte store); only rare events (metas, slot tails, errors) branch.

#ifndef EZ_EXP
#define EZ_EXP 0  // timing experiments only (1: no stores, 2: no data loads, 3: neither)
#endif

// One iteration = (parse the token whose header was loaded by the previous
// iteration) + (one 16-byte move).  The move's source load and the next
// header's load are issued together: a lane waits for memory once per
// iteration, and the hardware's unaligned loads do all byte alignment.
// Rare cases (metas, long lengths, runs shorter than 16, references before
// the slot, the batch's last bytes, slot tails) take branches.
__device__ __forceinline__ void fast_one(const DecompressArgs &A, const uint64_t s) {
    const uint8_t *b = A.in + A.in_off[s];
    const int64_t nb64 = (int64_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint8_t *in_end = A.in + A.in_off[A.count];  // loads never pass the last stream's end
    uint8_t *out = A.out + A.out_off[s];
    const int64_t cap64 = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    const int64_t limit = A.block_size_limit;
    // 32-bit positions; clamped loads need >= 16 input bytes in the batch and a 16-byte slot
    bool slow = in_end - A.in < 16 || nb64 >= (1ll << 30) || cap64 >= (1ll << 30) || cap64 < 16;
    const int32_t nb = slow ? 0 : (int32_t)nb64, cap = (int32_t)cap64;
    int32_t i = 0, pos = 0, bsl = -1;  // bsl: log2 of the window after MetaReset (-1: none yet)
    V16 h{0, 0};                       // 16 bytes at b + i (the next header)
    if (!slow) h = b + 16 <= in_end ? ld16v(b) : ld_clamped(b, A.in, in_end);
    // the token being written: rem bytes at out + dst from sp (input or output)
    int32_t rem = 0, dst = 0, step = 16;
    const uint8_t *sp = b;
    bool from_in = false, patt = false;
    V16 pv{0, 0};
#if EZ_EXP == 1 || EZ_EXP == 3
    uint64_t sinkv = 0;
#endif
    for (;;) {
        if (rem == 0) {
            if (i >= nb) break;
            const uint64_t lo = h.lo;
            const uint32_t t0 = (uint32_t)lo & 0xff, l7 = t0 & 0x7f;
            int32_t adv;
            if (t0 == 0 || t0 == 0x80) {
                if (t0 == 0) {  // padding (reader.go:221-224), a run of zero bytes at once
                    adv = lo ? (int32_t)(__builtin_ctzll(lo) >> 3) : (h.hi ? 8 + (int32_t)(__builtin_ctzll(h.hi) >> 3) : 16);
                } else {
                    // meta (continueMetaTag reader.go:272-325): header metas and breaks only
                    const uint32_t mb = (uint32_t)(lo >> 8) & 0xff, mt = mb & 0xf8, ml = mb & 7;
                    const int32_t mln = ml == 7 ? 0 : (1 << ml);
                    const uint32_t marg = (uint32_t)(lo >> 16) & 0xff;
                    const bool m_brk = mt == kMetaBreak && mln == 0;
                    const bool m_rst = mt == kMetaReset && mln == 1 && marg <= 32 && pos == 0 && (limit == 0 || (1ll << marg) <= limit);
                    const bool m_ver = mt == kMetaVer && mln == 1 && marg == 0;
                    const bool m_mag = mt == kMetaMagic && mln == 4 && (uint32_t)(lo >> 16) == 0x797a6165u;
                    if (ml == 6 || i + 2 + mln > nb || !(m_brk || m_rst || m_ver || m_mag)) { slow = true; break; }
                    if (m_rst) bsl = (int32_t)marg;
                    adv = 2 + mln;
                }
            } else {
                // Decoder.Tag reader.go:346-392 and Decoder.Offset :394-420, by selects
                const uint32_t lx = (uint32_t)(lo >> 8);
                const int64_t L = l7 < 124 ? (int64_t)l7
                                : (l7 == 124 ? 124 + (int64_t)(lx & 0xff) : (l7 == 125 ? 380 + (int64_t)(lx & 0xffff) : 65916 + (int64_t)lx));
                const uint32_t j = l7 < 124 ? 1 : (l7 == 124 ? 2 : (l7 == 125 ? 3 : 5));
                const bool cp = (t0 & 0x80) != 0;
                const uint64_t x = fun8(lo, h.hi, j);  // bytes from the offset on (header <= 11 bytes)
                const bool lng = (x & 0xff) == 0xff;
                const uint64_t y = lng ? fun8(lo, h.hi, j + 1) : x;
                const uint32_t o = (uint32_t)y & 0xff, ox = (uint32_t)(y >> 8);
                const int64_t D0 = o < 252 ? (int64_t)o : (o == 252 ? 252 + (int64_t)(ox & 0xff) : (o == 253 ? 508 + (int64_t)(ox & 0xffff) : 66044 + (int64_t)ox));
                const uint32_t k = o < 252 ? 1 : (o == 252 ? 2 : (o == 253 ? 3 : 5));
                const int64_t D = lng ? D0 : D0 + L;
                adv = cp ? (int32_t)(j + (lng ? 1 : 0) + k) : (int32_t)(j + L);
                const int64_t bs = bsl < 0 ? 0 : (1ll << bsl);
                const bool bad = l7 == 127 || (cp && o == 255) || (limit != 0 && L > limit) || bs == 0 ||
                                 pos + L > cap || (int64_t)i + (cp ? (int64_t)adv : (int64_t)j + L) > nb || (cp && D > bs);
                if (bad) { slow = true; break; }  // the exact decoder takes the stream
                dst = pos;
                rem = (int32_t)L;
                pos += (int32_t)L;
                from_in = !cp;
                sp = cp ? out + (dst - (int32_t)D) : b + (i + (int32_t)j);
                patt = cp && D < 16;
                step = 16;
                if (patt) {
                    // zero region (D == 0, reader.go:176-179) or a short-period run:
                    // one 16-byte pattern stored every `step` bytes
                    if (D == 0) {
                        pv = V16{0, 0};
                    } else {
                        const uint32_t per = (uint32_t)D;
                        pv = run_pattern(shr16(ld_clamped(out + dst - 16, out, out + cap), 16 - per), per);
                        step = (int32_t)(per * (16 / per));
                    }
                }
            }
            i += adv;
            // the next header, loaded beside this token's first move
            if (i < nb) h = b + i + 16 <= in_end ? ld16v(b + i) : ld_clamped(b + i, A.in, in_end);
        }
        if (rem > 0) {
            V16 v;
#if EZ_EXP != 2 && EZ_EXP != 3
            // inputs near the batch end / references before the slot read zeros there (rare)
            if (from_in ? sp + 16 > in_end : sp < out) v = from_in ? ld_clamped(sp, A.in, in_end) : ld_clamped(sp, out, out + cap);
            else v = ld16v(sp);
#else
            v = V16{(uint64_t)sp, h.lo};
#endif
            if (patt) v = pv;
#if EZ_EXP != 1 && EZ_EXP != 3
            if (rem >= 16 || dst + 16 <= cap) st16v(out + dst, v);
            else put_small(out + dst, v, (uint32_t)rem);
#else
            sinkv ^= v.lo;
#endif
            const int32_t kk = rem < step ? rem : step;
            dst += kk;
            sp += kk;
            rem -= kk;
        }
    }
#if EZ_EXP == 1 || EZ_EXP == 3
    if (sinkv == 0x123456789ull) pos++;
#endif
    if (slow) {
        const uint32_t at = atomicAdd(&A.slow[0], 1u);
        A.slow[1 + at] = (uint32_t)s;
    } else {
        A.out_size[s] = (uint64_t)pos;
        if (A.status) A.status[s] = EZ_OK;
    }
}

// grid-stride over streams (EZ_K2_WAVES caps the streams in flight, experiments)
// spw: streams per wave (64 = every lane; fewer = more waves per SIMD to hide latency)
__global__ __launch_bounds__(256) void k2_fast(DecompressArgs A, uint32_t spw) {
    const uint64_t todo = A.todo ? (uint64_t)A.todo[0] : A.count;
    const uint32_t l = threadIdx.x & 63;
    if (l >= spw) return;
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t k = w * spw + l; k < todo; k += nw * spw) fast_one(A, A.todo ? (uint64_t)A.todo[1 + k] : k);
}

__global__ __launch_bounds__(64) void k2_decompress(DecompressArgs A) {
    const int lane = lane_id();
    const uint64_t todo = A.slow ? (uint64_t)A.slow[0] : A.count;
    for (uint64_t k = blockIdx.x; k < todo; k += gridDim.x) {
        const uint64_t s = A.slow ? (uint64_t)A.slow[1 + k] : k;
        Dec d;
        d.b = A.in + A.in_off[s];
        d.nb = (int64_t)(A.in_off[s + 1] - A.in_off[s]);
        d.limit = A.block_size_limit;
        d.req_magic = A.require_magic != 0;
        d.skip_meta = A.skip_unsupported_meta != 0;
        uint8_t *out = A.out + A.out_off[s];
        const int64_t cap = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
        if (A.handle) {
            DecodeState &S = *A.st;
            d.bs = S.bs; d.mask = S.bs ? S.bs - 1 : 0; d.pos = S.pos; d.off = S.off; d.len = S.len;
            d.state = S.state; d.ver = S.ver; d.detail = 0; d.boff = A.boff;
            d.blk = out - d.pos;  // the kernel's launcher keeps min(pos, bs) bytes of history before out
            int64_t i = S.i, n = 0;
            const int err = d_read_loop(d, cap, &i, &n, false, lane);
            if (lane == 0) {
                S.bs = d.bs; S.pos = d.pos; S.off = d.off; S.len = d.len; S.state = d.state; S.ver = d.ver;
                S.i = i; S.n = n; S.detail = d.detail; S.err = err;
                S.hist = d.bs == 0 ? 0 : (d.pos < d.bs ? d.pos : d.bs);
            }
            return;
        }
        // batch: NewReaderBytes(in) read until EOF, ErrBreak skipped
        d.bs = 0; d.mask = 0; d.pos = 0; d.off = 0; d.len = 0; d.state = 0; d.ver = 0; d.detail = 0;
        d.boff = 0;
        d.blk = out;
        int64_t i = 0, total = 0;
        int err = EZ_OK;
        for (int64_t guard = 0;; guard++) {
            if (guard > d.nb + 64) { err = EZ_ESTUCK; break; }
            const int64_t left = cap - total;
            int64_t m;
            if (left > 0) {
                err = d_read_loop(d, left, &i, &m, false, lane);
            } else {
                err = d_read_loop(d, 1, &i, &m, true, lane);
                if (m > 0) { err = EZ_ENOSPC; break; }
            }
            total += m;
            if (err == EZ_OK || err == EZ_EBREAK) continue;
            if (err == EZ_ESHORTBUF) err = (d.state != 0 || i < d.nb) ? EZ_EUNEXPECTEDEOF : EZ_OK;
            break;
        }
        if (lane == 0) {
            A.out_size[s] = (uint64_t)total;
            if (A.status) A.status[s] = err;
        }
    }
}

}  // namespace

// two stream lists: K2g -> k2_fast hand-overs, k2_fast -> exact decoder hand-overs
static int g_decompress_variant = -1;  // -1: not read yet; 0: automatic; 'f', 'g', 'r', 'w'
void select_decompress_variant(int v) { g_decompress_variant = v; }

uint64_t decompress_workspace_words(uint64_t count) { return 2 * count + 32; }

hipError_t launch_decompress(const DecompressArgs &a, hipStream_t st) {
    if (a.count == 0) return hipSuccess;
    if (a.handle || !a.slow) {
        uint64_t grid = a.count < (1u << 30) ? a.count : (1u << 30);
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, a);
        return hipGetLastError();
    }
    // EZ_K2=exact (experiments): the exact decoder alone
    static const bool use_exact = getenv("EZ_K2") && strcmp(getenv("EZ_K2"), "exact") == 0;
    static const uint64_t long_slot = getenv("EZ_K2_LONG") ? (uint64_t)atoll(getenv("EZ_K2_LONG")) : (64u << 10);
    if (use_exact) {
        DecompressArgs b = a;
        b.slow = nullptr;
        uint64_t grid = b.count < (1u << 30) ? b.count : (1u << 30);
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, b);
        return hipGetLastError();
    }
    hipError_t e = hipMemsetAsync(a.slow, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    if (g_decompress_variant < 0) {
        const char *v = getenv("EZ_K2");
        g_decompress_variant = v && strcmp(v, "group") == 0 ? 'g' : (v && strcmp(v, "fast") == 0 ? 'f' : (v && strcmp(v, "wave") == 0 ? 'w' : 0));
    }
    if (g_decompress_variant == 'w' || (g_decompress_variant == 0 && a.max_out >= long_slot)) {
        // long streams (slots of 64 KiB and more, C2/C4): too few to give every lane one;
        // K2w gives each a wave, and its hand-overs go to the exact decoder
        e = launch_decompress_wave(a, st);
        if (e != hipSuccess) return e;
        const uint64_t grid = a.count < 4096 ? a.count : 4096;
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, a);
        return hipGetLastError();
    }
    // K2g (LDS group decoder) first when the slots are small; its hand-overs go
    // through k2_fast, whose hand-overs go to the exact decoder
    // K2g is opt-in: at C1 the lane-per-stream decoder is faster
    const uint32_t RG = g_decompress_variant == 'g' ? group_decode_region(a.max_out) : 0;
    if (RG) {
        uint32_t *list2 = a.slow + a.count + 16;
        e = hipMemsetAsync(list2, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return e;
        e = launch_decompress_group(a, RG, st);
        if (e != hipSuccess) return e;
        DecompressArgs f = a;
        f.todo = a.slow;
        f.slow = list2;
        const uint64_t fgrid = (a.count + 255) / 256;
        hipLaunchKernelGGL(k2_fast, dim3((unsigned)fgrid), dim3(256), 0, st, f, 64u);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        const uint64_t grid = a.count < 4096 ? a.count : 4096;
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, f);
        return hipGetLastError();
    }
    if (g_decompress_variant != 'f') {
        // K2r (default): k2_fast with the recent output in an LDS ring
        e = launch_decompress_ring(a, st);
        if (e != hipSuccess) return e;
        const uint64_t grid = a.count < 4096 ? a.count : 4096;
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, a);
        return hipGetLastError();
    }
    static const unsigned blk = getenv("EZ_K2_BLOCK") ? (unsigned)atoi(getenv("EZ_K2_BLOCK")) : 256u;
    static const uint64_t maxw = getenv("EZ_K2_WAVES") ? (uint64_t)atoll(getenv("EZ_K2_WAVES")) : 0;
    static const uint32_t spw = getenv("EZ_K2_SPW") ? (uint32_t)atoi(getenv("EZ_K2_SPW")) : 64u;
    const uint64_t lanes = (a.count + spw - 1) / spw * 64;  // threads launched
    uint64_t fgrid = (lanes + blk - 1) / blk;
    if (maxw && fgrid * blk / 64 > maxw) fgrid = (maxw * 64 + blk - 1) / blk;
    hipLaunchKernelGGL(k2_fast, dim3((unsigned)fgrid), dim3(blk), 0, st, a, spw);
    // exact decoder over the handed-over streams (count read on the device)
    uint64_t grid = a.count < 4096 ? a.count : 4096;
    hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace ez
