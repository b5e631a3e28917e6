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

#include <atomic>

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
        // (a stream a fast decoder handed over is recomputed from its start: so are its breaks)
        if (A.breaks && lane == 0) A.breaks[0] = 0;
        // K2t found the slot too small (a caller sizing its slot, end_state[0] = -2): no re-decode
        if (A.end_state && A.end_state[0] == -2) {
            if (lane == 0) {
                A.out_size[s] = 0;
                if (A.status) A.status[s] = EZ_ENOSPC;
            }
            continue;
        }
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
            if (err == EZ_EBREAK && A.breaks && lane == 0) {
                const uint64_t at = A.breaks[0]++;
                if (at < A.breaks_cap) A.breaks[1 + at] = (uint64_t)total;
            }
            if (err == EZ_OK || err == EZ_EBREAK) continue;
            if (err == EZ_ESHORTBUF) err = (d.state != 0 || i < d.nb) ? EZ_EUNEXPECTEDEOF : EZ_OK;
            break;
        }
        if (lane == 0) {
            A.out_size[s] = (uint64_t)total;
            if (A.status) A.status[s] = err;
            if (A.end_state) {
                A.end_state[0] = d.bs;
                A.end_state[1] = d.pos;
            }
        }
    }
}

}  // namespace

// the batch decoders: K2r (lane per stream, slots < 64 KiB) or K2t (token-parallel wave per stream,
// longer slots), each handing the streams it does not finish to the exact decoder; 'r', 't' / 'w'
// force one (tests, A/B; K2w is reached only this way)
static std::atomic<int> g_decompress_variant{-1};  // -1: not read yet; 0: automatic; 'r', 't', 'w', 'j'
void select_decompress_variant(int v) { g_decompress_variant = v; }
// the first K2 kernel of the last batch decode ('e': exact alone); atomic: the multi-device batches
// decode their shards on several host threads
static std::atomic<int> g_last_variant{0};
int last_decompress_variant() { return g_last_variant; }

// [slow list: 2 * count + 32 words][K2w / K2t's deferred literals: 4 words + count * kDefSlots records]
uint64_t decompress_workspace_words(uint64_t count) {
    return 2 * count + 32 + 4 + count * (uint64_t)kDefSlots * (sizeof(DeferLit) / 4);
}

namespace {
// the largest output slot of a batch (saturated at 2^32 - 1) into *mx
__global__ void k_max_slot(const uint64_t *out_off, uint64_t count, uint32_t *mx) {
    uint64_t m = 0;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < count; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t d = out_off[s + 1] - out_off[s];
        m = d > m ? d : m;
    }
    atomicMax(mx, (uint32_t)(m > 0xffffffffull ? 0xffffffffull : m));
}
}  // namespace

// The decoder a batch takes depends on its largest output slot: the caller's hint (ez_batch.max_len)
// when given, else measured here (one small kernel and a 4-byte read back, which waits for the stream).
static hipError_t largest_slot(const DecompressArgs &a, hipStream_t st, uint64_t *mo) {
    if (a.max_out != 0) {
        *mo = a.max_out;
        return hipSuccess;
    }
    uint32_t *mx = a.slow + 2 * a.count + 31;  // (the slow list's spare words)
    hipError_t e = hipMemsetAsync(mx, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    const uint64_t blocks = (a.count + 255) / 256;
    hipLaunchKernelGGL(k_max_slot, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), 0, st, a.out_off, a.count, mx);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    uint32_t h = 0;
    if ((e = hipMemcpyAsync(&h, mx, sizeof h, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    *mo = h;
    return hipSuccess;
}

hipError_t launch_decompress(const DecompressArgs &a0, hipStream_t st) {
    if (a0.count == 0) return hipSuccess;
    if (a0.handle || !a0.slow) {
        if (!a0.handle) g_last_variant = 'e';
        uint64_t grid = a0.count < (1u << 30) ? a0.count : (1u << 30);
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, a0);
        return hipGetLastError();
    }
    // EZ_K2=exact (experiments): the exact decoder alone
    static const bool use_exact = knob_str("EZ_K2") && strcmp(knob_str("EZ_K2"), "exact") == 0;
    static const uint64_t long_slot = (uint64_t)knob("EZ_K2_LONG", 64 << 10);
    if (use_exact) {
        g_last_variant = 'e';
        DecompressArgs b = a0;
        b.slow = nullptr;
        uint64_t grid = b.count < (1u << 30) ? b.count : (1u << 30);
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, b);
        return hipGetLastError();
    }
    DecompressArgs a = a0;
    hipError_t e = largest_slot(a0, st, &a.max_out);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.slow, 0, sizeof(uint32_t), st)) != hipSuccess) return e;
    int sel = g_decompress_variant.load();
    if (sel < 0) {
        const char *v = knob_str("EZ_K2");
        sel = v && strcmp(v, "wave") == 0 ? 'w'
              : (v && strcmp(v, "ring") == 0 ? 'r' : (v && strcmp(v, "tok") == 0 ? 't' : (v && strcmp(v, "jump") == 0 ? 'j' : 0)));
        int want = -1;
        (void)g_decompress_variant.compare_exchange_strong(want, sel);
    }
    const uint64_t exact_grid = a.count < 4096 ? a.count : 4096;
    // Slots under 64 KiB go to K2r's lane per stream; longer ones (C2, C4, the sweep's long streams) to
    // K2t (1 GiB batches, K2 ms, K2r / K2t: 8 KiB 1.89 / 4.99, 16 KiB 1.96 / 4.89, 32 KiB 3.50 / 5.06,
    // 64 KiB 6.69 / 5.31, 128 KiB 13.4 / 5.82, 256 KiB (C2; K2w 12.5) - / 7.0, 1 MiB (K2w 29.7) - / 14.4;
    // C4 fp32 K2w 0.145 / K2t 0.151, C4s 164 / 106 ms).
    int v = a.force ? a.force : (sel != 0 ? sel : (a.max_out >= long_slot ? 't' : 'r'));
    // A few long streams whose output is at least twice their input (copies, not literals) go to
    // K2j: K2t gives each stream one wave and walks its copy chains round by round, K2j the whole
    // chip (C4s, 64 x 4 MiB: K2t 93.7 ms, K2j 11.4 ms; a lone 16 MiB log stream 171 / 11.7 ms).
    // Literal-heavy buckets stay on K2t (C4 fp32 0.149 / 1.86 ms, C4h 0.31 / 2.65 ms), and so do
    // batches of more streams, whose chains K2t runs side by side (1,024 x 1 MiB: 12.9 / 58.8 ms).
    // K2j's time follows the batch's output, K2t's the longest stream's (256 x 1 MiB logs: K2t's
    // chain ~12.8 ms against K2j 15.6): K2j only while the output is at most 200 slots' worth.
    // The extents are the caller's hints (ez_batch.in_bytes / out_bytes); without them, four offsets
    // read back (which waits for the stream).
    if (v == 't' && !a.force && sel == 0 && a.count <= 256 && a.max_out >= ((uint64_t)1 << 20)) {
        uint64_t nin = 0, nout = 0;
        if ((e = batch_extents(a, st, &nin, &nout)) != hipSuccess) return e;
        a.in_bytes = nin;
        a.out_bytes = nout;
        if (nin >= (uint64_t)a.count * (64 << 10) && nout >= 2 * nin && nout <= 200 * a.max_out) v = 'j';
    }
    if (v == 'j' && !jump_applies(a)) v = 't';
    if (v == 'j') {
        // K2j: few long streams with the whole chip; its hand-overs go to the exact decoder.  Without
        // its workspace (a failed allocation, nothing launched) the batch takes K2t.
        e = launch_decompress_jump(a, st);
        if (e == hipSuccess) {
            g_last_variant = v;
            hipLaunchKernelGGL(k2_decompress, dim3((unsigned)exact_grid), dim3(64), 0, st, a);
            return hipGetLastError();
        }
        if (e != hipErrorOutOfMemory) return e;
        v = 't';
    }
    g_last_variant = v;
    if (v == 't') {
        // K2t: token-parallel, a wave per stream; its hand-overs go to the exact decoder, the long
        // literals it defers are moved last (the exact decoder writes the same bytes for a stream it takes)
        DecompressArgs b = a;
        b.defer = a.slow + 2 * a.count + 32;
        b.defer_cap = a.count * (uint64_t)kDefSlots;
        if ((e = hipMemsetAsync(b.defer, 0, 16, st)) != hipSuccess) return e;
        e = launch_decompress_tok(b, st);
        if (e != hipSuccess) return e;
#if (EZ_EXP & 4096)
        return e;  // debug builds: the hand-over codes stay in the statuses
#endif
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)exact_grid), dim3(64), 0, st, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        return launch_defer_copy(b, st);
    }
    if (v == 'w') {
        // K2w (forced: tests, A/B): a wave per stream with a scalar token walk; its hand-overs go to the
        // exact decoder; the long literals it defers are moved last
        DecompressArgs b = a;
        static const bool no_defer = knob("EZ_K2W_DEFER", 1) == 0;  // A/B
        b.defer = no_defer ? nullptr : a.slow + 2 * a.count + 32;
        b.defer_cap = a.count * (uint64_t)kDefSlots;
        if (b.defer && (e = hipMemsetAsync(b.defer, 0, 16, st)) != hipSuccess) return e;
        e = launch_decompress_wave(b, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)exact_grid), dim3(64), 0, st, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        return b.defer ? launch_defer_copy(b, st) : hipSuccess;
    }
    // K2r: one lane per stream with the recent output in an LDS ring
    e = launch_decompress_ring(a, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k2_decompress, dim3((unsigned)exact_grid), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace ez
