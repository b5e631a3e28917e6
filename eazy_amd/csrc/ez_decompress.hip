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
// kind, a mid-stream MetaReset, an unsupported or wide meta, a reference
// before the stream start, a length over BlockSizeLimit, a full output slot,
// a truncated token — hands the stream to the exact wave-per-stream decoder
// (k2_decompress over A.slow), which recomputes it from scratch.

typedef uint4 __attribute__((aligned(1))) uint4_u;
typedef unsigned __int128 u128;

__device__ __forceinline__ u128 to128(uint4 v) {
    return ((u128)((uint64_t)v.z | ((uint64_t)v.w << 32)) << 64) | ((uint64_t)v.x | ((uint64_t)v.y << 32));
}
__device__ __forceinline__ uint4 from128(u128 x) {
    const uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
__device__ __forceinline__ uint4 ld16(const uint8_t *p) { return *(const uint4_u *)p; }
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) { *(uint4_u *)p = v; }
__device__ __forceinline__ uint32_t bat(u128 h, uint32_t k) { return (uint32_t)(h >> (8 * k)) & 0xff; }
__device__ __forceinline__ uint32_t le32at(u128 h, uint32_t k) { return (uint32_t)(h >> (8 * k)); }

// 16 input bytes at q (q < end), never reading at or past `end` (bytes there
// read as 0): one clamped load shifted into place.  The launcher routes
// batches under 16 input bytes to the exact decoder.
__device__ __forceinline__ u128 ld_in(const uint8_t *q, const uint8_t *end) {
    const int64_t over = (q + 16) - end;
    if (over <= 0) return to128(ld16(q));
    const u128 x = to128(ld16(end - 16));
    return over >= 16 ? (u128)0 : x >> (8 * over);
}

// 16 bytes of a stream's output history at y (y < dst): bytes before the
// slot start read as 0 (the decoder's fresh window, reader.go:176-196).
// Needs a slot of at least 16 bytes when y < 0.
__device__ __forceinline__ u128 ld_hist(const uint8_t *out, int64_t y) {
    if (y >= 0) return to128(ld16(out + y));
    if (y <= -16) return 0;
    return to128(ld16(out)) << (8 * -y);
}

// k < 16 bytes of x at d: 8/4/2/1-byte stores, no loop
__device__ __forceinline__ void put_small(uint8_t *d, u128 x, int64_t k) {
    typedef uint64_t __attribute__((aligned(1))) u64_u;
    typedef uint32_t __attribute__((aligned(1))) u32_u;
    typedef uint16_t __attribute__((aligned(1))) u16_u;
    int64_t o = 0;
    if (k & 8) { *(u64_u *)(d + o) = (uint64_t)x; x >>= 64; o += 8; }
    if (k & 4) { *(u32_u *)(d + o) = (uint32_t)x; x >>= 32; o += 4; }
    if (k & 2) { *(u16_u *)(d + o) = (uint16_t)x; x >>= 16; o += 2; }
    if (k & 1) d[o] = (uint8_t)x;
}

// One iteration = (parse the next token from registers when the previous one
// is written) + (one 16-byte move).  All loads of an iteration — the move's
// source and the prefetch of the next 16 compressed bytes — are issued
// together, so a lane waits for memory once per iteration.
#ifndef EZ_EXP
#define EZ_EXP 0  // timing experiments only (1: no stores, 2: no data loads, 3: neither)
#endif
enum : int { M_REG = 0, M_IN = 1, M_OUT = 2, M_PAT = 3, M_PATLD = 4 };

// the low `per` bytes of x (1 <= per < 16) repeated over 16 bytes
__device__ __forceinline__ u128 run_pattern(u128 x, int32_t per) {
    x &= ((u128)1 << (8 * per)) - 1;
    x |= x << (8 * per);
    if (2 * per < 16) x |= x << (16 * per);
    if (4 * per < 16) x |= x << (32 * per);
    if (8 * per < 16) x |= x << (64 * per);
    return x;
}

__global__ __launch_bounds__(256) void k2_fast(DecompressArgs A) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= A.count) return;
    const uint8_t *b = A.in + A.in_off[s];
    int64_t nb = (int64_t)(A.in_off[s + 1] - A.in_off[s]);
    const uint8_t *in_end = A.in + A.in_off[A.count];  // loads never pass the last stream's end
    uint8_t *out = A.out + A.out_off[s];
    const int64_t cap = (int64_t)(A.out_off[s + 1] - A.out_off[s]);
    const int64_t limit = A.block_size_limit;
    int64_t i = 0, pos = 0, bs = 0;
    bool slow = in_end - A.in < 16;  // ld_in's clamped loads need 16 input bytes
    // register window over the compressed stream: bytes [wb, wb + 32); i - wb < 16 at a parse
    int64_t wb = 0;
    u128 c0 = 0, c1 = 0;
    if (!slow) {
        c0 = ld_in(b, in_end);
        c1 = ld_in(b + 16, in_end);
    } else {
        nb = 0;  // skip the loop: the exact decoder takes the stream
    }
    // the token being written: rem bytes at out + dst, from src (input or output offset)
    int64_t rem = 0, dst = 0, src = 0, Dd = 16;
    int32_t per = 0;
    int mode = M_REG;
#if EZ_EXP == 1 || EZ_EXP == 3
    u128 sinkv = 0;
#endif
    u128 v = 0;
    for (;;) {
        if (rem == 0) {
            if (i >= nb) break;
            const int64_t r = i - wb;
            const u128 h = r ? (c0 >> (8 * r)) | (c1 << (128 - 8 * r)) : c0;  // bytes i .. i+15
            const uint32_t t0 = (uint32_t)h & 0xff;
            if (t0 == 0) {  // padding (reader.go:221-224), a run of zero bytes at once
                const uint64_t lo = (uint64_t)h, hi = (uint64_t)(h >> 64);
                i += lo ? (__builtin_ctzll(lo) >> 3) : (hi ? 8 + (__builtin_ctzll(hi) >> 3) : 16);
            } else {
                // Decoder.Tag reader.go:346-392
                const uint32_t l7 = t0 & 0x7f;
                int64_t L;
                uint32_t j;
                if (l7 < 124) { L = l7; j = 1; }
                else if (l7 == 124) { L = 124 + bat(h, 1); j = 2; }
                else if (l7 == 125) { L = 380 + (le32at(h, 1) & 0xffff); j = 3; }
                else if (l7 == 126) { L = 65916 + (int64_t)le32at(h, 1); j = 5; }
                else { slow = true; break; }  // LenAlt -> ErrOverflow
                if (t0 & 0x80) {
                    if (L == 0) {
                        // meta (continueMetaTag reader.go:272-325)
                        if (i + 2 > nb) { slow = true; break; }
                        const uint32_t m = bat(h, 1);
                        const uint32_t meta = m & 0xf8, ml = m & 7;
                        int64_t ln;
                        if (ml == 7) ln = 0;
                        else if (ml < 6) ln = (int64_t)1 << ml;
                        else { slow = true; break; }  // wide meta length
                        if (i + 2 + ln > nb) { slow = true; break; }
                        if (meta == kMetaBreak && ln == 0) {
                            i += 2;  // ErrBreak: skipped in a batch
                        } else if (meta == kMetaReset && ln == 1) {
                            const uint32_t bsl = bat(h, 2);
                            if (bsl > 32 || (limit != 0 && ((int64_t)1 << bsl) > limit) || pos != 0) { slow = true; break; }
                            bs = (int64_t)1 << bsl;
                            i += 3;
                        } else if (meta == kMetaVer && ln == 1 && bat(h, 2) == 0) {
                            i += 3;
                        } else if (meta == kMetaMagic && ln == 4 && le32at(h, 2) == 0x797a6165u) {
                            i += 6;
                        } else {
                            slow = true;  // an error or an unsupported meta
                            break;
                        }
                    } else {
                        // Decoder.Offset reader.go:394-420
                        if (limit != 0 && L > limit) { slow = true; break; }
                        uint32_t o = bat(h, j);
                        const bool lng = o == 0xff;
                        if (lng) { j++; o = bat(h, j); }
                        int64_t D;
                        if (o < 252) { D = o; j += 1; }
                        else if (o == 252) { D = 252 + bat(h, j + 1); j += 2; }
                        else if (o == 253) { D = 508 + (le32at(h, j + 1) & 0xffff); j += 3; }
                        else if (o == 254) { D = 66044 + (int64_t)le32at(h, j + 1); j += 5; }
                        else { slow = true; break; }  // OffAlt
                        if (!lng) D += L;
                        if (i + j > nb || bs == 0 || D > bs || pos + L > cap || (D > pos && cap < 16)) { slow = true; break; }
                        i += j;
                        dst = pos;
                        rem = L;
                        pos += L;
                        Dd = 16;
                        if (D == 0) {  // zero region (reader.go:176-179)
                            mode = M_REG;
                            v = 0;
                        } else if (D < 16) {  // short-period run: a 16-byte pattern every Dd bytes
                            Dd = D * (16 / D);
                            per = (int32_t)D;
                            mode = M_PATLD;
                            src = dst - 16;
                        } else {
                            mode = M_OUT;
                            src = dst - D;
                        }
                    }
                } else {
                    // literal (reader.go:170-172)
                    if (limit != 0 && L > limit) { slow = true; break; }
                    if (bs == 0 || i + j + L > nb || pos + L > cap) { slow = true; break; }
                    dst = pos;
                    rem = L;
                    pos += L;
                    Dd = 16;
                    if (j + L <= 16) {  // bytes straight from the header window
                        mode = M_REG;
                        v = h >> (8 * j);
                    } else {
                        mode = M_IN;
                        src = i + j;
                    }
                    i += j + L;
                }
            }
        }
        // ---- loads of this iteration, issued together ----
        u128 raw = 0;
#if EZ_EXP != 2 && EZ_EXP != 3
        if (rem > 0 && (mode == M_IN || mode == M_OUT || mode == M_PATLD))
            raw = mode == M_IN ? ld_in(b + src, in_end) : ld_hist(out, src);
#else
        raw = c0 ^ (u128)src;
#endif
        const bool rebase = i - wb >= 32;
        u128 n0 = 0, n1 = 0;
        if (rebase) {
            n0 = ld_in(b + i, in_end);
            n1 = ld_in(b + i + 16, in_end);
        } else if (i - wb >= 16) {
            n1 = ld_in(b + wb + 32, in_end);
        }
        // ---- the move ----
        if (rem > 0) {
            if (mode == M_PATLD) {  // raw = the 16 bytes before dst; the period is its top `per` bytes
                v = run_pattern(raw >> (8 * (16 - per)), per);
                mode = M_PAT;
            } else if (mode != M_REG && mode != M_PAT) {
                v = raw;
            }
#if EZ_EXP != 1 && EZ_EXP != 3
            if (rem >= 16 || dst + 16 <= cap) st16(out + dst, from128(v));
            else put_small(out + dst, v, rem);
#else
            sinkv ^= v;
#endif
            const int64_t step = rem < Dd ? rem : Dd;
            dst += step;
            src += step;
            rem -= step;
        }
        if (rebase) {
            wb = i;
            c0 = n0;
            c1 = n1;
        } else if (i - wb >= 16) {
            wb += 16;
            c0 = c1;
            c1 = n1;
        }
    }
#if EZ_EXP == 1 || EZ_EXP == 3
    if ((uint64_t)sinkv == 0x123456789ull) pos++;
#endif
    if (slow) {
        const uint32_t at = atomicAdd(&A.slow[0], 1u);
        A.slow[1 + at] = (uint32_t)s;
    } else {
        A.out_size[s] = (uint64_t)pos;
        if (A.status) A.status[s] = EZ_OK;
    }
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

uint64_t decompress_workspace_words(uint64_t count) { return count + 16; }

hipError_t launch_decompress(const DecompressArgs &a, hipStream_t st) {
    if (a.count == 0) return hipSuccess;
    if (a.handle || !a.slow) {
        uint64_t grid = a.count < (1u << 30) ? a.count : (1u << 30);
        hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, a);
        return hipGetLastError();
    }
    hipError_t e = hipMemsetAsync(a.slow, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    static const unsigned blk = getenv("EZ_K2_BLOCK") ? (unsigned)atoi(getenv("EZ_K2_BLOCK")) : 256u;
    hipLaunchKernelGGL(k2_fast, dim3((unsigned)((a.count + blk - 1) / blk)), dim3(blk), 0, st, a);
    // exact decoder over the handed-over streams (count read on the device)
    uint64_t grid = a.count < 4096 ? a.count : 4096;
    hipLaunchKernelGGL(k2_decompress, dim3((unsigned)grid), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace ez
