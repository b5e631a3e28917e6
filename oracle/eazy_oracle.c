/*
 * eazy_oracle.c — line-by-line CPU restatement of tlog-dev/eazy
 * writer.go and reader.go (reference @ /root/reference).
 *
 * TEST INFRASTRUCTURE ONLY (see eazy_oracle.h).  Every function names the
 * reference lines it restates.  Go panics are mapped to OR_EINVAL.
 */
#include "eazy_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---- constants (writer.go:49-122) ---- */
enum {
    LITERAL = 0x00, COPY = 0x80, TAG_MASK = 0x80, TAG_LEN_MASK = 0x7f, META = 0x80,
    LEN1 = 124, LEN2 = 125, LEN4 = 126, LEN_ALT = 127,
    OFF1 = 252, OFF2 = 253, OFF4 = 254, OFF_ALT = 255, OFF_LONG = 255,
    META_MAGIC = 0 << 3, META_VER = 1 << 3, META_RESET = 2 << 3, META_BREAK = 3 << 3,
    META_TAG_MASK = 0xf8, META_LEN_MASK = 0x07, META_LEN_WIDE = 6, META_LEN0 = 7,
    MIN_COPY_CHUNK = 6,
};
#define MIB (1 << 20)

/* ---------------------------------------------------------------- Encoder */

/* Encoder.Tag writer.go:537-563 */
int or_enc_tag(uint8_t *b, size_t *len, int tag, int64_t l) {
    const int64_t reserve = 8;
    size_t k = *len;
    if (l < LEN1) { b[k++] = (uint8_t)(tag | l); *len = k; return OR_OK; }
    l -= LEN1;
    if (l < 0x100) { b[k++] = (uint8_t)(tag | LEN1); b[k++] = (uint8_t)l; *len = k; return OR_OK; }
    l -= 0x100;
    if (l < 0x10000) {
        b[k++] = (uint8_t)(tag | LEN2); b[k++] = (uint8_t)l; b[k++] = (uint8_t)(l >> 8);
        *len = k; return OR_OK;
    }
    l -= 0x10000;
    if (l < 0x100000000LL - reserve) {
        b[k++] = (uint8_t)(tag | LEN4);
        for (int s = 0; s < 32; s += 8) b[k++] = (uint8_t)(l >> s);
        *len = k; return OR_OK;
    }
    return OR_EINVAL; /* panic("too big length") */
}

/* Encoder.Offset writer.go:565-597 */
int or_enc_offset(uint8_t *b, size_t *len, int64_t off, int64_t l) {
    const int64_t reserve = 8;
    size_t k = *len;
    if (off >= l) off -= l;
    else b[k++] = OFF_LONG;
    if (off < OFF1) { b[k++] = (uint8_t)off; *len = k; return OR_OK; }
    off -= OFF1;
    if (off < 0x100) { b[k++] = OFF1; b[k++] = (uint8_t)off; *len = k; return OR_OK; }
    off -= 0x100;
    if (off < 0x10000) {
        b[k++] = OFF2; b[k++] = (uint8_t)off; b[k++] = (uint8_t)(off >> 8);
        *len = k; return OR_OK;
    }
    off -= 0x10000;
    if (off < 0x100000000LL - reserve) {
        b[k++] = OFF4;
        for (int s = 0; s < 32; s += 8) b[k++] = (uint8_t)(off >> s);
        *len = k; return OR_OK;
    }
    return OR_EINVAL; /* panic("too big offset") */
}

static int bits_len(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

/* Encoder.Meta writer.go:599-621 */
int or_enc_meta(uint8_t *b, size_t *len, int64_t meta, int64_t l) {
    if (meta & ~(int64_t)META_TAG_MASK) return OR_EINVAL; /* panic(meta) */
    size_t k = *len;
    if (l == 0) { b[k++] = META; b[k++] = (uint8_t)(meta | META_LEN0); *len = k; return OR_OK; }
    if (l < META_LEN_WIDE && (l & (l - 1)) == 0) {
        l = bits_len((uint64_t)l) - 1;
        b[k++] = META; b[k++] = (uint8_t)(meta | l); *len = k; return OR_OK;
    }
    if (l < OFF1) {
        b[k++] = META; b[k++] = (uint8_t)(meta | META_LEN_WIDE); b[k++] = (uint8_t)l;
        *len = k; return OR_OK;
    }
    b[k++] = META; b[k++] = (uint8_t)(meta | META_LEN_WIDE);
    *len = k;
    return or_enc_offset(b, len, l, 0);
}

/* ---------------------------------------------------------------- Decoder */

/* Decoder.Tag reader.go:346-392 */
int or_dec_tag(const uint8_t *b, int64_t n, int64_t st, int *tag, int64_t *l, int64_t *i_out) {
    *tag = 0; *l = 0;
    if (st >= n) { *i_out = st; return OR_ESHORTBUF; }
    int64_t i = st;
    *tag = b[i] & TAG_MASK;
    int64_t v = b[i] & TAG_LEN_MASK;
    i++;
    *l = v;
    switch (v) {
    case LEN1:
        if (i + 1 > n) { *i_out = st; return OR_ESHORTBUF; }
        v = LEN1 + (int64_t)b[i];
        i++;
        break;
    case LEN2:
        if (i + 2 > n) { *i_out = st; return OR_ESHORTBUF; }
        v = LEN1 + 0x100;
        v += (int64_t)b[i] | (int64_t)b[i + 1] << 8;
        i += 2;
        break;
    case LEN4:
        if (i + 4 > n) { *i_out = st; return OR_ESHORTBUF; }
        v = LEN1 + 0x100 + 0x10000;
        v += (int64_t)b[i] | (int64_t)b[i + 1] << 8 | (int64_t)b[i + 2] << 16 | (int64_t)b[i + 3] << 24;
        i += 4;
        break;
    case LEN_ALT:
        *i_out = st;
        return OR_EOVERFLOW;
    default:
        break;
    }
    *l = v;
    if (v < 0) { *i_out = st; return OR_EOVERFLOW; }
    *i_out = i;
    return OR_OK;
}

/* Decoder.basicOffset reader.go:422-472 */
static int dec_basic_offset(const uint8_t *b, int64_t n, int64_t st, int64_t *off, int64_t *i_out) {
    int64_t i = st;
    *off = 0;
    if (i == n) { *i_out = st; return OR_ESHORTBUF; }
    int64_t v = b[i];
    i++;
    *off = v;
    switch (v) {
    case OFF1:
        if (i + 1 > n) { *i_out = st; return OR_ESHORTBUF; }
        v = OFF1 + (int64_t)b[i];
        i++;
        break;
    case OFF2:
        if (i + 2 > n) { *i_out = st; return OR_ESHORTBUF; }
        v = OFF1 + 0x100;
        v += (int64_t)b[i] | (int64_t)b[i + 1] << 8;
        i += 2;
        break;
    case OFF4:
        if (i + 4 > n) { *i_out = st; return OR_ESHORTBUF; }
        v = OFF1 + 0x100 + 0x10000;
        v += (int64_t)b[i] | (int64_t)b[i + 1] << 8 | (int64_t)b[i + 2] << 16 | (int64_t)b[i + 3] << 24;
        i += 4;
        break;
    case OFF_ALT:
        *i_out = st;
        return OR_EOVERFLOW;
    default:
        break;
    }
    *off = v;
    if (v < 0) { *i_out = st; return OR_EOVERFLOW; }
    *i_out = i;
    return OR_OK;
}

/* Decoder.Offset reader.go:394-420 */
int or_dec_offset(const uint8_t *b, int64_t n, int64_t st, int64_t l, int64_t *off, int64_t *i_out) {
    int64_t i = st;
    *off = 0;
    if (i == n) { *i_out = st; return OR_ESHORTBUF; }
    int lng = b[i] == OFF_LONG;
    if (lng) i++;
    int64_t j;
    int err = dec_basic_offset(b, n, i, off, &j);
    if (err) { *i_out = st; return err; }
    if (!lng) *off += l;
    if (*off < 0) { *i_out = st; return OR_EOVERFLOW; }
    *i_out = j;
    return OR_OK;
}

/* Decoder.Meta reader.go:474-514 */
int or_dec_meta(const uint8_t *b, int64_t n, int64_t st, int64_t *meta, int64_t *l, int64_t *i_out) {
    int64_t i = st;
    *meta = 0; *l = 0;
    if (i == n) { *i_out = st; return OR_ESHORTBUF; }
    int64_t m = b[i];
    i++;
    *meta = m & META_TAG_MASK;
    int64_t v = m & META_LEN_MASK;
    if (v == META_LEN0) { *l = 0; *i_out = i; return OR_OK; }
    if (v < META_LEN_WIDE) { *l = (int64_t)1 << v; *i_out = i; return OR_OK; }
    if (i == n) { *l = 0; *i_out = st; return OR_ESHORTBUF; }
    v = b[i];
    i++;
    if (v < OFF1) { *l = v; *i_out = i; return OR_OK; }
    int64_t j;
    int err = dec_basic_offset(b, n, i - 1, &v, &j);
    *l = v;
    if (err) { *i_out = st; return err; }
    *i_out = j;
    return OR_OK;
}

/* ---------------------------------------------------------------- buffers */

typedef struct { uint8_t *p; int64_t len, cap; } obuf;

static void ob_reserve(obuf *b, int64_t extra) {
    if (b->len + extra <= b->cap) return;
    int64_t c = b->cap ? b->cap : 256;
    while (c < b->len + extra) c *= 2;
    b->p = (uint8_t *)realloc(b->p, (size_t)c);
    b->cap = c;
}
static void ob_put(obuf *b, const uint8_t *p, int64_t n) {
    ob_reserve(b, n);
    if (n) memcpy(b->p + b->len, p, (size_t)n);
    b->len += n;
}

/* ---------------------------------------------------------------- Writer */

struct or_writer {
    /* exported fields writer.go:23-34 */
    int append_magic;
    int64_t flush_threshold;
    int ver; /* w.e.Ver */
    /* output writer.go:36-38 */
    obuf b;
    int64_t written;
    /* window writer.go:40-45 */
    uint8_t *block;
    int64_t bs, mask, pos;
    uint32_t *ht;
    int64_t hs;
    unsigned hsh;
    /* the underlying io.Writer: an append-only Buf (eazy_test.go:1499-1505) */
    obuf sink;
    int64_t sink_accept, sink_writes;
};

/* Writer.init writer.go:161-185 */
static int w_init(or_writer *w, int64_t bs, int64_t hs) {
    if (((bs - 1) & bs) != 0 || bs < 32 || bs > ((int64_t)1 << 31)) return OR_EINVAL;
    if (((hs - 1) & hs) != 0 || hs < 4) return OR_EINVAL;
    w->mask = bs - 1;
    if (bs > w->bs) { free(w->block); w->block = (uint8_t *)calloc((size_t)bs, 1); }
    w->bs = bs;
    w->hsh = 32 - (unsigned)bits_len((uint64_t)(hs - 1));
    if (hs > w->hs) { free(w->ht); w->ht = (uint32_t *)calloc((size_t)hs, 4); }
    w->hs = hs;
    return OR_OK;
}

/* Writer.reset writer.go:187-200 */
static void w_reset(or_writer *w) {
    w->b.len = 0;
    w->pos = 0;
    w->written = 0;
    memset(w->block, 0, (size_t)w->bs);
    memset(w->ht, 0, (size_t)w->hs * 4);
}

/* NewWriter writer.go:133-145 */
or_writer *or_writer_new(int64_t block, int64_t htable) {
    or_writer *w = (or_writer *)calloc(1, sizeof(*w));
    w->append_magic = 1;
    w->sink_accept = -1;
    if (w_init(w, block, htable)) { or_writer_free(w); return NULL; }
    return w;
}

void or_writer_free(or_writer *w) {
    if (!w) return;
    free(w->block); free(w->ht); free(w->b.p); free(w->sink.p); free(w);
}
void or_writer_set_append_magic(or_writer *w, int on) { w->append_magic = on; }
void or_writer_set_version(or_writer *w, int ver) { w->ver = ver; }
void or_writer_set_flush_threshold(or_writer *w, int64_t t) { w->flush_threshold = t; }
void or_writer_set_sink_fault(or_writer *w, int64_t a) { w->sink_accept = a; }

/* Writer.isreset writer.go:403-405 */
static int w_isreset(const or_writer *w) { return w->written + w->b.len == 0; }

/* Writer.hash writer.go:491-493 */
static uint32_t w_hash(const or_writer *w, const uint8_t *p, int64_t i) {
    uint32_t x;
    memcpy(&x, p + i, 4); /* little-endian native load */
    return (uint32_t)(x * 0x1e35a7bdu) >> w->hsh;
}

/* appendMagic / appendReset / appendHeader writer.go:495-517 */
static void w_append_header(or_writer *w) {
    if (w->append_magic) {
        const uint8_t m[6] = {META, META_MAGIC | 2, 'e', 'a', 'z', 'y'};
        ob_put(&w->b, m, 6);
    }
    if (w->ver != 0) {
        const uint8_t v[3] = {META, META_VER | 0, (uint8_t)w->ver};
        ob_put(&w->b, v, 3);
    }
    const uint8_t r[3] = {META, META_RESET | 0, (uint8_t)__builtin_ctzll((uint64_t)w->bs)};
    ob_put(&w->b, r, 3);
}

static int w_tag(or_writer *w, int tag, int64_t l) {
    ob_reserve(&w->b, 16);
    size_t k = (size_t)w->b.len;
    int e = or_enc_tag(w->b.p, &k, tag, l);
    w->b.len = (int64_t)k;
    return e;
}
static int w_offset(or_writer *w, int64_t off, int64_t l) {
    ob_reserve(&w->b, 16);
    size_t k = (size_t)w->b.len;
    int e = or_enc_offset(w->b.p, &k, off, l);
    w->b.len = (int64_t)k;
    return e;
}

/* appendLiteral writer.go:519-522 */
static int w_literal(or_writer *w, const uint8_t *d, int64_t st, int64_t end) {
    int e = w_tag(w, LITERAL, end - st);
    ob_put(&w->b, d + st, end - st);
    return e;
}
/* appendCopy writer.go:524-527 */
static int w_copy(or_writer *w, int64_t st, int64_t end) {
    int e = w_tag(w, COPY, end - st);
    if (e) return e;
    return w_offset(w, w->pos - st, end - st);
}
/* copyData writer.go:529-535 */
static void w_copy_data(or_writer *w, const uint8_t *d, int64_t st, int64_t end) {
    while (st < end) {
        int64_t at = w->pos & w->mask;
        int64_t n = w->bs - at;
        if (n > end - st) n = end - st;
        memcpy(w->block + at, d + st, (size_t)n);
        st += n;
        w->pos += n;
    }
}

/* Writer.writeZeros writer.go:407-439 */
static int w_write_zeros(or_writer *w, const uint8_t *p, int64_t n, int64_t done, int64_t i,
                         int64_t *nextdone, int64_t *iend_out) {
    int64_t iend = i;
    while (iend < n && p[iend] == 0) iend++; /* the equal8 fast loop (:410-412) is equivalent */
    while (i > done && p[i - 1] == 0) i--;
    if (iend - i < MIN_COPY_CHUNK) { *nextdone = done; *iend_out = i + 1; return OR_OK; }
    if (done != i) {
        int e = w_literal(w, p, done, i);
        if (e) return e;
        w_copy_data(w, p, done, i);
    }
    int e = w_tag(w, COPY, iend - i);
    if (e) return e;
    const uint8_t z[2] = {OFF_LONG, 0};
    ob_put(&w->b, z, 2);
    w_copy_data(w, p, i, iend);
    *nextdone = iend; *iend_out = iend;
    return OR_OK;
}

static int is_zero8(const uint8_t *p) {
    uint64_t x;
    memcpy(&x, p, 8);
    return x == 0;
}

/* Writer.writeRunlen writer.go:441-489 */
static int w_write_runlen(or_writer *w, const uint8_t *p, int64_t n, int64_t done, int64_t st,
                          int64_t i, int64_t *nextdone, int64_t *iend_out) {
    if (st + 8 < n && is_zero8(p + st)) return w_write_zeros(w, p, n, done, st, nextdone, iend_out);
    int64_t jf = 0;
    while (i + jf < n && p[st + jf] == p[i + jf]) jf++;
    int64_t jb = -1;
    while (st + jb >= 0 && i + jb >= done && p[st + jb] == p[i + jb]) jb--;
    jb++;
    if (jf - jb < MIN_COPY_CHUNK) { *nextdone = done; *iend_out = i + 1; return OR_OK; }
    if (i - st >= w->bs - 8) { /* cut :464-473 */
        int64_t iend = done + i - st;
        int e = w_literal(w, p, done, iend);
        if (e) return e;
        w_copy_data(w, p, done, iend);
        *nextdone = iend; *iend_out = iend;
        return OR_OK;
    }
    int64_t ist = i + jb;
    int64_t iend = i + jf;
    int e = w_literal(w, p, done, ist); /* unconditional: may be a lone 0x00 */
    if (e) return e;
    w_copy_data(w, p, done, ist);
    e = w_tag(w, COPY, iend - ist);
    if (e) return e;
    e = w_offset(w, i - st, iend - ist);
    if (e) return e;
    w_copy_data(w, p, ist, iend);
    *nextdone = iend; *iend_out = iend;
    return OR_OK;
}

/* Writer.flush writer.go:387-401 (the sink is an in-memory Buf, optionally faulty) */
static int w_flush(or_writer *w) {
    int64_t n = w->b.len;
    int err = OR_OK;
    if (w->sink_accept >= 0) {
        if (n > w->sink_accept) n = w->sink_accept;
        err = OR_ESINK;
        w->sink_accept = -1;
    }
    ob_put(&w->sink, w->b.p, n);
    w->sink_writes++;
    w->written += n;
    if (err != OR_OK || n != w->b.len) w_reset(w);
    if (err != OR_OK) return err;
    w->b.len = 0;
    return OR_OK;
}

/* Writer.write writer.go:379-385 */
static int w_write_out(or_writer *w) {
    if (w->flush_threshold < 0 || w->b.len < w->flush_threshold) return OR_OK;
    return w_flush(w);
}

/* Writer.Write writer.go:206-337 */
int or_writer_write(or_writer *w, const uint8_t *p, int64_t n, int64_t *done_out) {
    int e;
    int64_t done = 0;
    if (w_isreset(w)) w_append_header(w);
    int64_t start = w->pos;
    for (int64_t i = 0; i + 4 <= n;) {
        uint32_t h = w_hash(w, p, i);
        int64_t pos = (int64_t)w->ht[h];
        w->ht[h] = (uint32_t)(start + i);
        int64_t off = pos - w->pos; /* forward offset */
        if (-off > w->bs) { i++; continue; }
        if (off >= 0 && i > done + off) { /* runlen encoding */
            e = w_write_runlen(w, p, n, done, done + off, i, &done, &i);
            if (e) return e;
            continue;
        }
        /* extend backward */
        int64_t ist = i - 1, st = pos - 1;
        while (ist >= done && p[ist] == w->block[st & w->mask]) { ist--; st--; }
        ist++; st++;
        /* extend forward (the equal8 loop :251-254 is result-equivalent) */
        int64_t iend = i, end = pos;
        while (iend < n && p[iend] == w->block[end & w->mask]) { iend++; end++; }
        /* check overflows :280-296 */
        int64_t blit = w->pos - w->bs;
        int64_t bend = blit + (iend - done);
        int64_t diff = bend - st;
        if (diff > 0) { end -= diff; iend -= diff; }
        diff = (end - w->bs) - blit;
        if (diff > 0) { end -= diff; iend -= diff; }
        if (end - st < MIN_COPY_CHUNK) { i++; continue; }
        if (done < ist) {
            e = w_literal(w, p, done, ist);
            if (e) return e;
            w_copy_data(w, p, done, ist);
        }
        if (w->pos - st > w->bs) return OR_EINVAL; /* panic("too big offset") */
        e = w_copy(w, st, end);
        if (e) return e;
        w_copy_data(w, p, ist, iend);
        if (i + 1 + 4 <= n) {
            h = w_hash(w, p, i + 1);
            w->ht[h] = (uint32_t)(start + i + 1);
        }
        i = iend;
        done = iend;
    }
    if (done < n) {
        e = w_literal(w, p, done, n);
        if (e) return e;
        w_copy_data(w, p, done, n);
        done = n;
    }
    e = w_write_out(w);
    if (e) { if (done_out) *done_out = 0; return e; }
    if (done_out) *done_out = done;
    return OR_OK;
}

/* WriteHeader writer.go:342-350 */
int or_writer_write_header(or_writer *w) {
    if (!w_isreset(w)) return OR_OK;
    w_append_header(w);
    return w_write_out(w);
}

/* WriteBreak writer.go:358-366 */
int or_writer_write_break(or_writer *w) {
    if (w_isreset(w)) w_append_header(w);
    const uint8_t br[2] = {META, META_BREAK | META_LEN0};
    ob_put(&w->b, br, 2);
    return w_write_out(w);
}

/* Flush writer.go:371-377 */
int or_writer_flush(or_writer *w) {
    if (w->b.len == 0) return OR_OK;
    return w_flush(w);
}

/* Reset writer.go:149-152 */
void or_writer_reset(or_writer *w) { w_reset(w); }

/* ResetSize writer.go:155-159 */
int or_writer_reset_size(or_writer *w, int64_t block, int64_t htable) {
    int e = w_init(w, block, htable);
    if (e) return e;
    w_reset(w);
    return OR_OK;
}

const uint8_t *or_writer_sink(const or_writer *w, int64_t *len) { *len = w->sink.len; return w->sink.p; }
void or_writer_sink_clear(or_writer *w) { w->sink.len = 0; }
int64_t or_writer_sink_writes(const or_writer *w) { return w->sink_writes; }
int64_t or_writer_pos(const or_writer *w) { return w->pos; }
/* testing hook: the stream position (w.pos) of a writer, ring and table unchanged; lets a test
   reach positions past 2^32 (the uint32 table values of writer.go:216-217) */
void or_writer_set_pos(or_writer *w, int64_t pos) { w->pos = pos; }

/* ---------------------------------------------------------------- Reader */

struct or_reader {
    int ver; /* r.d.Ver */
    uint8_t *block;
    int64_t block_len, block_cap, mask, pos;
    int64_t block_size_limit, buffer_size;
    int require_magic, skip_unsupported_meta;
    int state; /* 0, 'l', 'c' */
    int64_t off, len;
    /* input r.b / r.i / r.boff */
    uint8_t *b;
    int64_t blen, bcap, i, boff;
    /* the underlying io.Reader (NULL-equivalent when has_src == 0) */
    int has_src, eof_with_data;
    int64_t chunk;
    obuf src;
    int64_t src_r;
    int64_t detail;
};

static void r_set_bytes(or_reader *r, const uint8_t *b, int64_t n) {
    if (n > r->bcap) { free(r->b); r->b = (uint8_t *)malloc((size_t)n); r->bcap = n; }
    if (n) memcpy(r->b, b, (size_t)n);
    r->blen = n;
}

or_reader *or_reader_new_bytes(const uint8_t *b, int64_t n) {
    or_reader *r = (or_reader *)calloc(1, sizeof(*r));
    r_set_bytes(r, b, n);
    return r;
}

or_reader *or_reader_new(int eof_with_data, int64_t chunk) {
    or_reader *r = (or_reader *)calloc(1, sizeof(*r));
    r->block_size_limit = 16 * MIB;
    r->buffer_size = 64 * 1024;
    r->has_src = 1;
    r->eof_with_data = eof_with_data;
    r->chunk = chunk;
    return r;
}

void or_reader_free(or_reader *r) {
    if (!r) return;
    free(r->block); free(r->b); free(r->src.p); free(r);
}

void or_reader_src_append(or_reader *r, const uint8_t *b, int64_t n) { ob_put(&r->src, b, n); }

void or_reader_set(or_reader *r, int64_t lim, int64_t bufsz, int req, int skip) {
    r->block_size_limit = lim;
    r->buffer_size = bufsz;
    r->require_magic = req;
    r->skip_unsupported_meta = skip;
}

int64_t or_reader_detail(const or_reader *r) { return r->detail; }

/* ResetBytes reader.go:102-113 */
void or_reader_reset_bytes(or_reader *r, const uint8_t *b, int64_t n) {
    r->has_src = 0;
    r_set_bytes(r, b, n);
    r->block_len = 0;
    r->pos = 0;
    r->i = 0;
    r->boff = 0;
    r->state = 0;
}

/* Reset reader.go:96-99 */
void or_reader_reset(or_reader *r, int eof_with_data, int64_t chunk) {
    or_reader_reset_bytes(r, r->b, 0);
    r->has_src = 1;
    r->eof_with_data = eof_with_data;
    r->chunk = chunk;
    r->src.len = 0;
    r->src_r = 0;
}

/* the in-memory io.Reader */
static int src_read(or_reader *r, uint8_t *p, int64_t n, int64_t *got) {
    int64_t avail = r->src.len - r->src_r;
    int64_t k = n < avail ? n : avail;
    if (r->chunk > 0 && k > r->chunk) k = r->chunk;
    if (k) memcpy(p, r->src.p + r->src_r, (size_t)k);
    r->src_r += k;
    *got = k;
    if (r->eof_with_data) return r->src_r == r->src.len ? OR_EOF : OR_OK; /* BufReader :1512-1521 */
    return (k == 0 && n > 0) ? OR_EOF : OR_OK;                             /* bytes.Buffer */
}

/* Reader.reset reader.go:327-344 */
static void r_reset(or_reader *r, int64_t bs) {
    bs = (int64_t)1 << bs;
    if (bs > r->block_cap) {
        free(r->block);
        r->block = (uint8_t *)calloc((size_t)bs, 1);
        r->block_cap = bs;
    } else {
        memset(r->block, 0, (size_t)bs);
    }
    r->block_len = bs;
    r->pos = 0;
    r->mask = bs - 1;
    r->state = 0;
}

/* continueMetaTag reader.go:272-325 */
static int r_continue_meta(or_reader *r, int64_t st, int64_t *i_out) {
    int64_t i = st;
    st--;
    int64_t meta, l;
    int err = or_dec_meta(r->b, r->blen, i, &meta, &l, &i);
    if (err) { *i_out = i; return err; } /* named-result `return`: i is Meta's st */
    if (r->boff == 0 && st == 0 && meta != META_MAGIC && r->require_magic) { *i_out = st; return OR_ENOMAGIC; }
    if (i + l > r->blen) { *i_out = st; return OR_ESHORTBUF; }
    static const int64_t tag_len[4] = {4, 1, 1, 0};
    int64_t j = meta >> 3;
    if (j < 4 && l != tag_len[j]) { *i_out = st; return OR_EUNSUPMETA; }
    switch (meta) {
    case META_MAGIC:
        if (memcmp(r->b + i, "eazy", 4) != 0) { *i_out = st; return OR_EBADMAGIC; }
        break;
    case META_VER:
        r->ver = r->b[i];
        if (r->ver > 0) { r->detail = r->ver; *i_out = st; return OR_EUNSUPVER; }
        break;
    case META_RESET: {
        int64_t bs = r->b[i];
        if (bs > 32 || l != 1 || (r->block_size_limit != 0 && ((int64_t)1 << bs) > r->block_size_limit)) {
            *i_out = st;
            return OR_EOVERFLOW;
        }
        r_reset(r, bs);
        break;
    }
    case META_BREAK:
        *i_out = i + l;
        return OR_EBREAK;
    default:
        if (r->skip_unsupported_meta) break;
        r->detail = meta;
        *i_out = st;
        return OR_EUNSUPMETA;
    }
    i += l;
    *i_out = i;
    return OR_OK;
}

/* readTag reader.go:218-270 */
static int r_read_tag(or_reader *r, int64_t st, int64_t *i_out) {
    int64_t i = st;
    while (i < r->blen && r->b[i] == 0) i++; /* skip zero padding */
    st = i;
    int tag;
    int64_t l;
    int err = or_dec_tag(r->b, r->blen, st, &tag, &l, &i);
    if (err) { *i_out = st; return err; }
    if (r->boff == 0 && st == 0 && r->b[st] != META && r->require_magic) { *i_out = st; return OR_ENOMAGIC; }
    if (tag == META && l == 0) return r_continue_meta(r, i, i_out);
    if (r->block_size_limit != 0 && l > r->block_size_limit) { *i_out = st; return OR_EBLOCKLIMIT; }
    if (tag == LITERAL) {
        r->state = 'l';
        r->off = 0;
    } else {
        int64_t off;
        err = or_dec_offset(r->b, r->blen, i, l, &off, &i);
        if (err) { *i_out = st; return err; }
        r->off = off;
        if (r->off > r->block_len) { *i_out = st; return OR_EOVERFLOW; }
        r->off = r->pos - r->off;
        r->state = 'c';
    }
    r->len = l;
    *i_out = i;
    return OR_OK;
}

/* Reader.read reader.go:143-216 */
static int r_read(or_reader *r, uint8_t *p, int64_t plen, int64_t st, int64_t *n_out, int64_t *i_out) {
    int64_t i = st;
    int err;
    *n_out = 0;
    while (r->state == 0) {
        err = r_read_tag(r, i, &i);
        if (err) { *i_out = i; return err; }
    }
    if (r->block_len == 0) { *i_out = st; return OR_EMISSEDMETA; }
    if (r->state == 'l' && i == r->blen) { *i_out = i; return OR_ESHORTBUF; }
    int64_t end = r->len;
    if (end > plen) end = plen;
    if (r->state == 'l') {
        int64_t avail = r->blen - i;
        if (end > avail) end = avail;
        memcpy(p, r->b + i, (size_t)end);
        i += end;
    } else if (r->off + r->len <= r->pos) {
        int64_t at = r->off & r->mask;
        int64_t avail = r->block_len - at;
        if (end > avail) end = avail;
        memcpy(p, r->block + at, (size_t)end);
        r->off += end;
    } else if (r->off == r->pos) { /* zero region */
        memset(p, 0, (size_t)end);
    } else {
        int64_t run = r->pos - r->off;
        if (run > plen) run = plen;
        for (int64_t j = 0; j < run;) {
            int64_t at = (r->off + j) & r->mask;
            int64_t k = r->block_len - at;
            if (k > run - j) k = run - j;
            memcpy(p + j, r->block + at, (size_t)k);
            j += k;
        }
        for (int64_t j = run; j < end;) {
            int64_t k = j < end - j ? j : end - j; /* copy(p[j:end], p[:j]) */
            memcpy(p + j, p, (size_t)k);
            j += k;
        }
        r->off += end;
    }
    r->len -= end;
    int64_t n = 0;
    while (n < end) {
        int64_t at = r->pos & r->mask;
        int64_t m = r->block_len - at;
        if (m > end - n) m = end - n;
        memcpy(r->block + at, p + n, (size_t)m);
        n += m;
        r->pos += m;
    }
    if (r->len == 0) r->state = 0;
    *n_out = n;
    *i_out = i;
    return OR_OK;
}

/* Reader.more reader.go:516-543 */
static int r_more(or_reader *r) {
    if (!r->has_src) return OR_EOF;
    int64_t end = r->blen - r->i;
    memmove(r->b, r->b + r->i, (size_t)end);
    r->blen = end;
    r->boff += r->i;
    r->i = 0;
    int64_t want = r->blen == 0 ? r->buffer_size : r->blen + 1024;
    if (want < r->bcap) want = r->bcap; /* r.b[:cap(r.b)] */
    if (want > r->bcap) {
        r->b = (uint8_t *)realloc(r->b, (size_t)(want ? want : 1));
        r->bcap = want;
    }
    int64_t n;
    int err = src_read(r, r->b + end, r->bcap - end, &n);
    r->blen = end + n;
    if (n != 0 && err == OR_EOF) err = OR_OK;
    return err;
}

/* Reader.Read reader.go:116-141 */
int or_reader_read(or_reader *r, uint8_t *p, int64_t plen, int64_t *got) {
    int64_t n = 0, m, i;
    int err = OR_OK;
    while (n < plen && err == OR_OK) {
        err = r_read(r, p + n, plen - n, r->i, &m, &i);
        n += m;
        r->i = i;
        if (n == plen) break;
        if (err != OR_ESHORTBUF) continue;
        err = r_more(r);
        if (err == OR_EOF && (r->state != 0 || r->i < r->blen)) err = OR_EUNEXPECTEDEOF;
    }
    *got = n;
    return err;
}

/* ---------------------------------------------------------------- helpers */

int or_compress(int64_t block, int64_t htable, int append_magic, int ver, const uint8_t *data,
                const int64_t *lens, int k, uint8_t *out, int64_t cap, int64_t *out_len) {
    or_writer *w = or_writer_new(block, htable);
    if (!w) return OR_EINVAL;
    w->append_magic = append_magic;
    w->ver = ver;
    int64_t at = 0;
    for (int j = 0; j < k; j++) {
        int e = or_writer_write(w, data + at, lens[j], NULL);
        if (e) { or_writer_free(w); return e; }
        at += lens[j];
    }
    int64_t n;
    const uint8_t *s = or_writer_sink(w, &n);
    *out_len = n;
    if (n > cap) { or_writer_free(w); return OR_ESHORTBUF; }
    memcpy(out, s, (size_t)n);
    or_writer_free(w);
    return OR_OK;
}

int or_decompress(const uint8_t *in, int64_t n, int64_t buf_size, uint8_t *out, int64_t cap,
                  int64_t *out_len, int64_t *breaks) {
    or_reader *r = or_reader_new_bytes(in, n);
    uint8_t *buf = (uint8_t *)malloc((size_t)(buf_size > 0 ? buf_size : 1));
    int64_t total = 0, nb = 0;
    int err;
    for (;;) {
        int64_t got;
        err = or_reader_read(r, buf, buf_size, &got);
        if (total + got > cap) { err = OR_ESHORTBUF; break; }
        memcpy(out + total, buf, (size_t)got);
        total += got;
        if (err == OR_EBREAK) { nb++; continue; }
        if (err == OR_EOF) { err = OR_OK; break; }
        if (err) break;
    }
    free(buf);
    or_reader_free(r);
    *out_len = total;
    if (breaks) *breaks = nb;
    return err;
}

typedef struct {
    int kind;
    int64_t block, htable;
    const uint8_t *in;
    const int64_t *in_off, *in_sizes;
    int64_t count, next, grain;
    uint8_t *out;
    const int64_t *out_off;
    int64_t *sizes;
    int err;
    pthread_mutex_t mu;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    or_writer *w = NULL;
    if (j->kind == 0) w = or_writer_new(j->block, j->htable);
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int64_t s0 = j->next;
        j->next += j->grain;
        pthread_mutex_unlock(&j->mu);
        if (s0 >= j->count) break;
        int64_t s1 = s0 + j->grain < j->count ? s0 + j->grain : j->count;
        for (int64_t s = s0; s < s1; s++) {
            int e;
            if (j->kind == 0) {
                /* a fresh NewWriter per stream, exactly as Writer.Reset does */
                w_reset(w);
                int64_t n = j->in_off[s + 1] - j->in_off[s];
                e = or_writer_write(w, j->in + j->in_off[s], n, NULL);
                int64_t len;
                const uint8_t *src = or_writer_sink(w, &len);
                if (!e && len > j->out_off[s + 1] - j->out_off[s]) e = OR_ESHORTBUF;
                if (!e) memcpy(j->out + j->out_off[s], src, (size_t)len);
                j->sizes[s] = len;
                or_writer_sink_clear(w);
            } else {
                int64_t got;
                e = or_decompress(j->in + j->in_off[s], j->in_sizes[s], 1 << 16, j->out + j->out_off[s],
                                  j->out_off[s + 1] - j->out_off[s], &got, NULL);
                j->sizes[s] = got;
            }
            if (e) j->err = e;
        }
    }
    or_writer_free(w);
    return NULL;
}

/* streams handed out in grains of at most 64, and small enough that every
   thread gets work (a batch of 64 long streams spreads over all threads) */
int64_t or_batch_grain(int64_t count, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    int64_t g = count / ((int64_t)nthreads * 4);
    if (g > 64) g = 64;
    if (g < 1) g = 1;
    return g;
}

static int run_batch(batch_job *j, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    j->grain = or_batch_grain(j->count, nthreads);
    pthread_mutex_init(&j->mu, NULL);
    pthread_t *t = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int k = 0; k < nthreads; k++) pthread_create(&t[k], NULL, batch_worker, j);
    for (int k = 0; k < nthreads; k++) pthread_join(t[k], NULL);
    free(t);
    pthread_mutex_destroy(&j->mu);
    return j->err;
}

int or_compress_batch(int64_t block, int64_t htable, const uint8_t *in, const int64_t *in_off,
                      int64_t count, uint8_t *slots, const int64_t *slot_off, int64_t *sizes,
                      int nthreads) {
    batch_job j;
    memset(&j, 0, sizeof(j));
    j.kind = 0; j.block = block; j.htable = htable; j.in = in; j.in_off = in_off; j.count = count;
    j.out = slots; j.out_off = slot_off; j.sizes = sizes;
    return run_batch(&j, nthreads);
}

int or_decompress_batch(const uint8_t *in, const int64_t *in_off, const int64_t *in_sizes,
                        int64_t count, uint8_t *out, const int64_t *out_off, int64_t *out_sizes,
                        int nthreads) {
    batch_job j;
    memset(&j, 0, sizeof(j));
    j.kind = 1; j.in = in; j.in_off = in_off; j.in_sizes = in_sizes; j.count = count;
    j.out = out; j.out_off = out_off; j.sizes = out_sizes;
    return run_batch(&j, nthreads);
}
