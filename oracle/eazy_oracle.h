/*
 * eazy_oracle.h — CPU restatement of tlog-dev/eazy (writer.go / reader.go).
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker, not the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The shipped path is include/eazy.h (libeazy_amd.so, HIP/gfx950).
 *
 * Parity pinning: the reference is pure Go and no Go toolchain exists in
 * this image, so the reference cannot be built or run here.
 * This restatement is pinned by every exact-byte known-answer test the
 * reference's eazy_test.go holds (see tests/test_oracle_kat.py), by the
 * reference's testdata/fuzz corpora, and by a second independent restatement
 * in pure Python (tests/pyoracle.py).
 *
 * Error codes are numerically identical to include/eazy.h's EZ_* codes.
 */
#ifndef EAZY_ORACLE_H
#define EAZY_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    OR_OK = 0,
    OR_EOF = 1,            /* io.EOF */
    OR_ESHORTBUF = 2,      /* ErrShortBuffer (= io.ErrShortBuffer) reader.go:62 */
    OR_EUNEXPECTEDEOF = 3, /* io.ErrUnexpectedEOF reader.go:136 */
    OR_EOVERFLOW = 4,      /* ErrOverflow reader.go:61 */
    OR_EBADMAGIC = 5,      /* ErrBadMagic reader.go:58 */
    OR_ENOMAGIC = 6,       /* ErrNoMagic reader.go:60 */
    OR_EBLOCKLIMIT = 7,    /* ErrBlockSizeOverLimit reader.go:59 */
    OR_EUNSUPMETA = 8,     /* ErrUnsupportedMeta reader.go:63 */
    OR_EUNSUPVER = 9,      /* ErrUnsupportedVersion reader.go:64 */
    OR_EBREAK = 10,        /* ErrBreak reader.go:75 */
    OR_EMISSEDMETA = 11,   /* errors.New("missed meta") reader.go:155 */
    OR_EINVAL = 12,        /* a Go panic in the reference */
    OR_ESINK = 13,         /* error from the underlying io.Writer */
};

/* ---- low level codec: Encoder (writer.go:537-621) / Decoder (reader.go:346-514) ---- */
/* Encoders append to b[*len] (b must have >= 16 spare bytes); return OR_EINVAL on panic. */
int or_enc_tag(uint8_t *b, size_t *len, int tag, int64_t l);
int or_enc_offset(uint8_t *b, size_t *len, int64_t off, int64_t l);
int or_enc_meta(uint8_t *b, size_t *len, int64_t meta, int64_t l);
/* Decoders: return error code; *i_out is the Go `i` result (st on error). */
int or_dec_tag(const uint8_t *b, int64_t n, int64_t st, int *tag, int64_t *l, int64_t *i_out);
int or_dec_offset(const uint8_t *b, int64_t n, int64_t st, int64_t l, int64_t *off, int64_t *i_out);
int or_dec_meta(const uint8_t *b, int64_t n, int64_t st, int64_t *meta, int64_t *l, int64_t *i_out);

/* ---- Writer (writer.go:17-535) writing into an in-memory sink (eazy_test.go Buf) ---- */
typedef struct or_writer or_writer;
or_writer *or_writer_new(int64_t block, int64_t htable); /* NULL on panic (bad sizes) */
void or_writer_free(or_writer *w);
void or_writer_set_append_magic(or_writer *w, int on);
void or_writer_set_version(or_writer *w, int ver);
void or_writer_set_flush_threshold(or_writer *w, int64_t t);
/* sink_accept < 0: sink takes everything; otherwise the next sink Write accepts
 * at most sink_accept bytes and returns an error (models a failing io.Writer). */
void or_writer_set_sink_fault(or_writer *w, int64_t sink_accept);
int or_writer_write(or_writer *w, const uint8_t *p, int64_t n, int64_t *done);
int or_writer_write_header(or_writer *w);
int or_writer_write_break(or_writer *w);
int or_writer_flush(or_writer *w);
void or_writer_reset(or_writer *w);
int or_writer_reset_size(or_writer *w, int64_t block, int64_t htable);
const uint8_t *or_writer_sink(const or_writer *w, int64_t *len);
void or_writer_sink_clear(or_writer *w);
int64_t or_writer_sink_writes(const or_writer *w);
int64_t or_writer_pos(const or_writer *w);
void or_writer_set_pos(or_writer *w, int64_t pos); /* testing hook */

/* ---- Reader (reader.go:17-543) ---- */
typedef struct or_reader or_reader;
/* NewReaderBytes(b) (reader.go:89): copies b. */
or_reader *or_reader_new_bytes(const uint8_t *b, int64_t n);
/* NewReader(src) (reader.go:79) over an in-memory io.Reader.  eof_with_data=1
 * models eazy_test.go BufReader (last bytes returned together with io.EOF);
 * eof_with_data=0 models bytes.Buffer.  chunk>0 caps bytes returned per Read. */
or_reader *or_reader_new(int eof_with_data, int64_t chunk);
void or_reader_free(or_reader *r);
void or_reader_src_append(or_reader *r, const uint8_t *b, int64_t n);
void or_reader_set(or_reader *r, int64_t block_size_limit, int64_t buffer_size, int require_magic,
                   int skip_unsupported_meta);
int or_reader_read(or_reader *r, uint8_t *p, int64_t n, int64_t *got);
void or_reader_reset_bytes(or_reader *r, const uint8_t *b, int64_t n);
/* Reset(rd) with a fresh in-memory source. */
void or_reader_reset(or_reader *r, int eof_with_data, int64_t chunk);
int64_t or_reader_detail(const or_reader *r); /* meta id / version attached to the last error */

/* ---- whole-stream helpers (tests and the CPU baseline) ---- */
/* A fresh NewWriter(block,htable) receiving k Writes with FlushThreshold 0;
 * returns the concatenated sink bytes. */
int or_compress(int64_t block, int64_t htable, int append_magic, int ver, const uint8_t *data,
                const int64_t *lens, int k, uint8_t *out, int64_t cap, int64_t *out_len);
/* NewReaderBytes(in) read with a buf_size buffer until EOF or error (ErrBreak is
 * skipped and counted).  Returns the final error code (OR_OK on clean EOF). */
int or_decompress(const uint8_t *in, int64_t n, int64_t buf_size, uint8_t *out, int64_t cap,
                  int64_t *out_len, int64_t *breaks);
/* Independent streams, one Write each, spread over nthreads host threads. */
/* the number of streams one batch task takes (count / (4 * threads), clamped to [1, 64]) */
int64_t or_batch_grain(int64_t count, int nthreads);
int or_compress_batch(int64_t block, int64_t htable, const uint8_t *in, const int64_t *in_off,
                      int64_t count, uint8_t *slots, const int64_t *slot_off, int64_t *sizes,
                      int nthreads);
int or_decompress_batch(const uint8_t *in, const int64_t *in_off, const int64_t *in_sizes,
                        int64_t count, uint8_t *out, const int64_t *out_off, int64_t *out_sizes,
                        int nthreads);

#ifdef __cplusplus
}
#endif
#endif
