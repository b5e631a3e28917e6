/*
 * eazy.h — C-ABI of the MI355X-native eazy codec (libeazy_amd.so).
 *
 * This is the drop-in boundary a cgo shim binds (see INTEGRATION.md for the
 * Go side).  Plain pointers and sizes only.  Every entry point names the
 * reference (tlog-dev/eazy, Go) interface it replaces.
 *
 * Compute runs on AMD Instinct MI355X (gfx950) HIP kernels; there is no CPU
 * fallback: without a usable GPU every compute entry point returns
 * EZ_EDEVICE.  Only the scalar token codec (ez_encode_* / ez_decode_*) and
 * ez_compress_bound are host functions; they are the reference's exported
 * Encoder/Decoder value types, not the hot path.
 */
#ifndef EAZY_AMD_H
#define EAZY_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EZ_ABI_VERSION 2

/* ---- status codes: one per reference error value (reader.go:57-76) ---- */
enum {
    EZ_OK = 0,
    EZ_EOF = 1,            /* io.EOF */
    EZ_ESHORTBUF = 2,      /* ErrShortBuffer = io.ErrShortBuffer (reader.go:62) */
    EZ_EUNEXPECTEDEOF = 3, /* io.ErrUnexpectedEOF (reader.go:135-136) */
    EZ_EOVERFLOW = 4,      /* ErrOverflow (reader.go:61) */
    EZ_EBADMAGIC = 5,      /* ErrBadMagic (reader.go:58) */
    EZ_ENOMAGIC = 6,       /* ErrNoMagic (reader.go:60) */
    EZ_EBLOCKLIMIT = 7,    /* ErrBlockSizeOverLimit (reader.go:59) */
    EZ_EUNSUPMETA = 8,     /* ErrUnsupportedMeta (reader.go:63, 319) */
    EZ_EUNSUPVER = 9,      /* ErrUnsupportedVersion (reader.go:64, 303) */
    EZ_EBREAK = 10,        /* ErrBreak (reader.go:75) */
    EZ_EMISSEDMETA = 11,   /* errors.New("missed meta") (reader.go:155) */
    EZ_EINVAL = 12,        /* a reference panic: bad sizes (writer.go:162-168),
                              too big length/offset (:308-310, 562, 596), bad meta (:600-602) */
    EZ_ESINK = 13,         /* reserved for host shims: underlying io.Writer failed */
    EZ_ENOSPC = 14,        /* caller output buffer too small (C-ABI only) */
    EZ_EDEVICE = 15,       /* no usable MI355X / HIP runtime error */
    EZ_ESTUCK = 16         /* internal: a kernel's progress guard tripped */
};

/* ---- wire-format constants (writer.go:49-122) ---- */
#define EZ_LITERAL 0x00
#define EZ_COPY 0x80
#define EZ_META 0x80
#define EZ_LEN1 124
#define EZ_LEN2 125
#define EZ_LEN4 126
#define EZ_LEN_ALT 127
#define EZ_OFF1 252
#define EZ_OFF2 253
#define EZ_OFF4 254
#define EZ_OFF_LONG 255
#define EZ_META_MAGIC 0x00
#define EZ_META_VER 0x08
#define EZ_META_RESET 0x10
#define EZ_META_BREAK 0x18
#define EZ_META_LEN_WIDE 6
#define EZ_META_LEN0 7
#define EZ_VERSION 0

const char *ez_strerror(int code);

/* ---- which reference panic an EZ_EINVAL stands for, so a shim re-panics with Go's value ----
 * ez_encode_tag: always EZ_PANIC_LENGTH (writer.go:562); ez_encode_offset: EZ_PANIC_OFFSET
 * (:596); ez_encode_meta: EZ_PANIC_META when meta & ~0xf8 (:600-602, Go panics with the meta
 * int), else EZ_PANIC_OFFSET (its wide length goes through Offset); a Writer handle:
 * ez_writer_last_panic; NewWriter / ResetSize: ez_writer_size_panic. */
enum {
    EZ_PANIC_NONE = 0,
    EZ_PANIC_BLOCK = 1,  /* "block size must be a power of two (32 < bs < 1<<31)" writer.go:163 */
    EZ_PANIC_HTABLE = 2, /* "hash table size must be a power of two (hs >= 4)"    writer.go:167 */
    EZ_PANIC_LENGTH = 3, /* "too big length"                                       writer.go:562 */
    EZ_PANIC_OFFSET = 4, /* "too big offset"                                       writer.go:309, 596 */
    EZ_PANIC_META = 5    /* panic(meta)                                            writer.go:601 */
};
const char *ez_panic_message(int panic);
int ez_writer_size_panic(int64_t block, int64_t htable); /* Writer.init writer.go:161-169; 0 = valid */
int ez_abi_version(void);
/* Number of visible HIP devices (0 when none). */
int ez_device_count(void);

/* ---- low-level token codec: Encoder (writer.go:537-621), Decoder (reader.go:346-514) ----
 * Encoders append at b[*len] (cap = total capacity of b); EZ_EINVAL where Go panics.
 * Decoders mirror Go's (…, i, err) results: *i is `st` on any error. */
int ez_encode_tag(uint8_t *b, size_t cap, size_t *len, int tag, int64_t l);       /* Encoder.Tag    writer.go:537 */
int ez_encode_offset(uint8_t *b, size_t cap, size_t *len, int64_t off, int64_t l); /* Encoder.Offset writer.go:565 */
int ez_encode_meta(uint8_t *b, size_t cap, size_t *len, int64_t meta, int64_t l);  /* Encoder.Meta   writer.go:599 */
int ez_decode_tag(const uint8_t *b, size_t n, size_t st, int *tag, int64_t *l, size_t *i);       /* Decoder.Tag    reader.go:346 */
int ez_decode_offset(const uint8_t *b, size_t n, size_t st, int64_t l, int64_t *off, size_t *i); /* Decoder.Offset reader.go:394 */
int ez_decode_meta(const uint8_t *b, size_t n, size_t st, int64_t *meta, int64_t *l, size_t *i); /* Decoder.Meta   reader.go:474 */

/* Upper bound of the bytes one Write of n bytes can append (header included).
 * Derived (not in the reference); proved in tests/test_bound.py. */
size_t ez_compress_bound(size_t n);

/* ---- streaming Writer handle: the state of writer.go Writer (:17-46) ----
 * The ring (block), hash table and stream position live in HBM on `device`.
 * The io.Writer sink, the output buffer b, FlushThreshold and `written` stay
 * in the host shim (writer.go:379-401); the handle tracks isreset()
 * (writer.go:403) as "nothing emitted since the last reset". */
typedef struct ez_writer ez_writer;
int ez_writer_new(int64_t block, int64_t htable, int device, ez_writer **out); /* NewWriter writer.go:133 */
void ez_writer_free(ez_writer *w);
int ez_writer_set_append_magic(ez_writer *w, int on); /* Writer.AppendMagic writer.go:25 */
int ez_writer_set_version(ez_writer *w, int ver);     /* Writer.e.Ver writer.go:21 */
/* Writer.Write(p) writer.go:206-337: compresses p on the GPU and returns in
 * out[0..*out_n) exactly the bytes Go appends to w.b for this call (header
 * included on a pristine stream).  cap >= ez_compress_bound(n). */
int ez_writer_write(ez_writer *w, const uint8_t *p, size_t n, uint8_t *out, size_t cap, size_t *out_n);
/* k Writes on the handle in one device call, the same as k ez_writer_write calls in
 * turn: p holds the Writes back to back, Write j ending at p[ends[j]] (ends
 * non-decreasing); out receives their bytes back to back, Write j's ending at
 * out[out_ends[j]].  cap >= the sum of ez_compress_bound(len of Write j).  The
 * mirrors replay FlushThreshold per Write from out_ends, so a caller batching small
 * Writes sees the reference's sink calls (writer.go:379-401).  Errors as
 * ez_writer_write (the stream restarts). */
int ez_writer_write_batch(ez_writer *w, const uint8_t *p, const uint64_t *ends, size_t k, uint8_t *out, size_t cap,
                          uint64_t *out_ends);
int ez_writer_header(ez_writer *w, uint8_t *out, size_t cap, size_t *out_n); /* WriteHeader writer.go:342 */
int ez_writer_break(ez_writer *w, uint8_t *out, size_t cap, size_t *out_n);  /* WriteBreak  writer.go:358 */
int ez_writer_reset(ez_writer *w);                                          /* Reset       writer.go:149 (reset :187) */
int ez_writer_reset_size(ez_writer *w, int64_t block, int64_t htable);     /* ResetSize   writer.go:155 */
int ez_writer_is_reset(const ez_writer *w);                                 /* isreset     writer.go:403 */
int ez_writer_last_panic(const ez_writer *w); /* EZ_PANIC_* behind the handle's last EZ_EINVAL */
/* Testing hook (no reference counterpart): set w.pos, ring and table unchanged, so a test can
 * run Writes across stream position 2^32, where the table's uint32 values (writer.go:216-217)
 * stop matching; the C oracle has the same hook. */
int ez_writer_set_position(ez_writer *w, int64_t pos);

/* ---- streaming Reader handle: the decoder state of reader.go Reader (:17-40) ----
 * Window, position and current token live on the device.  The host shim owns
 * r.b / r.i / r.boff and the refill from io.Reader (more(), reader.go:516-543). */
typedef struct ez_reader ez_reader;
int ez_reader_new(int device, ez_reader **out); /* NewReader / NewReaderBytes reader.go:79, 89 */
void ez_reader_free(ez_reader *r);
/* Reader.BlockSizeLimit, RequireMagic, SkipUnsupportedMeta (reader.go:27-30) */
int ez_reader_configure(ez_reader *r, int64_t block_size_limit, int require_magic, int skip_unsupported_meta);
int ez_reader_reset(ez_reader *r); /* the decoder part of ResetBytes reader.go:102-113 */
/* The inner loop of Reader.Read (reader.go:119-133) without the refill:
 * decodes from b[i..b_len) (boff = absolute offset of b[0]) into p until p is
 * full (EZ_OK), the input runs short (EZ_ESHORTBUF: caller refills and calls
 * again), or another error.  *n = bytes produced, *i_out = new r.i,
 * *detail = meta id / version for EZ_EUNSUPMETA / EZ_EUNSUPVER. */
int ez_reader_read(ez_reader *r, const uint8_t *b, size_t b_len, size_t i, int64_t boff, uint8_t *p,
                   size_t p_len, size_t *n, size_t *i_out, int64_t *detail);
int ez_reader_pending(const ez_reader *r); /* r.state != 0 (reader.go:135) */
/* The b of this handle's Reads is the whole stream (NewReaderBytes / ResetBytes with no
 * io.Reader behind it; no reference counterpart): the first Read of a fresh stream then decodes
 * all of it at once on the device and the Reads are served from that output -- the same bytes,
 * ErrBreak / errors / EOF at the same Reads (streams with a Break meta, an error, RequireMagic
 * or SkipUnsupportedMeta keep the Read-by-Read decode). 0 (default): b may grow (NewReader). */
int ez_reader_set_whole(ez_reader *r, int whole);
/* 1 when this stream's Reads are being served from the whole-stream decode (tests, measurement). */
int ez_reader_whole_decoded(const ez_reader *r);
/* NewReader(io.Reader) handles (set_whole 0) read ahead: a Read with nothing decoded ahead and at
 * least 8 KiB of buffered input b[i..b_len) decodes every whole token of it at once on the device
 * (K2j continuing the stream from the handle's state, a literal the buffer ends inside of decoded as
 * far as it goes), and the Reads are served from that output -- the same bytes, ErrBreak and errors at
 * the same Reads as Read by Read, and ErrShortBuffer (the shim's refill, more()) with *i_out where
 * Read by Read would ask for more input.  A buffer the device path hands over (an error, a MetaReset
 * after output, ...) is decoded Read by Read until more input arrives.  The number of read-aheads
 * this handle has made (tests, measurement): */
int64_t ez_reader_ahead_count(const ez_reader *r);

/* ---- device-resident batches of independent streams (the GPU hot path) ----
 * One stream = a fresh NewWriter(block, htable) receiving one Write; its
 * bytes equal Go's `NewWriter(&buf, block, htable).Write(p)` output.
 * All pointers below are DEVICE pointers on the current HIP device; calls
 * are asynchronous on `hip_stream` (a hipStream_t, NULL = default stream). */
typedef struct {
    const uint8_t *in;       /* concatenated inputs */
    const uint64_t *in_off;  /* count+1 offsets into in */
    uint8_t *out;            /* output slots */
    const uint64_t *out_off; /* count+1 offsets: slot s = out[out_off[s] .. out_off[s+1]) */
    uint64_t *out_size;      /* count: bytes written into each slot */
    int32_t *status;         /* count: EZ_* per stream (may be NULL) */
    uint64_t count;
    uint64_t max_len;        /* host hint: max input length of a stream (decompress: max slot; 0 = unknown) */
    /* decompress, host hints (ABI 2): in_off[count] - in_off[0] and out_off[count] - out_off[0],
     * both 0 = unknown.  With them the decoder route and its workspace need no read-back of the
     * offsets, so the call never waits for the stream; compress ignores them. */
    uint64_t in_bytes;
    uint64_t out_bytes;
} ez_batch;

#define EZ_F_NO_MAGIC 0x1 /* compress: AppendMagic = false */

/* K1: compress every stream of b into its slot (slot >= ez_compress_bound(n)). */
int ez_compress_batch(int64_t block, int64_t htable, int flags, const ez_batch *b, void *hip_stream);
/* K1 for streams that each receive several Writes (Writer.Write writer.go:206
 * called k times on one NewWriter, FlushThreshold 0: the slot holds what the
 * sink receives over the k calls).  Stream s receives the Writes
 * k = write_idx[s] .. write_idx[s+1]-1 (device arrays, write_idx[count+1]);
 * Write k is in[prev .. write_end[k]) with prev = in_off[s] for the first.
 * max_writes: the most Writes of one stream (host hint).  Slots need
 * ez_compress_bound(n) + 5 bytes per Write.  Streams of any length: K1s takes
 * batches with 2 x length <= block, the general kernel the others. */
int ez_compress_batch_writes(int64_t block, int64_t htable, int flags, const ez_batch *b, const uint64_t *write_idx,
                             const uint64_t *write_end, uint64_t max_writes, void *hip_stream);
/* K3: exclusive scan of sizes -> packed_off[count+1], then gather the slots
 * densely into packed.  workspace >= ez_pack_workspace(count) device bytes. */
size_t ez_pack_workspace(uint64_t count);
int ez_pack_batch(const uint8_t *slots, const uint64_t *slot_off, const uint64_t *sizes, uint64_t count,
                  uint8_t *packed, uint64_t *packed_off, void *workspace, void *hip_stream);
/* K2: decode every compressed stream b->in[in_off[s]..in_off[s+1]) completely
 * (NewReaderBytes + read to EOF; ErrBreak markers are skipped) into its slot.
 * status[s] = EZ_OK on a clean end of stream, else the first error;
 * out_size[s] = bytes produced before it (out_size is required).
 * workspace >= ez_decompress_workspace(count) device bytes enables the
 * lane-per-stream fast decoder (streams it cannot take are handed to the
 * exact wave-per-stream decoder); NULL = exact decoder only. */
size_t ez_decompress_workspace(uint64_t count);
int ez_decompress_batch(int64_t block_size_limit, const ez_batch *b, void *workspace, void *hip_stream);

/* ---- host-memory batches over several devices (SURVEY §8b device_or_all) ----
 * Streams share no state (writer.go:40-45, reader.go:17-40), so a batch splits into contiguous
 * whole-stream shards, balanced by bytes, one per entry of `devices` (ndev entries; NULL or 0 =
 * every visible device; an entry may repeat: two shards on one device, each on its own HIP
 * stream); each shard runs on its own host thread: upload, the batch kernels, download.  All
 * pointers are HOST pointers; the calls return when the output is in host memory.
 *
 * Compress: stream s = in[in_off[s] .. in_off[s+1]) as one Write to a fresh NewWriter(block,
 * htable); packed gets the streams' outputs back to back, packed_off[count+1] their offsets
 * (a host exclusive scan of the shards' packed sizes), status[count] (may be NULL) EZ_* per
 * stream.  packed_cap < packed_off[count] -> EZ_ENOSPC with packed_off filled, packed untouched
 * (sum of ez_compress_bound(n) always suffices). */
int ez_compress_batch_multi(int64_t block, int64_t htable, int flags, const uint8_t *in, const uint64_t *in_off, uint64_t count,
                            const int *devices, int ndev, uint8_t *packed, uint64_t packed_cap, uint64_t *packed_off,
                            int32_t *status);
/* Decompress: stream s = in[in_off[s] .. in_off[s+1]) read to EOF as NewReaderBytes does (Break
 * metas skipped) into out[out_off[s] .. out_off[s+1]); out_size[count] bytes produced,
 * status[count] (may be NULL) EZ_OK or the first error, as ez_decompress_batch. */
int ez_decompress_batch_multi(int64_t block_size_limit, const uint8_t *in, const uint64_t *in_off, uint64_t count,
                              const int *devices, int ndev, uint8_t *out, const uint64_t *out_off, uint64_t *out_size,
                              int32_t *status);

/* Frees the device scratch kept between batch calls (no reference counterpart; a caching
 * allocator's empty_cache): K1 / K1c scratch and K2j workspaces per (device, HIP stream), the
 * multi-device calls' pooled shard buffers, the Reader handles' shared K2j workspace; device < 0 =
 * every device.  Scratch in use by a concurrent call is kept.  Entries beyond 8 streams per device
 * are also freed least recently used first as new streams arrive. */
int ez_release_cached(int device);
/* Introspection (tests, measurement): the shards of the last ez_*_batch_multi call in this process
 * (returns their number; up to cap entries filled, any pointer may be NULL): each shard's device and
 * its device interval (upload to download) in ms from the earliest shard start on that device. */
int ez_multi_last_shards(int *dev, double *t0_ms, double *t1_ms, int cap);

/* Introspection (no reference counterpart): the K1 kernel a batch of `count`
 * fresh streams of <= max_len bytes would run on the current device, as a
 * character: 's' K1s (parse + token writer; fresh streams with 2n <= block and
 * at most 4096 table entries), 'x' K1x (data-parallel rounds over the emitting
 * positions, then the general kernel; other fresh single-Write batches of streams
 * up to 2 GiB, at least one of 64 KiB or more, at most 4096 table entries),
 * 'w' general wave per stream (everything else);
 * EZ_EDEVICE (negated) without a device. */
int ez_compress_kernel(int64_t block, int64_t htable, uint64_t max_len, uint64_t count);
/* Testing / A-B measurement (no reference counterpart): force the K1 kernel of
 * later batch calls in this process ('s' K1s, 'S' K1s with the u32
 * exchange table, 'w' general alone, 'x' K1x at any stream length, 'l' K1L alone (the lean
 * parse for long fresh streams, which otherwise continues K1x's dense streams); 0 = automatic choice).  A forced kernel that cannot take a batch falls
 * back to the automatic choice.  Not thread-safe against concurrent calls. */
int ez_select_compress_kernel(int kind);
/* Testing / A-B measurement: the first K2 kernel of later batch decodes with a
 * workspace ('r' lane-per-stream with an LDS ring of recent output, 't'
 * token-parallel wave per stream, 'w' wave per stream with a scalar token walk; 0 = automatic:
 * 't' when a slot is 64 KiB or more, else 'r'; the largest
 * slot is max_len when the caller gives it, else measured on the device, which waits for the
 * stream).  Streams the chosen kernel cannot take go on to the exact decoder. */
int ez_select_decompress_kernel(int kind);
/* Introspection: the first K2 kernel the last ez_decompress_batch call of this process ran
 * ('r', 't', 'w'; 'e' the exact decoder alone; 0 none yet). */
int ez_decompress_kernel_last(void);
/* Testing: K1c (the chunk-parallel parse of long fresh streams, which proves each stream's parse
 * is Go's or gives it to K1L) counts its verdicts while counting is on: counts (6 words, may be
 * NULL) gets {streams proven, chunk error or re-visit, no common copy end, a judgement changed,
 * record slot, path segments} so far; enable 1 clears them and turns counting on (each K1c batch
 * then waits for its verdicts), 0 turns it off. */
int ez_compress_k1c_stats(int enable, uint64_t *counts);

#ifdef __cplusplus
}
#endif
#endif /* EAZY_AMD_H */
