// ez_internal.h — launch interface between the C-ABI (ez_capi.hip) and the
// gfx950 kernels (ez_compress.hip, ez_decompress.hip, ez_pack.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ez {

// Timing / A-B switches.  Only experiment builds (make exp: -DEZ_KNOBS) read them from the
// environment; the product library reads no environment and runs the defaults (kernel choices for
// tests go through ez_select_compress_kernel / ez_select_decompress_kernel).
#ifdef EZ_KNOBS
const char *knob_str(const char *name);
int knob(const char *name, int dflt);
#else
inline const char *knob_str(const char *) { return nullptr; }
inline int knob(const char *, int dflt) { return dflt; }
#endif

// K1x per-stream state (ez_compress_spec.hip): speculation restarts at `from`, the pending literal
// starts at `done`, the stream's output so far is `op` bytes; flags: 0 active, 1 finished
struct SpecState {
    uint32_t from, done, op, flags;
};
// K2w: a long literal kd_copy moves after the decoders (len bytes from in[src] to out[dst])
struct DeferLit {
    uint64_t src, dst, len;
};
constexpr int kDefSlots = 8;  // deferred literals per stream at most
// a literal whose bytes K1x copies at the end (kx_copy): len bytes from in[src] to out[dst]
struct SpecLit {
    uint64_t src, dst, len;
};

// One K1 launch: `count` independent streams (batch) or one stream of a
// writer handle (ring != nullptr, ht_global persistent).
struct CompressArgs {
    const uint8_t *in;
    const uint64_t *in_off;   // count+1
    uint8_t *out;
    const uint64_t *out_off;  // count+1 (slot capacities)
    uint64_t *out_size;       // count
    int32_t *status;          // count or nullptr
    uint64_t count;
    int64_t bs;               // block (window) size, power of two
    int64_t hs;               // hash-table entries, power of two
    int append_magic;
    int ver;
    int header;               // emit the stream header first (isreset)
    // writer-handle mode
    int64_t start;            // stream position of in[0] (w.pos at Write entry)
    uint8_t *ring;            // the handle's ring (block), updated in place; nullptr = fresh stream
    uint32_t *ht_global;      // persistent hash table (handle) / per-block scratch (large hs)
    uint64_t max_len;         // max stream length (0 = unknown)
    // batch of multi-Write streams (nullptr = one Write per stream): stream s receives
    // the Writes k = write_idx[s] .. write_idx[s+1]-1, Write k ending at in[write_end[k]]
    const uint64_t *write_idx;
    const uint64_t *write_end;
    uint64_t max_writes;      // the most Writes of one stream (records reserved for their ends)
    uint64_t *write_out;      // general kernel: the output size after each Write (nullptr: not recorded)
    // K1x rounds (ez_compress_spec.hip): the general kernel resumes a stream from K1x's state
    //   spec_mode 1: at spec_first[s] (streams with ~0u there are skipped), with the table
    //                spec_tab[s]; stops after the first accepted copy and stores its state back;
    //                its literals' bytes are left to kx_copy (a record in spec_lit each)
    //   spec_mode 2: at spec[s].from, to the end of the stream
    // streams whose spec[s].flags != 0 are finished and skipped
    int spec_mode;
    SpecState *spec;
    const uint32_t *spec_first;
    uint32_t *spec_tab;
    SpecLit *spec_lit;
    uint32_t *spec_nlit;
    uint32_t win_bytes;       // general kernel, long streams: LDS window bytes (set by its launcher)
    int no_k1c;               // K1c's workspace could not be had: K1L alone (set by the C-ABI's retry)
    // a Writer handle's Write on K1L's LDS path: when set, the kernel's last act is storing done_seq
    // there (pinned host memory, system scope) so that the caller can wait by polling it
    uint32_t *done_flag;
    uint32_t done_seq;
};


// One K2 launch.  Batch: count complete streams from fresh Readers.
// Handle: count == 1 with the streaming state in `st`.
struct DecodeState {
    int64_t bs;       // len(r.block) (0 = no MetaReset seen yet)
    int64_t pos;      // r.pos
    int64_t off;      // r.off (absolute)
    int64_t len;      // r.len
    int32_t state;    // 0, 'l', 'c'
    int32_t ver;      // r.d.Ver
    int64_t i;        // r.i (in / out)
    int64_t n;        // bytes produced (out)
    int64_t detail;   // meta id / version of the last error
    int64_t hist;     // bytes of the current block held before out (handle mode)
    int32_t err;      // result code
    int32_t pad;
};

struct DecompressArgs {
    const uint8_t *in;
    const uint64_t *in_off;   // count+1
    uint8_t *out;
    const uint64_t *out_off;  // count+1 (capacities)
    uint64_t *out_size;       // count
    int32_t *status;          // count or nullptr
    uint64_t count;
    int64_t block_size_limit;
    int require_magic;
    int skip_unsupported_meta;
    int handle;               // 1 = single streaming call (Reader.Read loop without refill)
    int64_t boff;             // handle: absolute offset of in[0]
    DecodeState *st;          // handle: state in/out
    uint32_t *slow;           // batch: [0] = count, [1..] = streams the fast path handed over (nullptr = exact path only)
    uint32_t *defer;          // K2w: [0] = count, records (DeferLit) from word 4: long literals kd_copy moves
    uint64_t defer_cap;       // records reserved
    uint64_t max_out;         // batch: host hint, largest output slot (0 = unknown)
    const uint32_t *todo;     // batch: [0] = count, [1..] = the streams to decode (nullptr = all)
    // one-stream batches (count == 1, a Reader handle's whole-stream decode), optional, K2t and the exact
    // decoder: breaks[0] counts the Break metas the decoders skip (reader.go:306-307) and breaks[1 ..
    // breaks_cap] get their output positions (unordered); end_state gets {len(r.block), r.pos} at the end
    // of the stream (the Reader's state after the last token, for a Read-by-Read continuation)
    uint64_t *breaks;
    uint64_t breaks_cap;
    int64_t *end_state;
    // K2j's workspace, optional (jump_workspace_bytes): a synchronous caller (a Reader handle) passes
    // one it owns; without it the launcher keeps one per (device, HIP stream)
    void *jws;
    uint64_t jws_cap;
    int force;                // batch: the first K2 kernel ('r', 't', ...; 0 = the automatic / selected one)
    // batch: host hints, in_off[count] - in_off[0] and out_off[count] - out_off[0] (0 = unknown: the
    // K2j route and its workspace then read the offsets back, which waits for the stream)
    uint64_t in_bytes, out_bytes;
    // K2j, one stream (count == 1) continuing a Reader's stream (ez_reader_read's read-ahead, c_on):
    // the input is what the Reader has buffered, so it may end inside a token (the chain stops before
    // it); c_bsl: the window's log2 at the input's start (-1: none yet); c_hist: bytes of the window's
    // history right before out + out_off[0] (the last min(r.pos, len(r.block)) decoded bytes);
    // c_pos0: r.pos there (a MetaReset then hands the stream over unless c_pos0 and the output before
    // it are 0).  end_state then gets {window bytes, output bytes, input consumed by whole tokens, and
    // for a literal starting there whose body runs past the input its header length and length}
    int c_on;
    int32_t c_bsl;
    uint64_t c_hist;
    int64_t c_pos0;
};

// words of workspace the two-level batch decoder needs
uint64_t decompress_workspace_words(uint64_t count);

hipError_t launch_compress(const CompressArgs &a, hipStream_t s);
// K1s: fresh streams, parse kernel + token-writer kernel (ez_compress_split.hip);
// scratch = 16-byte match records, split_scratch_words u32 words
uint32_t split_stride_words(const CompressArgs &a);
uint64_t split_scratch_words(const CompressArgs &a);
void select_split_table(bool t32);  // force the u32 exchange table (tests, A/B)
hipError_t launch_compress_split(const CompressArgs &a, uint32_t *scratch, hipStream_t s);
// the K1 kernel a batch launch takes: 's' K1s (parse + token writer), 'w' general wave per stream
char compress_variant(const CompressArgs &a);
void select_compress_variant(int v);  // 0 = automatic, else a variant letter (tests, A/B)
// K1L: the lean parse for long fresh streams (ez_compress_split.hip); resumes K1x's streams (spec_mode 2)
bool long_applies(const CompressArgs &a);
uint64_t long_scratch_bytes(const CompressArgs &a);
hipError_t launch_long(const CompressArgs &a, uint8_t *recs, hipStream_t s);
// K1L on a Writer handle's single Write (the handle's ring as history, its table in and out)
bool long_ring_applies(const CompressArgs &a);
// Writes up to this many bytes K1L stages in LDS (the input read once): the handle path then lets the
// kernels read the Write from, and write the output to, pinned host memory (no copies)
constexpr uint64_t kHandleLdsWrite = 49152;
uint64_t long_ring_scratch_bytes(const CompressArgs &a);
hipError_t launch_long_ring(const CompressArgs &a, uint8_t *recs, hipStream_t s);
bool compress_forced_general();  // ez_select_compress_kernel('w') (tests, A/B)
bool compress_forced_long();     // ez_select_compress_kernel('l'): K1L alone, without K1c (tests, A/B)
// K1c (chunk-parallel K1L, ez_compress_split.hip): counting of its verdicts (ez_compress_k1c_stats)
bool chunk_applies(const CompressArgs &a);
void k1c_stats(int enable, uint64_t *out);
// K1x: the data-parallel first pass for long fresh single-Write streams (ez_compress_spec.hip)
bool spec_applies(const CompressArgs &a, bool any_len = false);  // any_len: also below 64 KiB (forced)
uint64_t spec_scratch_bytes(const CompressArgs &a);
hipError_t launch_compress_spec(const CompressArgs &a, uint8_t *scratch, hipStream_t s);
// the general kernel for one launch (ez_compress.hip); K1x calls it in its resume modes
hipError_t launch_general(const CompressArgs &a, hipStream_t s);
// u32 words of global hash-table scratch a batch launch needs (hs too big for LDS)
uint64_t compress_scratch_words(const CompressArgs &a);
hipError_t launch_decompress(const DecompressArgs &a, hipStream_t s);
void select_decompress_variant(int v);
int last_decompress_variant();  // the first K2 kernel of the last batch decode
// K2r: one lane per stream with a 512-byte LDS ring of recent output (ez_decompress_ring.hip)
hipError_t launch_decompress_ring(const DecompressArgs &a, hipStream_t s);
hipError_t launch_decompress_wave(const DecompressArgs &a, hipStream_t s);  // K2w, long streams
hipError_t launch_defer_copy(const DecompressArgs &a, hipStream_t s);       // K2w's deferred literals
// K2j (ez_decompress_jump.hip): batches of at most 1,024 streams, chip-wide token starts, token
// records and pointer jumping over the copied bytes; streams it cannot take go to slow
bool jump_applies(const DecompressArgs &a);
uint64_t jump_workspace_bytes(uint64_t count, uint64_t in_total, uint64_t out_total);
// (hipErrorOutOfMemory: its workspace could not be had, nothing was launched)
hipError_t launch_decompress_jump(const DecompressArgs &a, hipStream_t s);
class DevCache;
DevCache &jump_cache();  // K2j's workspaces per (device, HIP stream)
// in_off[count] - in_off[0], out_off[count] - out_off[0]: the caller's hints, else read back (waits)
hipError_t batch_extents(const DecompressArgs &a, hipStream_t s, uint64_t *in_bytes, uint64_t *out_bytes);
hipError_t launch_decompress_tok(const DecompressArgs &a, hipStream_t s);   // K2t, token-parallel wave per stream
bool lds_exchange_in_lane_order();  // the LDS property K1s-T32 relies on (checked once)
bool lds_mskor_in_lane_order();     // the LDS property k1_lean's one-atomic visit relies on (checked once)
bool lds_mskor64_in_lane_order();   // the same on 12-bit fields of 64-bit words (k1_lean<12>)
hipError_t launch_pack(const uint8_t *slots, const uint64_t *slot_off, const uint64_t *sizes, uint64_t count,
                       uint8_t *packed, uint64_t *packed_off, void *workspace, hipStream_t s);
size_t pack_workspace(uint64_t count);

}  // namespace ez
