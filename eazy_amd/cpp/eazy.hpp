// eazy.hpp — C++ host side of the MI355X eazy codec, over the C-ABI of
// include/eazy.h (libeazy_amd.so).
//
// It mirrors the reference Go package's exported surface (tlog-dev/eazy):
// the same names, argument meaning and error behaviour, so C++ callers and
// the parity tests (tests/cpp/eazy_test.cpp) read like eazy_test.go.
//
//   Go (reference)                               C++ (here)
//   NewWriter(w io.Writer, block, htable int)    eazy::NewWriter(IoWriter*, block, htable)   writer.go:133
//   (*Writer).Write(p) (int, error)              Writer::Write(p, n) -> {n, Err}             writer.go:206
//   WriteHeader / WriteBreak / Flush             Writer::WriteHeader / WriteBreak / Flush    writer.go:342-377
//   Reset(w) / ResetSize(w, block, htable)       Writer::Reset / ResetSize                   writer.go:149-159
//   Writer.AppendMagic / FlushThreshold          Writer::AppendMagic / FlushThreshold        writer.go:23-34
//   NewReader(r io.Reader) / NewReaderBytes(b)   eazy::NewReader / NewReaderBytes            reader.go:79, 89
//   (*Reader).Read(p) (int, error)               Reader::Read(p, n) -> {n, Err}              reader.go:116
//   Reset(r) / ResetBytes(b)                     Reader::Reset / ResetBytes                  reader.go:96-113
//   BlockSizeLimit, BufferSize, RequireMagic,    same public fields                          reader.go:27-30
//   SkipUnsupportedMeta
//   Encoder{Ver}.Tag/Offset/Meta                 eazy::Encoder                               writer.go:537-621
//   Decoder{Ver}.Tag/Offset/Meta                 eazy::Decoder                               reader.go:346-514
//   error values ErrOverflow, ErrBreak, ...      eazy::Err (one code per value)              reader.go:57-76
//   panics (bad sizes, impossible lengths)       eazy::Panic exception                        writer.go:162-168
//   Dumper / NewDumper(w) / Dump(p)              eazy::Dumper / NewDumper / Dump              reader.go:43-54, 545-732
//
// The compute (Writer.Write's match-find/emit, Reader.Read's decode) runs in
// the HIP kernels behind the C-ABI; with no usable GPU those calls fail with
// Err::Device (there is no CPU fallback).  The io.Writer / io.Reader plumbing,
// the output buffer, FlushThreshold and the input refill (more()) live here,
// exactly where the reference keeps them (writer.go:379-401, reader.go:516-543).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <tuple>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/eazy.h"

namespace eazy {

constexpr int64_t KiB = 1 << 10;
constexpr int64_t MiB = 1 << 20;

// Token and meta constants (writer.go:49-122)
constexpr int Literal = EZ_LITERAL, Copy = EZ_COPY, Meta = EZ_META;
constexpr int Len1 = EZ_LEN1, Len2 = EZ_LEN2, Len4 = EZ_LEN4, LenAlt = EZ_LEN_ALT;
constexpr int Off1 = EZ_OFF1, Off2 = EZ_OFF2, Off4 = EZ_OFF4, OffLong = EZ_OFF_LONG;
constexpr int MetaMagic = EZ_META_MAGIC, MetaVer = EZ_META_VER, MetaReset = EZ_META_RESET, MetaBreak = EZ_META_BREAK;
constexpr int MetaLenWide = EZ_META_LEN_WIDE, MetaLen0 = EZ_META_LEN0, MetaTagMask = 0xf8;
constexpr const char Magic[] = "eazy";

// One code per reference error value (reader.go:57-76) plus the C-ABI's own.
enum class Err : int {
    OK = EZ_OK,
    EOF_ = EZ_EOF,                        // io.EOF
    ShortBuffer = EZ_ESHORTBUF,           // ErrShortBuffer
    UnexpectedEOF = EZ_EUNEXPECTEDEOF,    // io.ErrUnexpectedEOF
    Overflow = EZ_EOVERFLOW,              // ErrOverflow
    BadMagic = EZ_EBADMAGIC,              // ErrBadMagic
    NoMagic = EZ_ENOMAGIC,                // ErrNoMagic
    BlockSizeOverLimit = EZ_EBLOCKLIMIT,  // ErrBlockSizeOverLimit
    UnsupportedMeta = EZ_EUNSUPMETA,      // ErrUnsupportedMeta
    UnsupportedVersion = EZ_EUNSUPVER,    // ErrUnsupportedVersion
    Break = EZ_EBREAK,                    // ErrBreak
    MissedMeta = EZ_EMISSEDMETA,          // "missed meta"
    Invalid = EZ_EINVAL,                  // a Go panic (thrown as Panic by this header)
    Sink = EZ_ESINK,                      // the io.Writer failed
    NoSpace = EZ_ENOSPC,
    Device = EZ_EDEVICE,                  // no usable MI355X
    Stuck = EZ_ESTUCK,
};

inline const char *ErrString(Err e) { return ez_strerror((int)e); }

// What Go does with panic(): invalid sizes, impossible lengths, bad meta.  what() is the
// reference's panic value (writer.go:163, 167, 309, 562, 596); Encoder.Meta panics with the
// meta int itself (writer.go:601): then has_value and value hold it, and what() is its decimal.
struct Panic : std::logic_error {
    explicit Panic(const std::string &w) : std::logic_error(w) {}
    explicit Panic(int64_t v) : std::logic_error(std::to_string(v)), has_value(true), value(v) {}
    bool has_value = false;
    int64_t value = 0;
};

// err.Error() of the Go value an Err stands for (reader.go:57-76): the wrapped forms carry the
// detail (the version, reader.go:303 "%w: %v"; the meta id, :319 "%w: 0x%x").
inline std::string ErrorText(Err e, int64_t detail = 0) {
    char buf[32];
    if (e == Err::UnsupportedVersion) {
        snprintf(buf, sizeof buf, ": %lld", (long long)detail);
        return std::string(ez_strerror((int)e)) + buf;
    }
    if (e == Err::UnsupportedMeta) {
        snprintf(buf, sizeof buf, ": 0x%llx", (long long)detail);
        return std::string(ez_strerror((int)e)) + buf;
    }
    return ez_strerror((int)e);
}

// io.Writer: returns bytes taken and an error (Err::OK on success).
struct IoWriter {
    virtual ~IoWriter() = default;
    virtual std::pair<size_t, Err> Write(const uint8_t *p, size_t n) = 0;
};

// io.Reader with Go semantics: may return n > 0 together with Err::EOF_.
struct IoReader {
    virtual ~IoReader() = default;
    virtual std::pair<size_t, Err> Read(uint8_t *p, size_t n) = 0;
};

// bytes.Buffer-like in-memory sink/source (the reference tests' low.Buf / bytes.Buffer)
struct Buffer : IoWriter, IoReader {
    std::vector<uint8_t> b;
    size_t r = 0;
    std::pair<size_t, Err> Write(const uint8_t *p, size_t n) override {
        b.insert(b.end(), p, p + n);
        return {n, Err::OK};
    }
    std::pair<size_t, Err> Read(uint8_t *p, size_t n) override {
        if (r >= b.size()) return {0, Err::EOF_};
        const size_t k = n < b.size() - r ? n : b.size() - r;
        std::memcpy(p, b.data() + r, k);
        r += k;
        return {k, Err::OK};
    }
    void Append(const std::vector<uint8_t> &x) { b.insert(b.end(), x.begin(), x.end()); }
};

namespace detail {
inline void panic_if(int st, int panic) {
    if (st == EZ_EINVAL) throw Panic(ez_panic_message(panic));
}
inline void size_panic(int64_t block, int64_t htable) {  // Writer.init writer.go:161-169
    const int p = ez_writer_size_panic(block, htable);
    if (p != EZ_PANIC_NONE) throw Panic(ez_panic_message(p));
}
}  // namespace detail

// ---------------------------------------------------------------- codec
struct Encoder {  // writer.go:537-621
    int Ver = 0;
    void Tag(std::vector<uint8_t> &b, int tag, int64_t l) const { app(b, [&](uint8_t *d, size_t c, size_t *n) { return ez_encode_tag(d, c, n, tag, l); }, EZ_PANIC_LENGTH); }
    void Offset(std::vector<uint8_t> &b, int64_t off, int64_t l) const { app(b, [&](uint8_t *d, size_t c, size_t *n) { return ez_encode_offset(d, c, n, off, l); }, EZ_PANIC_OFFSET); }
    void MetaTag(std::vector<uint8_t> &b, int64_t meta, int64_t l) const {
        if (meta & ~(int64_t)MetaTagMask) throw Panic(meta);  // panic(meta) writer.go:600-602
        app(b, [&](uint8_t *d, size_t c, size_t *n) { return ez_encode_meta(d, c, n, meta, l); }, EZ_PANIC_OFFSET);
    }

  private:
    template <class F>
    static void app(std::vector<uint8_t> &b, F f, int panic) {
        const size_t at = b.size();
        b.resize(at + 16);
        size_t n = at;
        const int st = f(b.data(), b.size(), &n);
        detail::panic_if(st, panic);
        b.resize(n);
    }
};

struct Decoder {  // reader.go:346-514; every result carries the next index i (st on error)
    int Ver = 0;
    Err Tag(const std::vector<uint8_t> &b, size_t st, int *tag, int64_t *l, size_t *i) const {
        return (Err)ez_decode_tag(b.data(), b.size(), st, tag, l, i);
    }
    Err Offset(const std::vector<uint8_t> &b, size_t st, int64_t l, int64_t *off, size_t *i) const {
        return (Err)ez_decode_offset(b.data(), b.size(), st, l, off, i);
    }
    Err MetaTag(const std::vector<uint8_t> &b, size_t st, int64_t *meta, int64_t *l, size_t *i) const {
        return (Err)ez_decode_meta(b.data(), b.size(), st, meta, l, i);
    }
};

// ---------------------------------------------------------------- Writer
class Writer {
  public:
    IoWriter *W = nullptr;   // Writer.Writer (writer.go:18)
    bool AppendMagic = true;  // writer.go:23-25
    int FlushThreshold = 0;   // writer.go:27-34: 0 = each Write, -1 = manual, N = buffered bytes
    int Ver = 0;              // w.e.Ver

    Writer(IoWriter *w, int64_t block, int64_t htable, int device = 0) : W(w) {
        detail::size_panic(block, htable);
        const int st = ez_writer_new(block, htable, device, &h_);
        if (st != EZ_OK) throw std::runtime_error(std::string("eazy: NewWriter: ") + ez_strerror(st));
    }
    ~Writer() { ez_writer_free(h_); }
    Writer(const Writer &) = delete;
    Writer &operator=(const Writer &) = delete;

    // Writer.Write writer.go:206-337: {len(p), OK} or {0, err}.
    std::pair<size_t, Err> Write(const uint8_t *p, size_t n) {
        sync();
        size_t got = 0;
        const size_t at = b_.size();
        b_.resize(at + ez_compress_bound(n));
        const int st = ez_writer_write(h_, p, n, b_.data() + at, b_.size() - at, &got);
        b_.resize(at + (st == EZ_OK ? got : 0));
        if (st != EZ_OK) return {0, failed(st)};
        const Err e = write();
        if (e != Err::OK) return {0, e};
        return {n, Err::OK};
    }
    std::pair<size_t, Err> Write(const std::vector<uint8_t> &p) { return Write(p.data(), p.size()); }
    std::pair<size_t, Err> Write(const std::string &p) { return Write((const uint8_t *)p.data(), p.size()); }

    // k Writes in one device call (no reference counterpart): the sink sees what Write on each
    // in turn gives it -- the handle returns where each Write's bytes end and FlushThreshold is
    // replayed per Write; a short sink write that restarts the stream sends the remaining Writes
    // through Write.  p holds the Writes back to back, Write j ending at p[ends[j]].
    // {bytes of the Writes done, first error}.
    std::pair<size_t, Err> WriteBatch(const uint8_t *p, const uint64_t *ends, size_t k) {
        if (k == 0) return {0, Err::OK};
        sync();
        size_t cap = 0;
        for (size_t j = 0; j < k; j++) cap += ez_compress_bound((size_t)(ends[j] - (j ? ends[j - 1] : 0)));
        std::vector<uint8_t> tmp(cap ? cap : 1);
        std::vector<uint64_t> oe(k);
        const int st = ez_writer_write_batch(h_, p, ends, k, tmp.data(), cap, oe.data());
        if (st != EZ_OK) return {0, failed(st)};
        const uint64_t gen = resets_;
        for (size_t j = 0, prev = 0; j < k; prev = oe[j], j++) {
            b_.insert(b_.end(), tmp.begin() + (ptrdiff_t)prev, tmp.begin() + (ptrdiff_t)oe[j]);
            const Err e = write();
            if (e != Err::OK) return {(size_t)(j ? ends[j - 1] : 0), e};
            if (resets_ != gen) {  // the stream restarted: the rest on the new stream
                for (size_t q = j + 1; q < k; q++) {
                    auto [n, e2] = Write(p + ends[q - 1], (size_t)(ends[q] - ends[q - 1]));
                    if (e2 != Err::OK) return {(size_t)ends[q - 1], e2};
                }
                break;
            }
        }
        return {(size_t)ends[k - 1], Err::OK};
    }

    Err WriteHeader() {  // writer.go:342-350
        if (!isreset()) return Err::OK;
        return append_call(ez_writer_header);
    }
    Err WriteBreak() { return append_call(ez_writer_break); }  // writer.go:358-366
    Err Flush() { return b_.empty() ? Err::OK : flush(); }      // writer.go:371-377
    void Reset(IoWriter *w) {                                    // writer.go:149-152
        W = w;
        reset();
    }
    void ResetSize(IoWriter *w, int64_t block, int64_t htable) {  // writer.go:155-159
        W = w;
        detail::size_panic(block, htable);
        const int st = ez_writer_reset_size(h_, block, htable);
        if (st != EZ_OK)  // (the sizes passed size_panic: a device failure; the handle keeps its old sizes)
            throw std::runtime_error(std::string("eazy: ResetSize: ") + ez_strerror(st));
        b_.clear();
        written_ = 0;
    }

  private:
    ez_writer *h_ = nullptr;
    std::vector<uint8_t> b_;  // w.b
    int64_t written_ = 0;     // w.written
    uint64_t resets_ = 0;     // stream restarts (WriteBatch's replay)

    void sync() {
        ez_writer_set_append_magic(h_, AppendMagic ? 1 : 0);
        ez_writer_set_version(h_, Ver);
    }
    bool isreset() const { return written_ + (int64_t)b_.size() == 0 && ez_writer_is_reset(h_); }  // writer.go:403-405
    Err append_call(int (*f)(ez_writer *, uint8_t *, size_t, size_t *)) {
        sync();
        const size_t at = b_.size();
        b_.resize(at + 32);
        size_t got = 0;
        const int st = f(h_, b_.data() + at, 32, &got);
        b_.resize(at + (st == EZ_OK ? got : 0));
        if (st != EZ_OK) return (Err)st;
        return write();
    }
    // A failed Write: when the device history had taken it, the handle restarted its stream (it is
    // reset now) and the mirror forgets w.b and written too; a failure found before anything reached
    // the device (NoSpace, bad Write ends, no device) leaves both as they were.  Invalid with a
    // reference panic behind it throws that panic; without one it is an invalid argument.
    Err failed(int st) {
        if (ez_writer_is_reset(h_)) {
            resets_++;
            b_.clear();
            written_ = 0;
        }
        if (st == EZ_EINVAL) {
            const int p = ez_writer_last_panic(h_);
            if (p != EZ_PANIC_NONE) throw Panic(ez_panic_message(p));
            throw std::invalid_argument("eazy: Write: invalid arguments");
        }
        return (Err)st;
    }
    void reset() {  // writer.go:187-200
        resets_++;
        ez_writer_reset(h_);
        b_.clear();
        written_ = 0;
    }
    Err write() {  // writer.go:379-385
        if (FlushThreshold < 0 || (int64_t)b_.size() < FlushThreshold) return Err::OK;
        return flush();
    }
    Err flush() {  // writer.go:387-401: a failed or short sink write restarts the stream
        auto [n, err] = W->Write(b_.data(), b_.size());
        written_ += (int64_t)n;
        if (err != Err::OK || n != b_.size()) reset();
        if (err != Err::OK) return err;
        b_.clear();
        return Err::OK;
    }
};

inline std::unique_ptr<Writer> NewWriter(IoWriter *w, int64_t block, int64_t htable, int device = 0) {
    return std::make_unique<Writer>(w, block, htable, device);
}

// ---------------------------------------------------------------- Reader
class Reader {
  public:
    IoReader *R = nullptr;              // Reader.Reader (reader.go:20)
    int64_t BlockSizeLimit = 16 * MiB;  // NewReader default (reader.go:79-86); NewReaderBytes: 0
    int BufferSize = 64 * 1024;
    bool RequireMagic = false;
    bool SkipUnsupportedMeta = false;
    int64_t Detail = 0;  // meta id / version of the last UnsupportedMeta / UnsupportedVersion

    explicit Reader(int device = 0) {
        const int st = ez_reader_new(device, &h_);
        if (st != EZ_OK) throw std::runtime_error(std::string("eazy: NewReader: ") + ez_strerror(st));
    }
    ~Reader() { ez_reader_free(h_); }
    Reader(const Reader &) = delete;
    Reader &operator=(const Reader &) = delete;

    void Reset(IoReader *r) {  // reader.go:96-99
        ResetBytes(nullptr, 0);
        R = r;
        ez_reader_set_whole(h_, 0);
    }
    // (a whole buffer: the handle decodes it at once on the first Read, ez_reader_set_whole)
    void ResetBytes(const uint8_t *b, size_t n) {  // reader.go:102-113
        R = nullptr;
        b_.assign(b, b + n);
        bcap_ = n;
        i_ = 0;
        boff_ = 0;
        ez_reader_reset(h_);
        ez_reader_set_whole(h_, 1);
    }
    void ResetBytes(const std::vector<uint8_t> &b) { ResetBytes(b.data(), b.size()); }

    // Reader.Read reader.go:116-141: data and error together, like Go.
    std::pair<size_t, Err> Read(uint8_t *p, size_t n) {
        ez_reader_configure(h_, BlockSizeLimit, RequireMagic ? 1 : 0, SkipUnsupportedMeta ? 1 : 0);
        size_t got = 0;
        Err err = Err::OK;
        while (got < n && err == Err::OK) {
            size_t m = 0, i = 0;
            int64_t det = 0;
            err = (Err)ez_reader_read(h_, b_.data(), b_.size(), i_, boff_, p + got, n - got, &m, &i, &det);
            if (err == Err::Device) return {got, err};
            got += m;
            i_ = i;
            Detail = det;
            if (got == n) break;
            if (err != Err::ShortBuffer) continue;
            err = more();
            if (err == Err::EOF_ && (ez_reader_pending(h_) || i_ < b_.size())) err = Err::UnexpectedEOF;
        }
        return {got, err};
    }
    std::pair<std::vector<uint8_t>, Err> Read(size_t n) {
        std::vector<uint8_t> p(n);
        auto [k, e] = Read(p.data(), n);
        p.resize(k);
        return {p, e};
    }
    // the C-ABI handle (tests, measurement: ez_reader_whole_decoded, ez_reader_set_whole)
    ez_reader *Handle() const { return h_; }

  private:
    ez_reader *h_ = nullptr;
    std::vector<uint8_t> b_;  // r.b
    size_t bcap_ = 0;         // cap(r.b)
    size_t i_ = 0;            // r.i
    int64_t boff_ = 0;        // r.boff

    // cap(append(s, ...)) for a []byte of capacity c grown to n elements: Go 1.20's growslice and
    // roundupsize (runtime/slice.go, runtime/sizeclasses.go; the reference's go.mod)
    static size_t go_append_cap(size_t c, size_t n) {
        if (n <= c) return c;
        size_t nc = c;
        if (n > 2 * c) nc = n;
        else if (c < 256) nc = 2 * c;
        else
            while (nc < n) nc += (nc + 3 * 256) / 4;
        static const uint16_t cls[] = {8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320, 352, 384, 416,
                                       448, 480, 512, 576, 640, 704, 768, 896, 1024, 1152, 1280, 1408, 1536, 1792, 2048, 2304, 2688, 3072, 3200,
                                       3456, 4096, 4864, 5376, 6144, 6528, 6784, 6912, 8192, 9472, 9728, 10240, 10880, 12288, 13568, 14336,
                                       16384, 18432, 19072, 20480, 21760, 24576, 27264, 28672, 32768};
        if (nc < 32768) {
            for (uint16_t k : cls)
                if (k >= nc) return k;
        }
        return (nc + 8191) & ~(size_t)8191;
    }

    Err more() {  // reader.go:516-543
        if (!R) return Err::EOF_;
        b_.erase(b_.begin(), b_.begin() + (ptrdiff_t)i_);
        boff_ += (int64_t)i_;
        i_ = 0;
        const size_t end = b_.size();
        // r.b = make([]byte, r.BufferSize), or append(r.b, make([]byte, 1024)...) in the same array
        // while it has room: the io.Reader is offered r.b[end:cap(r.b)]
        bcap_ = end == 0 ? (size_t)BufferSize : go_append_cap(bcap_, end + 1024);
        b_.resize(bcap_);
        auto [k, err] = R->Read(b_.data() + end, b_.size() - end);
        b_.resize(end + k);
        if (k != 0 && err == Err::EOF_) err = Err::OK;
        return err;
    }
};

inline std::unique_ptr<Reader> NewReader(IoReader *r, int device = 0) {  // reader.go:79-86
    auto x = std::make_unique<Reader>(device);
    x->R = r;
    return x;
}

inline std::unique_ptr<Reader> NewReaderBytes(const std::vector<uint8_t> &b, int device = 0) {  // reader.go:89-94
    auto x = std::make_unique<Reader>(device);
    x->ResetBytes(b);
    x->BlockSizeLimit = 0;
    x->BufferSize = 0;
    return x;
}

// ---------------------------------------------------------------- Dumper (reader.go:43-54, 545-732)
// The debug printer of a compressed stream, host side as in the reference: the tokens are walked
// with the C-ABI's Decoder and printed one line each in the reference's text format (Go fmt verbs:
// %x widths, %q quoting, % x).  Checked against eazy_amd/dump.py (tests/cpp/eazy_test.cpp).
namespace detail {
#include "eazy_isprint.inc"

inline bool is_print(uint32_t r) {  // strconv.IsPrint as dump.py restates it
    size_t lo = 0, hi = sizeof kPrintRanges / sizeof kPrintRanges[0];
    while (lo < hi) {
        const size_t m = (lo + hi) / 2;
        if (r < kPrintRanges[m][0]) hi = m;
        else if (r > kPrintRanges[m][1]) lo = m + 1;
        else return true;
    }
    return false;
}

// utf8.DecodeRune of b[i..n): {rune, width}; {0xFFFD, 1} for an invalid encoding
inline std::pair<uint32_t, int> decode_rune(const uint8_t *b, size_t n, size_t i) {
    const uint32_t c = b[i];
    if (c < 0x80) return {c, 1};
    const int w = c >= 0xC2 && c <= 0xDF ? 2 : c >= 0xE0 && c <= 0xEF ? 3 : c >= 0xF0 && c <= 0xF4 ? 4 : 0;
    if (w == 0 || i + (size_t)w > n) return {0xFFFD, 1};
    // the second byte's range depends on the first (no overlongs, surrogates or > U+10FFFF)
    const uint32_t c1 = b[i + 1];
    const uint32_t lo = c == 0xE0 ? 0xA0 : c == 0xF0 ? 0x90 : 0x80, hi = c == 0xED ? 0x9F : c == 0xF4 ? 0x8F : 0xBF;
    if (c1 < lo || c1 > hi) return {0xFFFD, 1};
    uint32_t r = w == 2 ? (c & 0x1F) : w == 3 ? (c & 0x0F) : (c & 0x07);
    r = (r << 6) | (c1 & 0x3F);
    for (int k = 2; k < w; k++) {
        const uint32_t ck = b[i + (size_t)k];
        if (ck < 0x80 || ck > 0xBF) return {0xFFFD, 1};
        r = (r << 6) | (ck & 0x3F);
    }
    return {r, w};
}

// fmt's %q of a []byte (strconv.Quote); *runes = its length in code points (fmt pads by those)
inline std::string go_quote(const uint8_t *b, size_t n, size_t *runes = nullptr) {
    std::string s = "\"";
    size_t cnt = 1;
    char esc[16];
    for (size_t i = 0; i < n;) {
        const auto [r, w] = decode_rune(b, n, i);
        if (w == 1 && r == 0xFFFD) {
            snprintf(esc, sizeof esc, "\\x%02x", b[i]);
            s += esc;
            cnt += 4;
            i++;
            continue;
        }
        const uint8_t *raw = b + i;
        i += (size_t)w;
        if (r == '"' || r == '\\') {
            s += '\\';
            s += (char)r;
            cnt += 2;
        } else if (is_print(r)) {
            s.append((const char *)raw, (size_t)w);
            cnt += 1;
        } else if (r >= 7 && r <= 13) {  // \a \b \t \n \v \f \r
            s += '\\';
            s += "abtnvfr"[r - 7];
            cnt += 2;
        } else if (r < 0x20 || r == 0x7F) {
            snprintf(esc, sizeof esc, "\\x%02x", r);
            s += esc;
            cnt += 4;
        } else if (r < 0x10000) {
            snprintf(esc, sizeof esc, "\\u%04x", r);
            s += esc;
            cnt += 6;
        } else {
            snprintf(esc, sizeof esc, "\\U%08x", r);
            s += esc;
            cnt += 10;
        }
    }
    s += '"';
    if (runes) *runes = cnt + 1;
    return s;
}

inline void appendf(std::string &s, const char *fmt, long long a, long long b = 0) {
    char t[64];
    snprintf(t, sizeof t, fmt, a, b);
    s += t;
}
}  // namespace detail

class Dumper {
  public:
    IoWriter *W = nullptr;  // Dumper.Writer (nullptr: the text stays in Text())
    // called once per printed item: input range, output offset, kind ('p','m','l','c','e'), length, offset
    std::function<void(int64_t ioff, int64_t iend, int64_t ooff, uint8_t tag, int64_t l, int64_t off)> Debug;
    int64_t GlobalOffset = 0;  // < 0: no global-offset column

    // Dumper.Write reader.go:602-710: prints every whole token of p; {bytes those took, error}
    std::pair<size_t, Err> Write(const uint8_t *p, size_t n) {
        b_.clear();
        size_t i = 0;
        const Err e = walk(p, n, &i);
        boff_ += (int64_t)i;
        if (GlobalOffset >= 0) GlobalOffset += (int64_t)i;
        Err out = e;
        if (W) {
            const Err we = W->Write((const uint8_t *)b_.data(), b_.size()).second;
            if (out == Err::OK) out = we;
        }
        return {i, out};
    }
    std::pair<size_t, Err> Write(const std::vector<uint8_t> &p) { return Write(p.data(), p.size()); }

    // Dumper.ReadFrom reader.go:563-600: a token cut by a read boundary is carried to the next read
    std::pair<int64_t, Err> ReadFrom(IoReader *r) {
        if (p_.empty()) p_.resize(0x10000);
        size_t kept = 0;
        int64_t total = 0;
        Err err = Err::OK;
        for (;;) {
            size_t k;
            std::tie(k, err) = r->Read(p_.data() + kept, p_.size() - kept);
            if (k == 0) break;
            total += (int64_t)k;
            size_t used;
            std::tie(used, err) = Write(p_.data(), kept + k);
            std::memmove(p_.data(), p_.data() + used, kept + k - used);
            kept = kept + k - used;
            if (err != Err::OK && err != Err::ShortBuffer) break;
        }
        if (err == Err::EOF_) err = Err::OK;
        if (kept != 0 && err == Err::OK) err = Err::UnexpectedEOF;
        return {total, err};
    }

    Err Close() {  // reader.go:712-732
        if (GlobalOffset >= 0) detail::appendf(b_, "%6llx  ", GlobalOffset);
        detail::appendf(b_, "%4llx  %6llx  ", 0, pos_);
        if (Debug) Debug(boff_, boff_, pos_, 'e', 0, 0);
        return Err::OK;
    }

    const std::string &Text() const { return b_; }  // what the last Write / Close printed (d.b)

  private:
    int ver_ = 0;        // Decoder.Ver (a version meta sets it)
    int64_t pos_ = 0;    // output position (r.pos)
    int64_t boff_ = 0;   // input consumed by earlier Writes (r.boff)
    std::string b_;
    std::vector<uint8_t> p_;

    void dbg(size_t st, size_t i, char kind, int64_t l, int64_t off) {
        if (Debug) Debug(boff_ + (int64_t)st, boff_ + (int64_t)i, pos_, (uint8_t)kind, l, off);
    }
    Err walk(const uint8_t *p, size_t n, size_t *at) {
        size_t i = 0;
        for (;;) {
            *at = i;
            if (i >= n) return Err::OK;
            const size_t st = i;
            if (GlobalOffset >= 0) detail::appendf(b_, "%6llx  ", GlobalOffset + (long long)st);
            detail::appendf(b_, "%4llx  %6llx  ", (long long)st, pos_);
            while (i < n && p[i] == 0) i++;
            if (i > st) {
                detail::appendf(b_, "pad  %4llx\n", (long long)(i - st));
                dbg(st, i, 'p', (int64_t)(i - st), 0);
                continue;
            }
            int tag = 0;
            int64_t l = 0;
            size_t j = st;
            Err e = (Err)ez_decode_tag(p, n, i, &tag, &l, &j);
            if (e != Err::OK) return *at = st, e;
            if (tag == Meta && l == 0) {
                int64_t meta = 0, ml = 0;
                size_t k = j;
                e = (Err)ez_decode_meta(p, n, j, &meta, &ml, &k);
                if (e != Err::OK) return *at = k, e;
                if (k + (size_t)ml > n) return *at = k, Err::ShortBuffer;
                if (meta == MetaVer && ml == 1) ver_ = p[k];
                size_t runes = 0;
                const std::string q = detail::go_quote(p + k, (size_t)ml, &runes);
                detail::appendf(b_, "meta %2llx %llx  ", meta >> 3, ml);
                b_ += q;
                for (; runes < 8; runes++) b_ += ' ';
                b_ += "  ";
                for (int64_t x = 0; x < ml; x++) detail::appendf(b_, x ? " %02llx" : "%02llx", p[k + (size_t)x]);
                b_ += '\n';
                dbg(st, k, 'm', ml, meta);
                i = k + (size_t)ml;
            } else if (tag == Literal) {
                if (j + (size_t)l > n) return *at = j, Err::ShortBuffer;
                detail::appendf(b_, "lit  %4llx        ", l);
                b_ += detail::go_quote(p + j, (size_t)l);
                b_ += '\n';
                dbg(st, j, 'l', l, 0);
                i = j + (size_t)l;
                pos_ += l;
            } else {  // Copy
                const bool lng = j < n && p[j] == OffLong;
                int64_t off = 0;
                size_t k = j;
                e = (Err)ez_decode_offset(p, n, j, l, &off, &k);
                if (e != Err::OK) return *at = st, e;
                detail::appendf(b_, "copy %4llx  off %4llx", l, off);
                if (lng) b_ += "  (long)";
                b_ += '\n';
                dbg(st, k, 'c', l, off);
                i = k;
                pos_ += l;
            }
        }
    }
};

inline std::unique_ptr<Dumper> NewDumper(IoWriter *w) {  // reader.go:557-561
    auto d = std::make_unique<Dumper>();
    d->W = w;
    return d;
}

// Dump reader.go:545-555: the debug print of a compressed buffer, with the error that stopped it
inline std::string Dump(const uint8_t *p, size_t n) {
    Dumper d;
    const Err e = d.Write(p, n).second;
    d.Close();
    std::string s = d.Text();
    if (e != Err::OK) s += "\nerror: " + ErrorText(e);
    return s;
}
inline std::string Dump(const std::vector<uint8_t> &p) { return Dump(p.data(), p.size()); }

// ---------------------------------------------------------------- batches (the GPU hot path)
// One stream per buffer = a fresh NewWriter(block, htable) receiving one
// Write; device pointers, asynchronous on `hip_stream`.  See include/eazy.h.
// Invalid sizes throw the reference's Panic (Writer.init); other invalid batch arguments throw
// std::invalid_argument (Err::Invalid is never returned).
inline Err CompressBatch(int64_t block, int64_t htable, bool append_magic, const ez_batch &b, void *hip_stream) {
    const int st = ez_compress_batch(block, htable, append_magic ? 0 : EZ_F_NO_MAGIC, &b, hip_stream);
    if (st == EZ_EINVAL) {
        detail::size_panic(block, htable);
        throw std::invalid_argument("eazy: CompressBatch: invalid batch arguments");
    }
    return (Err)st;
}
// ez_release_cached: the device scratch kept between batch calls freed (device < 0: every device)
inline Err ReleaseCached(int device = -1) { return (Err)ez_release_cached(device); }

inline Err DecompressBatch(int64_t block_size_limit, const ez_batch &b, void *workspace, void *hip_stream) {
    return (Err)ez_decompress_batch(block_size_limit, &b, workspace, hip_stream);
}

// Host-memory batches over several devices (ez_compress_batch_multi / ez_decompress_batch_multi):
// bufs[k] is one Write to a fresh NewWriter(block, htable); out[k] gets its compressed bytes,
// computed in contiguous whole-stream shards, one per entry of `devices` (empty: every device).
// Err::Device without a usable device; a stream's own error otherwise (the first one).
inline Err CompressBatchMulti(const std::vector<std::vector<uint8_t>> &bufs, int64_t block, int64_t htable,
                              std::vector<std::vector<uint8_t>> &out, const std::vector<int> &devices = {},
                              bool append_magic = true) {
    detail::size_panic(block, htable);
    std::vector<uint64_t> off(bufs.size() + 1, 0);
    uint64_t cap = 16;
    for (size_t k = 0; k < bufs.size(); k++) {
        off[k + 1] = off[k] + bufs[k].size();
        cap += ez_compress_bound(bufs[k].size());
    }
    std::vector<uint8_t> in;
    in.reserve(off.back());
    for (const auto &b : bufs) in.insert(in.end(), b.begin(), b.end());
    std::vector<uint8_t> packed(cap);
    std::vector<uint64_t> poff(bufs.size() + 1, 0);
    std::vector<int32_t> status(bufs.size() + 1, 0);
    const int st = ez_compress_batch_multi(block, htable, append_magic ? 0 : EZ_F_NO_MAGIC, in.data(), off.data(), bufs.size(),
                                           devices.empty() ? nullptr : devices.data(), (int)devices.size(), packed.data(), cap,
                                           poff.data(), status.data());
    if (st == EZ_EINVAL) throw std::invalid_argument("eazy: CompressBatchMulti: invalid arguments");
    if (st != EZ_OK) return (Err)st;
    out.assign(bufs.size(), {});
    for (size_t k = 0; k < bufs.size(); k++) {
        if (status[k] != EZ_OK) return (Err)status[k];
        out[k].assign(packed.begin() + (ptrdiff_t)poff[k], packed.begin() + (ptrdiff_t)poff[k + 1]);
    }
    return Err::OK;
}

// Every stream read to EOF (NewReaderBytes; Break metas skipped) into a slot of slot_bytes[k]
// bytes: out[k] = (its output, its first error or OK).
inline Err DecompressBatchMulti(const std::vector<std::vector<uint8_t>> &streams, const std::vector<uint64_t> &slot_bytes,
                                std::vector<std::pair<std::vector<uint8_t>, Err>> &out, const std::vector<int> &devices = {},
                                int64_t block_size_limit = 0) {
    if (slot_bytes.size() != streams.size()) throw std::invalid_argument("eazy: DecompressBatchMulti: one slot per stream");
    std::vector<uint64_t> off(streams.size() + 1, 0), ooff(streams.size() + 1, 0);
    for (size_t k = 0; k < streams.size(); k++) {
        off[k + 1] = off[k] + streams[k].size();
        ooff[k + 1] = ooff[k] + slot_bytes[k];
    }
    std::vector<uint8_t> in;
    in.reserve(off.back());
    for (const auto &b : streams) in.insert(in.end(), b.begin(), b.end());
    std::vector<uint8_t> buf(ooff.back() + 1);
    std::vector<uint64_t> sizes(streams.size() + 1, 0);
    std::vector<int32_t> status(streams.size() + 1, 0);
    const int st = ez_decompress_batch_multi(block_size_limit, in.data(), off.data(), streams.size(),
                                             devices.empty() ? nullptr : devices.data(), (int)devices.size(), buf.data(), ooff.data(),
                                             sizes.data(), status.data());
    if (st == EZ_EINVAL) throw std::invalid_argument("eazy: DecompressBatchMulti: invalid arguments");
    if (st != EZ_OK) return (Err)st;
    out.assign(streams.size(), {});
    for (size_t k = 0; k < streams.size(); k++)
        out[k] = {std::vector<uint8_t>(buf.begin() + (ptrdiff_t)ooff[k], buf.begin() + (ptrdiff_t)(ooff[k] + sizes[k])), (Err)status[k]};
    return Err::OK;
}

}  // namespace eazy
