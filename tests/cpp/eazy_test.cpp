// eazy_test.cpp — the reference's tests (eazy_test.go) restated in C++ over
// the C++ host side (eazy_amd/cpp/eazy.hpp) and the C-ABI.  Exact-byte
// expectations are the Go tests' known answers.
//
//   ./eazy_test          all tests (needs an MI355X for the Writer/Reader ones)
//   ./eazy_test --cpu    host-only tests: the token codec, compress bound, ABI
#include <chrono>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../eazy_amd/cpp/eazy.hpp"

using namespace eazy;
using Bytes = std::vector<uint8_t>;

static int g_fail = 0, g_run = 0;
#define CHECK(c)                                                             \
    do {                                                                     \
        if (!(c)) {                                                          \
            std::printf("    %s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            throw 1;                                                         \
        }                                                                    \
    } while (0)

static Bytes B(const std::string &s) { return Bytes(s.begin(), s.end()); }
static Bytes H(const std::string &hex) {
    Bytes b;
    for (size_t i = 0; i + 1 < hex.size(); i += 2) b.push_back((uint8_t)std::stoi(hex.substr(i, 2), nullptr, 16));
    return b;
}
static Bytes cat(Bytes a, const Bytes &b) {
    a.insert(a.end(), b.begin(), b.end());
    return a;
}
static Bytes sub(const Bytes &a, size_t from, size_t to = (size_t)-1) {
    if (to > a.size()) to = a.size();
    return Bytes(a.begin() + (ptrdiff_t)from, a.begin() + (ptrdiff_t)to);
}

static void run(const char *name, const std::function<void()> &f) {
    g_run++;
    try {
        f();
        std::printf("PASS %s\n", name);
    } catch (...) {
        g_fail++;
        std::printf("FAIL %s\n", name);
    }
}

static void write_ok(Writer &w, const Bytes &p) {
    auto [n, e] = w.Write(p);
    CHECK(e == Err::OK);
    CHECK(n == p.size());
}

static std::pair<Bytes, Err> rd(Reader &r, size_t n) { return r.Read(n); }

// ---------------------------------------------------------------- host-only
static void TestPrintLengthEncoding() {  // eazy_test.go:1406-1450
    const std::pair<int64_t, const char *> kat[] = {{1, "01"}, {123, "7b"}, {124, "7c00"}, {379, "7cff"},
                                                    {380, "7d0000"}, {65915, "7dffff"}, {65916, "7e00000000"}};
    Encoder e;
    Decoder d;
    for (auto &[l, h] : kat) {
        Bytes b;
        e.Tag(b, Literal, l);
        CHECK(b == H(h));
        int tag = -1;
        int64_t got = -1;
        size_t i = 0;
        CHECK(d.Tag(b, 0, &tag, &got, &i) == Err::OK);
        CHECK(tag == Literal && got == l && i == b.size());
    }
}

static void TestPrintOffsetEncoding() {  // eazy_test.go:1452-1497
    const std::pair<int64_t, const char *> kat[] = {{1, "01"}, {251, "fb"}, {252, "fc00"}, {507, "fcff"},
                                                    {508, "fd0000"}, {66043, "fdffff"}, {66044, "fe00000000"}};
    Encoder e;
    for (auto &[o, h] : kat) {
        Bytes b;
        e.Offset(b, o, 0);
        CHECK(b == H(h));
    }
    Bytes b;
    e.Offset(b, 5, 10);
    CHECK(b == H("ff05"));
    b.clear();
    e.Offset(b, 20, 10);
    CHECK(b == H("0a"));
    int64_t off = 0;
    size_t i = 0;
    CHECK(Decoder().Offset(H("fd0365"), 0, 0, &off, &i) == Err::OK);
    CHECK(off == 26367 && i == 3);  // TestBug1's offset
}

static void TestReaderShortBuffer() {  // eazy_test.go:858-978
    Encoder e;
    Decoder d;
    for (int64_t tlen : {(int64_t)20, (int64_t)0x100, (int64_t)0x200, (int64_t)0x50000000}) {
        Bytes b;
        e.Tag(b, Copy, tlen);
        for (size_t k = 0; k < b.size(); k++) {
            int tag = 0;
            int64_t l = 0;
            size_t i = 99;
            CHECK(d.Tag(sub(b, 0, k), 0, &tag, &l, &i) == Err::ShortBuffer);
            CHECK(i == 0);
        }
    }
    for (int64_t toff : {(int64_t)20, (int64_t)0x100, (int64_t)0x200, (int64_t)0x500, (int64_t)0x50000000}) {
        for (int64_t l : {(int64_t)10, toff + 10}) {
            Bytes b;
            e.Offset(b, toff, l);
            for (size_t k = 0; k < b.size(); k++) {
                int64_t off = 0;
                size_t i = 99;
                CHECK(d.Offset(sub(b, 0, k), 0, l, &off, &i) == Err::ShortBuffer && i == 0);
            }
            int64_t off = 0;
            size_t i = 0;
            CHECK(d.Offset(b, 0, l, &off, &i) == Err::OK && off == toff && i == b.size());
        }
    }
    for (int64_t tlen : {(int64_t)0, (int64_t)4, (int64_t)0x80, (int64_t)0x100, (int64_t)0x500, (int64_t)0x50000000}) {
        Bytes b;
        e.MetaTag(b, 10 << 3, tlen);
        for (size_t k = 1; k < b.size(); k++) {
            int64_t m = 0, l = 0;
            size_t i = 99;
            CHECK(d.MetaTag(sub(b, 0, k), 1, &m, &l, &i) == Err::ShortBuffer && i == 1);
        }
        int64_t m = 0, l = 0;
        size_t i = 0;
        CHECK(d.MetaTag(b, 1, &m, &l, &i) == Err::OK && m == (10 << 3) && l == tlen && i == b.size());
    }
}

static void TestEncoderPanics() {  // eazy_test.go:895, 946, TestMeta :814
    Encoder e;
    Bytes b;
    bool p1 = false, p2 = false, p3 = false, p4 = false;
    // the panic values themselves (writer.go:562, 596, 601)
    try { e.Tag(b, Literal, 0x110000000LL); } catch (const Panic &p) { p1 = std::string(p.what()) == "too big length"; }
    try { e.Offset(b, 0x110000000LL, 10); } catch (const Panic &p) { p2 = std::string(p.what()) == "too big offset"; }
    try { e.MetaTag(b, 1024, 4); } catch (const Panic &p) { p3 = p.has_value && p.value == 1024; }
    try { e.MetaTag(b, MetaReset, 0x110000000LL); } catch (const Panic &p) { p4 = std::string(p.what()) == "too big offset"; }
    CHECK(p1 && p2 && p3 && p4);
}

static std::string size_panic(int64_t bs, int64_t hs) {
    try {
        Buffer buf;
        NewWriter(&buf, bs, hs);
    } catch (const Panic &p) {
        return p.what();
    } catch (...) {
        return "(no panic)";
    }
    return "(no panic)";
}

static void TestErrorText() {  // reader.go:57-76, 303, 319; Writer.init writer.go:161-169
    CHECK(ErrorText(Err::BadMagic) == "bad magic");
    CHECK(ErrorText(Err::BlockSizeOverLimit) == "block size is more than the limit");
    CHECK(ErrorText(Err::NoMagic) == "no magic");
    CHECK(ErrorText(Err::Overflow) == "length/offset overflow");
    CHECK(ErrorText(Err::ShortBuffer) == "short buffer");
    CHECK(ErrorText(Err::UnsupportedMeta, 0x28) == "unsupported meta tag: 0x28");
    CHECK(ErrorText(Err::UnsupportedVersion, 1) == "unsupported file format version: 1");
    CHECK(ErrorText(Err::Break) == "break point");
    CHECK(ErrorText(Err::MissedMeta) == "missed meta");
    CHECK(ErrorText(Err::EOF_) == "EOF");
    CHECK(ErrorText(Err::UnexpectedEOF) == "unexpected EOF");
    const std::string bsp = "block size must be a power of two (32 < bs < 1<<31)";
    const std::string hsp = "hash table size must be a power of two (hs >= 4)";
    CHECK(size_panic(31, 16) == bsp && size_panic(16, 16) == bsp && size_panic(1LL << 32, 16) == bsp);
    CHECK(size_panic(48, 3) == bsp);  // the block check comes first
    CHECK(size_panic(1024, 3) == hsp && size_panic(1024, 6) == hsp && size_panic(1024, 0) == hsp);
}

static void TestCompressBound() {  // include/eazy.h, tests/test_bound.py
    for (size_t n : {0UL, 1UL, 4096UL, 1UL << 20})
        CHECK(ez_compress_bound(n) == n + n / 4 + 32);
    CHECK(ez_abi_version() == EZ_ABI_VERSION);
}

// ---------------------------------------------------------------- device
static void TestMagic() {  // eazy_test.go:39-64
    Buffer buf;
    auto w = NewWriter(&buf, MiB, 512);
    CHECK(w->WriteHeader() == Err::OK);
    CHECK(buf.b == H("800265617a79801014"));
    CHECK(w->WriteHeader() == Err::OK);
    CHECK(buf.b.size() == 9);
    write_ok(*w, Bytes{0});
    CHECK(buf.b == H("800265617a7980101401" "00"));
}

static void TestLiteral() {  // eazy_test.go:66-104
    Buffer buf;
    auto w = NewWriter(&buf, 32, 16);
    w->AppendMagic = false;
    write_ok(*w, B("very_first_message"));
    auto r = NewReaderBytes(buf.b);
    CHECK(rd(*r, 10) == std::make_pair(B("very_first"), Err::OK));
    CHECK(rd(*r, 10) == std::make_pair(B("_message"), Err::EOF_));
}

static void TestCopy() {  // eazy_test.go:106-183
    Buffer buf;
    auto w = NewWriter(&buf, 32, 16);
    w->AppendMagic = false;
    write_ok(*w, B("prefix_1234_suffix"));
    const size_t st = buf.b.size();
    write_ok(*w, B("prefix_567_suffix"));
    CHECK(sub(buf.b, st) == cat(cat(Bytes{Copy | 7, 0x12 - 7, Literal | 3}, B("567")), Bytes{Copy | 7, 0x11 - 7}));
    CHECK(sub(buf.b, 0, st) == cat(Bytes{Meta, MetaReset, 5, 0x12}, B("prefix_1234_suffix")));
    auto r = NewReaderBytes(buf.b);
    CHECK(rd(*r, 10) == std::make_pair(B("prefix_123"), Err::OK));
    CHECK(rd(*r, 10) == std::make_pair(B("4_suffixpr"), Err::OK));
    CHECK(rd(*r, 30) == std::make_pair(B("efix_567_suffix"), Err::EOF_));
}

struct BufNoEOF : IoReader {  // bytes.Buffer: never returns data together with EOF
    Bytes b;
    size_t r = 0;
    std::pair<size_t, Err> Read(uint8_t *p, size_t n) override {
        if (r >= b.size()) return {0, Err::EOF_};
        const size_t k = std::min(n, b.size() - r);
        std::memcpy(p, b.data() + r, k);
        r += k;
        return {k, Err::OK};
    }
};

static void TestBug1() {  // eazy_test.go:185-207
    BufNoEOF src;
    src.b = {Meta, MetaReset, 14, Literal | 3, 0x94, 0xa8, 0xfb, Copy | 9};
    auto r = NewReader(&src);
    auto [got, err] = rd(*r, 1000);
    CHECK(err == Err::UnexpectedEOF);
    CHECK(got == (Bytes{0x94, 0xa8, 0xfb}));
    src.b.insert(src.b.end(), {0xfd, 0x03, 0x65});
    auto [got2, err2] = rd(*r, 1000);
    CHECK(err2 == Err::Overflow);
    CHECK(got2.empty());
}

static void TestPadding() {  // eazy_test.go:209-268
    Buffer buf;
    auto w = NewWriter(&buf, 32, 16);
    write_ok(*w, B("prefix_1234_suffix"));
    const Bytes head = buf.b;
    const Bytes pad(32 - head.size() % 32, 0);
    write_ok(*w, B("prefix_567_suffix"));
    const Bytes all = cat(cat(head, pad), sub(buf.b, head.size()));
    auto r = NewReaderBytes(all);
    CHECK(rd(*r, 10) == std::make_pair(B("prefix_123"), Err::OK));
    CHECK(rd(*r, 10) == std::make_pair(B("4_suffixpr"), Err::OK));
    CHECK(rd(*r, 30) == std::make_pair(B("efix_567_suffix"), Err::EOF_));
}

static void TestZeroRegion() {  // eazy_test.go:270-280
    auto r = NewReaderBytes(Bytes{Meta, MetaReset, 2, Meta, MetaVer, 0, Copy | 10, OffLong, 0});
    CHECK(rd(*r, 16) == std::make_pair(Bytes(10, 0), Err::EOF_));
}

static void TestBreak() {  // eazy_test.go:342-415
    Buffer buf;
    auto w = NewWriter(&buf, 32, 16);
    w->AppendMagic = false;
    write_ok(*w, B("message1"));
    CHECK(w->WriteBreak() == Err::OK);
    write_ok(*w, B("qwessage2"));
    auto r = NewReaderBytes(buf.b);
    CHECK(rd(*r, 20) == std::make_pair(B("message1"), Err::Break));
    CHECK(rd(*r, 20) == std::make_pair(B("qwessage2"), Err::EOF_));
}

static void TestReaderRequireMagic() {  // eazy_test.go:417-431
    Buffer buf;
    auto w = NewWriter(&buf, 1024, 32);
    w->AppendMagic = false;
    write_ok(*w, Bytes{0});
    Buffer src;
    src.b = buf.b;
    auto r = NewReader(&src);
    r->RequireMagic = true;
    CHECK(rd(*r, 1).second == Err::NoMagic);
}

static void TestFlush() {  // eazy_test.go:433-491
    Buffer buf;
    auto w = NewWriter(&buf, 1024, 32);
    w->AppendMagic = false;
    w->FlushThreshold = -1;
    CHECK(w->WriteHeader() == Err::OK);
    write_ok(*w, B("aaabbb"));
    CHECK(w->WriteBreak() == Err::OK);
    write_ok(*w, B("ccc"));
    CHECK(buf.b.empty());
    CHECK(w->Flush() == Err::OK);
    CHECK(buf.b.size() == 16);
    CHECK(w->WriteBreak() == Err::OK);
    CHECK(buf.b.size() == 16);
    CHECK(w->Flush() == Err::OK);
    CHECK(buf.b == H("80100a06616161626262801f03636363801f"));
    Buffer src;
    src.b = buf.b;
    auto r = NewReader(&src);
    CHECK(rd(*r, 10) == std::make_pair(B("aaabbb"), Err::Break));
    CHECK(rd(*r, 10) == std::make_pair(B("ccc"), Err::Break));
    CHECK(rd(*r, 10) == std::make_pair(Bytes{}, Err::EOF_));
}

static void TestFlushReset() {  // eazy_test.go:493-512
    Buffer buf;
    auto w = NewWriter(&buf, 1024, 32);
    w->AppendMagic = false;
    w->FlushThreshold = -1;
    write_ok(*w, B("123"));
    CHECK(buf.b.empty());
    w->Reset(&buf);
    w->FlushThreshold = 0;
    write_ok(*w, B("456"));
    CHECK(buf.b == H("80100a03343536"));
}

static void TestRunlenDecoder() {  // eazy_test.go:581-597
    Buffer src;
    src.b = H("8010048008000161" "85ff01" "026263" "85ff02" "027878");
    auto r = NewReader(&src);
    CHECK(rd(*r, 1000) == std::make_pair(B("aaaaaabcbcbcbxx"), Err::EOF_));
}

static void TestRunlenEncoder() {  // eazy_test.go:599-670
    Buffer buf;
    auto w = NewWriter(&buf, 128, 16);
    write_ok(*w, Bytes{0});
    size_t off = buf.b.size();
    write_ok(*w, B("aaaaaaabcbcbcbcbxx"));
    CHECK(sub(buf.b, off) == H("016186ff0102626387ff02027878"));
    Bytes data(0x1005, '0');
    off = buf.b.size();
    write_ok(*w, data);
    CHECK(sub(buf.b, off) == H("0130fd880eff01"));
    for (size_t k = 3; k < data.size(); k++) data[k] = 0;
    off = buf.b.size();
    write_ok(*w, data);
    CHECK(sub(buf.b, off) == H("03303030fd860eff00"));
}

static void TestUnsupportedVersion() {  // eazy_test.go:749-762
    Buffer buf;
    auto w = NewWriter(&buf, 1024, 32);
    w->Ver = 1;
    w->Write(Bytes{1, 2});
    auto r = NewReaderBytes(buf.b);
    auto [got, err] = rd(*r, 1);
    CHECK(err == Err::UnsupportedVersion && got.empty());
    CHECK(ErrorText(err, r->Detail) == "unsupported file format version: 1");
}

struct FailingSink : IoWriter {  // accepts `accept` bytes once, then fails
    Buffer *dst;
    long accept = -1;
    std::pair<size_t, Err> Write(const uint8_t *p, size_t n) override {
        if (accept < 0) return dst->Write(p, n);
        const size_t k = std::min(n, (size_t)accept);
        dst->Write(p, k);
        accept = -1;
        return {k, Err::Sink};
    }
};

static void TestSinkFailureResets() {  // writer.go:387-401
    Buffer buf;
    FailingSink s;
    s.dst = &buf;
    auto w = NewWriter(&s, 1024, 32);
    write_ok(*w, B("first message, first message"));
    const size_t good = buf.b.size();
    s.accept = 3;
    auto [n, e] = w->Write(B("second message"));
    CHECK(e == Err::Sink && n == 0);
    CHECK(buf.b.size() == good + 3);
    const size_t st = buf.b.size();
    write_ok(*w, B("third message"));
    CHECK(sub(buf.b, st, st + 6) == H("800265617a79"));  // a fresh stream with its header
}

static void TestBatchMatchesWriter() {  // the GPU batch path == one NewWriter(MiB,1024).Write per stream
    std::vector<Bytes> streams;
    for (int s = 0; s < 40; s++) {
        Bytes p;
        for (int k = 0; k < 300 + 97 * s; k++) p.push_back((uint8_t)("level=info path=/api/v1/items "[(k * 7 + s) % 31] ^ (k % 53 == 0 ? s : 0)));
        streams.push_back(p);
    }
    std::vector<uint64_t> in_off{0}, out_off{0};
    Bytes in;
    for (auto &p : streams) {
        in.insert(in.end(), p.begin(), p.end());
        in_off.push_back(in.size());
        out_off.push_back(out_off.back() + ez_compress_bound(p.size()));
    }
    const size_t count = streams.size();
    uint8_t *d_in, *d_out;
    uint64_t *d_in_off, *d_out_off, *d_size;
    int32_t *d_status;
    CHECK(hipMalloc(&d_in, in.size() + 16) == hipSuccess);
    CHECK(hipMalloc(&d_out, out_off.back() + 16) == hipSuccess);
    CHECK(hipMalloc(&d_in_off, 8 * (count + 1)) == hipSuccess);
    CHECK(hipMalloc(&d_out_off, 8 * (count + 1)) == hipSuccess);
    CHECK(hipMalloc(&d_size, 8 * count) == hipSuccess);
    CHECK(hipMalloc(&d_status, 4 * count) == hipSuccess);
    (void)hipMemcpy(d_in, in.data(), in.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_in_off, in_off.data(), 8 * (count + 1), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_out_off, out_off.data(), 8 * (count + 1), hipMemcpyHostToDevice);
    ez_batch b{d_in, d_in_off, d_out, d_out_off, d_size, d_status, count, 0};
    CHECK(CompressBatch(MiB, 1024, true, b, nullptr) == Err::OK);
    CHECK(hipDeviceSynchronize() == hipSuccess);
    Bytes out(out_off.back());
    std::vector<uint64_t> size(count);
    std::vector<int32_t> status(count);
    (void)hipMemcpy(out.data(), d_out, out.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(size.data(), d_size, 8 * count, hipMemcpyDeviceToHost);
    (void)hipMemcpy(status.data(), d_status, 4 * count, hipMemcpyDeviceToHost);
    for (size_t s = 0; s < count; s++) {
        Buffer buf;
        auto w = NewWriter(&buf, MiB, 1024);
        write_ok(*w, streams[s]);
        CHECK(status[s] == 0);
        CHECK(sub(out, out_off[s], out_off[s] + size[s]) == buf.b);
    }
    for (void *p : {(void *)d_in, (void *)d_out, (void *)d_in_off, (void *)d_out_off, (void *)d_size, (void *)d_status}) (void)hipFree(p);
}

struct Recorder : IoWriter {  // an io.Writer keeping every call's bytes
    std::vector<Bytes> calls;
    std::pair<size_t, Err> Write(const uint8_t *p, size_t n) override {
        calls.emplace_back(p, p + n);
        return {n, Err::OK};
    }
};

// Batches over a device list (ez_compress_batch_multi / ez_decompress_batch_multi through the C++
// mirror): two shards on the one card ({0, 0}), three, and every device, each equal to one
// NewWriter(MiB, 1024).Write per stream, and the streams decode back.
static void TestBatchMulti() {
    std::vector<Bytes> streams;
    for (int s = 0; s < 57; s++) {
        Bytes p;
        for (int k = 0; k < (s % 9 == 0 ? 0 : 200 + 131 * s); k++)
            p.push_back((uint8_t)("level=warn ip=10.0.3.7 path=/api/v2/users "[(k * 5 + s) % 41] ^ (k % 61 == 0 ? s : 0)));
        streams.push_back(p);
    }
    std::vector<Bytes> want;
    for (auto &p : streams) {
        Buffer buf;
        auto w = NewWriter(&buf, MiB, 1024);
        if (!p.empty()) write_ok(*w, p);
        else {
            auto [n, err] = w->Write(p.data(), 0);
            CHECK(n == 0 && err == Err::OK);
        }
        want.push_back(buf.b);
    }
    for (const std::vector<int> &devs : {std::vector<int>{0, 0}, std::vector<int>{0, 0, 0}, std::vector<int>{}}) {
        std::vector<std::vector<uint8_t>> got;
        CHECK(CompressBatchMulti(streams, MiB, 1024, got, devs) == Err::OK);
        CHECK(got == want);
        std::vector<uint64_t> slots;
        for (auto &p : streams) slots.push_back(p.size());
        std::vector<std::pair<std::vector<uint8_t>, Err>> dec;
        CHECK(DecompressBatchMulti(got, slots, dec, devs) == Err::OK);
        for (size_t k = 0; k < streams.size(); k++) CHECK(dec[k].second == Err::OK && dec[k].first == streams[k]);
    }
}

static void TestWriteBatch() {  // Writer::WriteBatch == Write on each in turn (same sink calls)
    Bytes data;
    std::vector<uint64_t> ends;
    for (int j = 0; j < 120; j++) {
        const int n = (j * 37) % 200;
        for (int k = 0; k < n; k++) data.push_back((uint8_t)("ts=1 level=warn msg=\"disk\" "[(k * 3 + j) % 29]));
        ends.push_back(data.size());
    }
    for (int thr : {0, 100, -1}) {
        Recorder a, b;
        auto wa = NewWriter(&a, 2048, 64), wb = NewWriter(&b, 2048, 64);
        wa->FlushThreshold = wb->FlushThreshold = thr;
        for (size_t j = 0; j < ends.size(); j++) write_ok(*wa, sub(data, j ? ends[j - 1] : 0, ends[j]));
        for (size_t j = 0; j < ends.size(); j += 30) {  // batches of 30 Writes
            std::vector<uint64_t> e;
            const uint64_t base = j ? ends[j - 1] : 0;
            for (size_t q = j; q < j + 30; q++) e.push_back(ends[q] - base);
            auto [n, err] = wb->WriteBatch(data.data() + base, e.data(), e.size());
            CHECK(err == Err::OK && n == e.back());
        }
        CHECK(wa->Flush() == Err::OK && wb->Flush() == Err::OK);
        CHECK(a.calls == b.calls);
    }
}

// Handles that are created and dropped give their device memory back: a drop-in caller never
// closes a Writer or Reader (the reference has nothing to close), so the destructor must free
// the ring, the table, the HIP stream and the staging buffers.
static size_t device_free() {
    size_t fr = 0, tot = 0;
    CHECK(hipMemGetInfo(&fr, &tot) == hipSuccess);
    return fr;
}
static void TestHandleLeak() {
    Bytes p;
    for (int k = 0; k < 4096; k++) p.push_back((uint8_t)("ts=2 level=info msg=\"ok\" "[(k * 5) % 27]));
    {  // warm: the first handles initialise the runtime and the kernels' one-time probes
        Buffer buf;
        auto w = NewWriter(&buf, MiB, 1024);
        write_ok(*w, p);
        auto r = NewReaderBytes(buf.b);
        (void)r->Read(p.size());
    }
    CHECK(hipDeviceSynchronize() == hipSuccess);
    const size_t base = device_free();
    for (int round = 0; round < 64; round++) {
        Buffer buf;
        auto w = NewWriter(&buf, 4 * MiB, 4096);  // a 4 MiB ring and a 16 KiB table per handle
        write_ok(*w, p);
        auto r = NewReaderBytes(buf.b);
        auto [out, e] = r->Read(p.size());
        CHECK(out == p);
    }
    CHECK(hipDeviceSynchronize() == hipSuccess);
    const size_t after = device_free();
    // 64 leaked Writers would hold >= 256 MiB; allow the allocator's slack (a few MiB)
    std::printf("    device free: %zu -> %zu MiB\n", base >> 20, after >> 20);
    CHECK(after + (16u << 20) >= base);
}

struct Chunked : IoReader {  // an io.Reader returning at most `step` bytes per call
    Bytes b;
    size_t at = 0, step = 1;
    std::pair<size_t, Err> Read(uint8_t *p, size_t n) override {
        if (at >= b.size()) return {0, Err::EOF_};
        size_t k = std::min({n, step, b.size() - at});
        std::memcpy(p, b.data() + at, k);
        at += k;
        return {k, Err::OK};
    }
};

// --dump FILE: for every hex-encoded stream in FILE (one per line) its Dump, then what
// Dumper::ReadFrom prints from reads of 7 bytes and the error it ends with, each followed by a
// line "----": tests/test_cpp.py compares them with eazy_amd/dump.py (host only)
static int dump_file(const char *path) {
    FILE *f = std::fopen(path, "r");
    if (!f) return 2;
    std::string line;
    int c;
    for (;;) {
        line.clear();
        while ((c = std::fgetc(f)) != EOF && c != '\n') line += (char)c;
        if (!line.empty()) {
            std::printf("%s\n----\n", Dump(H(line)).c_str());
            Buffer text;
            auto d = NewDumper(&text);
            Chunked r;
            r.b = H(line);
            r.step = 7;
            auto [tot, err] = d->ReadFrom(&r);
            std::printf("%s|%lld|%s\n----\n", std::string(text.b.begin(), text.b.end()).c_str(), (long long)tot, ez_strerror((int)err));
        }
        if (c == EOF) break;
    }
    std::fclose(f);
    return 0;
}

// --perf-reader COMP PLAIN READ: NewReaderBytes(COMP) read to EOF with Read(READ bytes) through the
// C++ mirror (the drop-in path without Python), checked against PLAIN; prints the rate and the time
// of the first Read (the whole-stream decode)
static std::vector<uint8_t> read_file(const char *path) {
    std::vector<uint8_t> b;
    FILE *f = std::fopen(path, "rb");
    if (!f) return b;
    uint8_t tmp[1 << 16];
    size_t k;
    while ((k = std::fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + k);
    std::fclose(f);
    return b;
}
static int perf_reader(const char *comp_path, const char *plain_path, size_t rs, int whole) {
    const std::vector<uint8_t> comp = read_file(comp_path), plain = read_file(plain_path);
    std::vector<uint8_t> got(plain.size() + rs), p(rs);
    {  // (once per process: the HIP runtime's start and the device's decode workspace, by a first Reader
        // over the same stream; the timed one is a fresh handle)
        auto w = NewReaderBytes(comp);
        std::vector<uint8_t> q(4096);
        (void)w->Read(q.data(), q.size());
    }
    const auto t0 = std::chrono::steady_clock::now();
    auto r = NewReaderBytes(comp);
    if (!whole) ez_reader_set_whole(r->Handle(), 0);
    size_t at = 0;
    double first = -1;
    Err e = Err::OK;
    for (;;) {
        auto [n, err] = r->Read(p.data(), rs);
        if (first < 0) first = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (at + n > got.size()) return 3;
        std::memcpy(got.data() + at, p.data(), n);
        at += n;
        e = err;
        if (err != Err::OK) break;
    }
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const bool ok = e == Err::EOF_ && at == plain.size() && std::memcmp(got.data(), plain.data(), at) == 0;
    std::printf("{\"reader\": \"%s\", \"read_bytes\": %zu, \"MiBps\": %.1f, \"first_read_ms\": %.2f, \"ok\": %s}\n",
                whole ? "whole" : "read_by_read", rs, (double)at / t / 1048576.0, first * 1e3, ok ? "true" : "false");
    return ok ? 0 : 1;
}

// --perf-stream COMP PLAIN READ PIECE: NewReader over an io.Reader that returns PIECE bytes per call
// (the README's usage, reader.go:79-86), read to EOF with Read(READ bytes) through the C++ mirror;
// checked against PLAIN; prints the rate and the handle's read-ahead count
static int perf_stream(const char *comp_path, const char *plain_path, size_t rs, size_t piece) {
    const std::vector<uint8_t> comp = read_file(comp_path), plain = read_file(plain_path);
    std::vector<uint8_t> got(plain.size() + rs), p(rs);
    {  // (once per process: the HIP runtime's start and the device's decode workspace)
        Chunked warm;
        warm.b = comp;
        warm.step = piece;
        auto w = NewReader(&warm);
        for (int k = 0; k < 64; k++) (void)w->Read(p.data(), rs);
    }
    Chunked src;
    src.b = comp;
    src.step = piece;
    const auto t0 = std::chrono::steady_clock::now();
    auto r = NewReader(&src);
    size_t at = 0;
    Err e = Err::OK;
    for (;;) {
        auto [n, err] = r->Read(p.data(), rs);
        if (at + n > got.size()) return 3;
        std::memcpy(got.data() + at, p.data(), n);
        at += n;
        e = err;
        if (err != Err::OK) break;
    }
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const bool ok = e == Err::EOF_ && at == plain.size() && std::memcmp(got.data(), plain.data(), at) == 0;
    std::printf("{\"reader\": \"stream\", \"read_bytes\": %zu, \"piece\": %zu, \"MiBps\": %.1f, \"read_aheads\": %lld, \"ok\": %s}\n", rs,
                piece, (double)at / t / 1048576.0, (long long)ez_reader_ahead_count(r->Handle()), ok ? "true" : "false");
    return ok ? 0 : 1;
}

// --reader-ahead: a 3 MiB log-like stream written by the mirror's Writer, read back through
// NewReader(io.Reader) in 64 KiB pieces with Read(4096) and in 9,000-byte pieces with Read(777): the
// bytes equal the input and the handle read ahead
static int reader_ahead_test() {
    Bytes plain;
    uint32_t x = 12345;
    const char *words[] = {"GET /api/v1/items ", "status=200 ", "user=alice ", "latency_ms=", "trace=", "INFO ", "WARN ", "\n"};
    while (plain.size() < (3u << 20)) {
        x = x * 1103515245u + 12345u;
        const char *wd = words[(x >> 16) % 8];
        plain.insert(plain.end(), wd, wd + std::strlen(wd));
        const std::string num = std::to_string((x >> 8) % 100000);
        plain.insert(plain.end(), num.begin(), num.end());
    }
    Buffer buf;
    auto w = NewWriter(&buf, MiB, 1024);
    for (size_t at = 0; at < plain.size(); at += 65536) {
        const size_t n = std::min((size_t)65536, plain.size() - at);
        auto [k, err] = w->Write(plain.data() + at, n);
        if (err != Err::OK || k != n) return 2;
    }
    for (auto [piece, rs] : {std::pair<size_t, size_t>{65536, 4096}, {9000, 777}}) {
        Chunked src;
        src.b = buf.b;
        src.step = piece;
        auto r = NewReader(&src);
        Bytes got, p(rs);
        Err e = Err::OK;
        for (;;) {
            auto [n, err] = r->Read(p.data(), rs);
            got.insert(got.end(), p.begin(), p.begin() + (ptrdiff_t)n);
            e = err;
            if (err != Err::OK) break;
        }
        const long long ra = (long long)ez_reader_ahead_count(r->Handle());
        std::printf("piece %zu read %zu: %zu bytes, %s, read-aheads %lld\n", piece, rs, got.size(), ez_strerror((int)e), ra);
        if (e != Err::EOF_ || got != plain || ra <= 0) return 1;
    }
    std::printf("ok\n");
    return 0;
}

// Dumper::ReadFrom with the stream in one read prints what one Write prints, and a stream cut
// inside a token ends in UnexpectedEOF (reader.go:563-600).  (Reads that cut a token do not
// print what Dump prints: like the reference, Write reports the bytes up to the cut token's
// tag as taken; the comparison with the Python mirror covers that case.)
static void TestDumperReadFrom() {
    Bytes s = H("8003");  // (a meta header is not needed: the Dumper prints what it is given)
    Encoder e;
    s.clear();
    e.MetaTag(s, MetaMagic, 4);
    s = cat(s, B("eazy"));
    e.MetaTag(s, MetaReset, 1);
    s.push_back(20);
    e.Tag(s, Literal, 5);
    s = cat(s, B("hello"));
    e.Tag(s, Copy, 10);
    e.Offset(s, 5, 10);
    s.push_back(0);
    s.push_back(0);
    e.Tag(s, Literal, 130);
    for (int k = 0; k < 130; k++) s.push_back((uint8_t)(k * 7));
    Dumper whole;
    whole.GlobalOffset = -1;
    CHECK(whole.Write(s).second == Err::OK);
    for (size_t step : {s.size(), (size_t)4096}) {
        Buffer text;
        auto d = NewDumper(&text);
        d->GlobalOffset = -1;
        Chunked r;
        r.b = s;
        r.step = step;
        auto [tot, err] = d->ReadFrom(&r);
        CHECK(err == Err::OK && tot == (int64_t)s.size());
        CHECK(std::string(text.b.begin(), text.b.end()) == whole.Text());
    }
    Chunked cut;
    cut.b = sub(s, 0, s.size() - 3);
    cut.step = cut.b.size();
    Buffer sink;
    auto d = NewDumper(&sink);
    CHECK(d->ReadFrom(&cut).second == Err::UnexpectedEOF);
    CHECK(Dump(sub(s, 0, s.size() - 3)).find("\nerror: short buffer") != std::string::npos);
}

int main(int argc, char **argv) {
    if (argc > 2 && std::string(argv[1]) == "--dump") return dump_file(argv[2]);
    if (argc > 5 && std::string(argv[1]) == "--perf-reader") return perf_reader(argv[2], argv[3], (size_t)std::atol(argv[4]), std::atoi(argv[5]));
    if (argc > 5 && std::string(argv[1]) == "--perf-stream") return perf_stream(argv[2], argv[3], (size_t)std::atol(argv[4]), (size_t)std::atol(argv[5]));
    if (argc > 1 && std::string(argv[1]) == "--reader-ahead") return reader_ahead_test();
    const bool cpu = argc > 1 && std::string(argv[1]) == "--cpu";
    run("TestPrintLengthEncoding", TestPrintLengthEncoding);
    run("TestPrintOffsetEncoding", TestPrintOffsetEncoding);
    run("TestReaderShortBuffer", TestReaderShortBuffer);
    run("TestEncoderPanics", TestEncoderPanics);
    run("TestErrorText", TestErrorText);
    run("TestCompressBound", TestCompressBound);
    run("TestDumperReadFrom", TestDumperReadFrom);
    if (!cpu) {
        if (ez_device_count() <= 0) {
            std::printf("FAIL no MI355X visible\n");
            return 2;
        }
        run("TestMagic", TestMagic);
        run("TestLiteral", TestLiteral);
        run("TestCopy", TestCopy);
        run("TestBug1", TestBug1);
        run("TestPadding", TestPadding);
        run("TestZeroRegion", TestZeroRegion);
        run("TestBreak", TestBreak);
        run("TestReaderRequireMagic", TestReaderRequireMagic);
        run("TestFlush", TestFlush);
        run("TestFlushReset", TestFlushReset);
        run("TestRunlenDecoder", TestRunlenDecoder);
        run("TestRunlenEncoder", TestRunlenEncoder);
        run("TestUnsupportedVersion", TestUnsupportedVersion);
        run("TestSinkFailureResets", TestSinkFailureResets);
        run("TestBatchMatchesWriter", TestBatchMatchesWriter);
        run("TestWriteBatch", TestWriteBatch);
        run("TestHandleLeak", TestHandleLeak);
        run("TestBatchMulti", TestBatchMulti);
    }
    std::printf("%d/%d passed\n", g_run - g_fail, g_run);
    return g_fail ? 1 : 0;
}
