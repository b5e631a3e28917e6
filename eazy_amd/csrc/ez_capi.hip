// ez_capi.hip — implementation of include/eazy.h over the gfx950 kernels.
//
// Host-side responsibilities only: argument validation (the reference's
// panics), HBM buffer management for the streaming handles, H2D/D2H of the
// handles' per-call data, and kernel launches.  All compression and
// decompression runs in K1/K2/K3; there is no CPU code path for them.
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <algorithm>
#include <vector>
#include <memory>
#include <thread>
#include <chrono>

#include "ez_cache.h"
#include "ez_format.h"
#include "ez_internal.h"

namespace {

int g_device_count = -1;
std::mutex g_mu;

int device_count() {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_device_count < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        g_device_count = n;
    }
    return g_device_count;
}

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (device_count() <= 0) return;
        if (hipGetDevice(&prev) != hipSuccess) return;
        if (dev >= 0 && dev != prev && hipSetDevice(dev) != hipSuccess) return;
        ok = true;
    }
    ~DeviceGuard() {
        if (ok && prev >= 0) (void)hipSetDevice(prev);
    }
};

#define EZ_HIP(x)                                   \
    do {                                            \
        if ((x) != hipSuccess) return EZ_EDEVICE;   \
    } while (0)

// grow-only device buffer
struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return EZ_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = n < 4096 ? 4096 : n + n / 4;
        if (hipMalloc(&p, c) != hipSuccess) return EZ_EDEVICE;
        cap = c;
        return EZ_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const { return (T *)p; }
};

bool pow2(int64_t x) { return x > 0 && (x & (x - 1)) == 0; }

// Writer.init size checks (writer.go:161-169)
bool valid_writer_sizes(int64_t bs, int64_t hs) {
    if (!pow2(bs) || bs < 32 || bs > ((int64_t)1 << 31)) return false;
    if (!pow2(hs) || hs < 4) return false;
    return true;
}

// appendHeader writer.go:495-517
size_t header_bytes(uint8_t *b, int append_magic, int ver, int64_t bs) {
    size_t k = 0;
    if (append_magic) {
        const uint8_t m[6] = {0x80, 0x02, 'e', 'a', 'z', 'y'};
        memcpy(b, m, 6);
        k = 6;
    }
    if (ver != 0) {
        b[k++] = 0x80; b[k++] = 0x08; b[k++] = (uint8_t)ver;
    }
    b[k++] = 0x80; b[k++] = 0x10; b[k++] = (uint8_t)__builtin_ctzll((uint64_t)bs);
    return k;
}

// K1 scratch (match records / global hash tables / K1c's logs), one per (device, HIP stream), each
// locked only by the call using it: batch calls on distinct streams run concurrently (SURVEY §8b
// threading; ez_cache.h)
ez::DevCache &k1_cache() {
    static ez::DevCache *c = new ez::DevCache();  // (never destroyed: no hipFree after the runtime's teardown)
    return *c;
}

}  // namespace

// ------------------------------------------------------------------ misc

extern "C" const char *ez_strerror(int code) {
    switch (code) {
    case EZ_OK: return "ok";
    case EZ_EOF: return "EOF";
    case EZ_ESHORTBUF: return "short buffer";
    case EZ_EUNEXPECTEDEOF: return "unexpected EOF";
    case EZ_EOVERFLOW: return "length/offset overflow";
    case EZ_EBADMAGIC: return "bad magic";
    case EZ_ENOMAGIC: return "no magic";
    case EZ_EBLOCKLIMIT: return "block size is more than the limit";
    case EZ_EUNSUPMETA: return "unsupported meta tag";
    case EZ_EUNSUPVER: return "unsupported file format version";
    case EZ_EBREAK: return "break point";
    case EZ_EMISSEDMETA: return "missed meta";
    case EZ_EINVAL: return "invalid argument (reference panic)";
    case EZ_ESINK: return "underlying writer failed";
    case EZ_ENOSPC: return "output buffer too small";
    case EZ_EDEVICE: return "no usable MI355X device / HIP error";
    case EZ_ESTUCK: return "kernel progress guard tripped";
    default: return "unknown error";
    }
}

// the value each reference panic carries (writer.go:163, 167, 309/596, 562, 601)
extern "C" const char *ez_panic_message(int panic) {
    switch (panic) {
    case EZ_PANIC_BLOCK: return "block size must be a power of two (32 < bs < 1<<31)";
    case EZ_PANIC_HTABLE: return "hash table size must be a power of two (hs >= 4)";
    case EZ_PANIC_LENGTH: return "too big length";
    case EZ_PANIC_OFFSET: return "too big offset";
    case EZ_PANIC_META: return "meta";  // Go panics with the meta value itself (an int)
    default: return "";
    }
}

// Writer.init writer.go:161-169: the block check comes first
extern "C" int ez_writer_size_panic(int64_t block, int64_t htable) {
    if (((block - 1) & block) != 0 || block < 32 || block > ((int64_t)1 << 31)) return EZ_PANIC_BLOCK;
    if (((htable - 1) & htable) != 0 || htable < 4) return EZ_PANIC_HTABLE;
    return EZ_PANIC_NONE;
}

extern "C" int ez_abi_version(void) { return EZ_ABI_VERSION; }

#ifdef EZ_KNOBS
namespace ez {
const char *knob_str(const char *name) { return getenv(name); }
int knob(const char *name, int dflt) {
    const char *v = getenv(name);
    return v ? atoi(v) : dflt;
}
}  // namespace ez
#endif
extern "C" int ez_device_count(void) { return device_count(); }

// ------------------------------------------------------------------ token codec

extern "C" int ez_encode_tag(uint8_t *b, size_t cap, size_t *len, int tag, int64_t l) {
    uint8_t t[16];
    const int k = ez::enc_tag(t, tag, l);
    if (k < 0) return EZ_EINVAL;
    if (*len + (size_t)k > cap) return EZ_ENOSPC;
    memcpy(b + *len, t, (size_t)k);
    *len += (size_t)k;
    return EZ_OK;
}

extern "C" int ez_encode_offset(uint8_t *b, size_t cap, size_t *len, int64_t off, int64_t l) {
    uint8_t t[16];
    const int k = ez::enc_offset(t, off, l);
    if (k < 0) return EZ_EINVAL;
    if (*len + (size_t)k > cap) return EZ_ENOSPC;
    memcpy(b + *len, t, (size_t)k);
    *len += (size_t)k;
    return EZ_OK;
}

extern "C" int ez_encode_meta(uint8_t *b, size_t cap, size_t *len, int64_t meta, int64_t l) {
    uint8_t t[16];
    const int k = ez::enc_meta(t, meta, l);
    if (k < 0) return EZ_EINVAL;
    if (*len + (size_t)k > cap) return EZ_ENOSPC;
    memcpy(b + *len, t, (size_t)k);
    *len += (size_t)k;
    return EZ_OK;
}

extern "C" int ez_decode_tag(const uint8_t *b, size_t n, size_t st, int *tag, int64_t *l, size_t *i) {
    int64_t j;
    const int e = ez::dec_tag(b, (int64_t)n, (int64_t)st, tag, l, &j);
    *i = (size_t)j;
    return e;
}

extern "C" int ez_decode_offset(const uint8_t *b, size_t n, size_t st, int64_t l, int64_t *off, size_t *i) {
    int64_t j;
    const int e = ez::dec_offset(b, (int64_t)n, (int64_t)st, l, off, &j);
    *i = (size_t)j;
    return e;
}

extern "C" int ez_decode_meta(const uint8_t *b, size_t n, size_t st, int64_t *meta, int64_t *l, size_t *i) {
    int64_t j;
    const int e = ez::dec_meta(b, (int64_t)n, (int64_t)st, meta, l, &j);
    *i = (size_t)j;
    return e;
}

extern "C" size_t ez_compress_bound(size_t n) { return (size_t)ez::compress_bound(n); }

// ------------------------------------------------------------------ Writer handle

// pinned host staging (one copy each way per call, no pageable bounce)
struct HBuf {
    void *p = nullptr;
    size_t cap = 0;
    unsigned flags = hipHostMallocDefault;  // (a Writer's: coherent, the kernels read and write it in place)
    int ensure(size_t n) {
        if (n <= cap) return EZ_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t c = n < 65536 ? 65536 : n + n / 4;
        if (hipHostMalloc(&p, c, flags) != hipSuccess) return EZ_EDEVICE;
        cap = c;
        return EZ_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const { return (T *)p; }
};

struct ez_writer {
    int device = 0;
    int64_t bs = 0, hs = 0;
    int append_magic = 1;
    int ver = 0;
    bool pristine = true;  // isreset(): nothing emitted since the last reset
    // the device's ring and table may hold a Write that failed and was not reset (writer_zero itself
    // failed): the next call resets them first, and fails until that works
    bool tainted = false;
    int64_t pos = 0;       // w.pos
    int last_panic = EZ_PANIC_NONE;  // the reference panic behind the last EZ_EINVAL
    // dev: [input | in_off[2] out_off[2] out_size status write_idx[2] | write_end[k] | write_out[k] | output]
    DBuf ring, ht, dev;
    DBuf recs;             // K1L's match records (single Writes, ez::long_ring_applies)
    HBuf host;             // the same layout, pinned
    uint8_t *host_dev = nullptr;  // the device's address of `host` (zero-copy Writes), or nullptr
    void *host_alias_of = nullptr;  // the host.p host_dev was taken for
    uint32_t seq = 0;               // the zero-copy path's completion flag value of the last Write
    hipStream_t stream = nullptr;
};

namespace {

int writer_zero(ez_writer *w) {
    EZ_HIP(hipMemsetAsync(w->ring.p, 0, (size_t)w->bs, w->stream));
    EZ_HIP(hipMemsetAsync(w->ht.p, 0, (size_t)w->hs * 4, w->stream));
    EZ_HIP(hipStreamSynchronize(w->stream));
    w->pos = 0;
    w->pristine = true;
    w->tainted = false;
    return EZ_OK;
}

// a call that changes the device history starts from a clean one
int writer_clean(ez_writer *w) { return w->tainted ? writer_zero(w) : EZ_OK; }

int writer_alloc(ez_writer *w, int64_t bs, int64_t hs) {
    if (w->ring.ensure((size_t)bs)) return EZ_EDEVICE;
    if (w->ht.ensure((size_t)hs * 4)) return EZ_EDEVICE;
    w->bs = bs;
    w->hs = hs;
    return EZ_OK;
}

}  // namespace

extern "C" int ez_writer_new(int64_t block, int64_t htable, int device, ez_writer **out) {
    *out = nullptr;
    if (!valid_writer_sizes(block, htable)) return EZ_EINVAL;
    DeviceGuard g(device);
    if (!g.ok) return EZ_EDEVICE;
    ez_writer *w = new ez_writer();
    w->device = device;
    w->host.flags = hipHostMallocCoherent;
    if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess) {
        delete w;
        return EZ_EDEVICE;
    }
    int e = writer_alloc(w, block, htable);
    if (!e) e = writer_zero(w);
    if (e) {
        ez_writer_free(w);
        return e;
    }
    *out = w;
    return EZ_OK;
}

extern "C" void ez_writer_free(ez_writer *w) {
    if (!w) return;
    DeviceGuard g(w->device);
    w->ring.release();
    w->ht.release();
    w->dev.release();
    w->recs.release();
    w->host.release();
    if (w->stream) (void)hipStreamDestroy(w->stream);
    delete w;
}

extern "C" int ez_writer_set_append_magic(ez_writer *w, int on) {
    w->append_magic = on ? 1 : 0;
    return EZ_OK;
}

extern "C" int ez_writer_set_version(ez_writer *w, int ver) {
    w->ver = ver;
    return EZ_OK;
}

extern "C" int ez_writer_is_reset(const ez_writer *w) { return w->pristine || w->tainted ? 1 : 0; }

extern "C" int ez_writer_last_panic(const ez_writer *w) { return w->last_panic; }

// testing hook: w.pos of a handle, ring and table unchanged (positions past 2^32)
extern "C" int ez_writer_set_position(ez_writer *w, int64_t pos) {
    if (pos < 0) return EZ_EINVAL;
    w->pos = pos;
    return EZ_OK;
}

namespace {

// k Writes on the handle in one launch (k = 1: Writer.Write; k > 1: the same Writes in turn):
// p holds them back to back, Write j ending at p[ends[j]]; out receives what each appends to
// w.b, Write j's bytes ending at out[out_ends[j]].  One host->device copy (the Writes and the
// launch metadata, from pinned staging), the general kernel with the handle's ring and table,
// one device->host copy (status, sizes and bytes), one synchronisation.
// The handle's args for Write j of k (K1L path): stream position, header on a pristine stream's first
ez::CompressArgs long_args(const ez_writer *w, uint8_t *D, uint64_t *dm, size_t j, uint64_t len, int64_t start) {
    ez::CompressArgs a{};
    a.in = D;
    a.in_off = dm;
    a.out = D;
    a.out_off = dm + 2;
    a.out_size = dm + 4;
    a.status = (int32_t *)(dm + 5);
    a.count = 1;
    a.bs = w->bs;
    a.hs = w->hs;
    a.append_magic = w->append_magic;
    a.ver = w->ver;
    a.header = w->pristine && j == 0 ? 1 : 0;
    a.start = start;
    a.ring = w->ring.as<uint8_t>();
    a.ht_global = w->ht.as<uint32_t>();
    a.max_len = len;
    return a;
}

// k Writes (k >= 1) through K1L on the handle's ring and table, one after another on the handle's
// HIP stream (the parse, the token writer and the ring update of each, no host round trip between
// them): one host->device copy, one device->host copy and one synchronisation for all of them.
// Returns -1 when a Write does not qualify (ez::long_ring_applies): the caller takes the general kernel.
int writer_run_long(ez_writer *w, const uint8_t *p, const uint64_t *ends, size_t k, uint8_t *out, size_t cap, uint64_t *out_ends,
                    size_t bound) {
    if (ez::compress_forced_general()) return -1;
    DeviceGuard g(w->device);
    if (!g.ok) return EZ_EDEVICE;
    const size_t n = (size_t)ends[k - 1];
    uint64_t recmax = 0;
    for (size_t j = 0; j < k; j++) {
        const uint64_t len = ends[j] - (j ? ends[j - 1] : 0);
        const ez::CompressArgs a = long_args(w, nullptr, nullptr, j, len, w->pos + (int64_t)(j ? ends[j - 1] : 0));
        if (!ez::long_ring_applies(a)) return -1;
        const uint64_t r = ez::long_ring_scratch_bytes(a);
        recmax = r > recmax ? r : recmax;
    }
    // [input | per Write: in_off[2] out_off[2] out_size status | outputs, Write j's at its bound prefix]
    const size_t o_meta = (n + 15) & ~(size_t)15;
    const size_t o_o = (o_meta + 6 * 8 * k + 15) & ~(size_t)15;
    const size_t o_flag = (o_o + bound + 16 + 63) & ~(size_t)63;  // the completion flag (zero-copy path)
    const size_t total = o_flag + 64;
    // Writes K1L stages in LDS (read once): the kernels read them, and write the output, in the pinned
    // host buffer itself -- no host->device and device->host copies (a 100-byte Write's fixed cost)
    bool zc = true;
    for (size_t j = 0; j < k; j++) zc = zc && ends[j] - (j ? ends[j - 1] : 0) <= ez::kHandleLdsWrite;
    if (w->host.ensure(total) || w->recs.ensure((size_t)recmax)) return EZ_EDEVICE;
    if (zc && w->host_alias_of != w->host.p) {  // the device's address of the pinned buffer
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, w->host.p, 0) != hipSuccess) {
            (void)hipGetLastError();
            dp = nullptr;
        }
        w->host_dev = (uint8_t *)dp;
        w->host_alias_of = w->host.p;
    }
    zc = zc && w->host_dev != nullptr;
    if (!zc && w->dev.ensure(total)) return EZ_EDEVICE;
    uint8_t *H = w->host.as<uint8_t>(), *D = zc ? w->host_dev : w->dev.as<uint8_t>();
    memcpy(H, p, n);
    uint64_t *m = (uint64_t *)(H + o_meta);
    size_t boff = 0;
    for (size_t j = 0; j < k; j++) {
        const uint64_t len = ends[j] - (j ? ends[j - 1] : 0);
        const size_t b = ez_compress_bound((size_t)len);
        uint64_t *mj = m + 6 * j;
        mj[0] = j ? ends[j - 1] : 0;
        mj[1] = ends[j];
        mj[2] = o_o + boff;
        mj[3] = o_o + boff + b;
        mj[4] = 0;
        mj[5] = 0;
        boff += b;
    }
    if (!zc) EZ_HIP(hipMemcpyAsync(D, H, o_meta + 6 * 8 * k, hipMemcpyHostToDevice, w->stream));
    w->tainted = true;  // (cleared when the call completes, or by the reset of a failed one)
    hipError_t he = hipSuccess;
    volatile uint32_t *flag = (volatile uint32_t *)(H + o_flag);
    const uint32_t seq = ++w->seq;
    *flag = seq + 1;  // (not the value this call waits for, whatever the buffer held)
    for (size_t j = 0; j < k && he == hipSuccess; j++) {
        const uint64_t len = ends[j] - (j ? ends[j - 1] : 0);
        ez::CompressArgs a = long_args(w, D, (uint64_t *)(D + o_meta) + 6 * j, j, len, w->pos + (int64_t)(j ? ends[j - 1] : 0));
        if (zc && j + 1 == k) {  // the last Write's kernel signals its end in the pinned buffer
            a.done_flag = (uint32_t *)(D + o_flag);
            a.done_seq = seq;
        }
        he = ez::launch_long_ring(a, w->recs.as<uint8_t>(), w->stream);
    }
    if (he == hipSuccess && !zc) he = hipMemcpyAsync(H + o_meta, D + o_meta, o_o - o_meta + bound, hipMemcpyDeviceToHost, w->stream);
    bool seen = false;
    if (he == hipSuccess && zc) {
        // wait by polling the flag (a few microseconds sooner than the runtime's synchronisation); a
        // kernel that does not signal within 100 ms is waited for, and its error reported, by the runtime
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0; !(seen = *flag == seq); spin++)
            if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) break;
    }
    if (he == hipSuccess && !seen) he = hipStreamSynchronize(w->stream);
    if (he != hipSuccess) {
        (void)writer_zero(w);
        return EZ_EDEVICE;
    }
    int st = EZ_OK;
    size_t got = 0;
    for (size_t j = 0; j < k && !st; j++) {
        st = (int)(int32_t)(m[6 * j + 5] & 0xffffffffu);
        got += (size_t)m[6 * j + 4];
    }
    if (!st && got > cap) st = EZ_ENOSPC;  // cannot happen (cap >= the sum of the bounds)
    if (st) {
        if (st == EZ_EINVAL) w->last_panic = EZ_PANIC_OFFSET;  // (Writes of < 2^26 bytes: no length panic)
        const int z = writer_zero(w);
        return z ? z : st;
    }
    size_t at = 0;
    for (size_t j = 0; j < k; j++) {
        const size_t sz = (size_t)m[6 * j + 4];
        if (sz) memcpy(out + at, H + (size_t)m[6 * j + 2], sz);
        at += sz;
        if (out_ends) out_ends[j] = at;
    }
    w->pos += (int64_t)n;
    w->pristine = false;
    w->tainted = false;
    return EZ_OK;
}

int writer_run(ez_writer *w, const uint8_t *p, const uint64_t *ends, size_t k, uint8_t *out, size_t cap, uint64_t *out_ends) {
    w->last_panic = EZ_PANIC_NONE;  // (set again only by a failure of this call)
    const size_t n = k ? (size_t)ends[k - 1] : 0;
    size_t bound = 0;
    for (size_t j = 0; j < k; j++) {
        if (ends[j] < (j ? ends[j - 1] : 0)) return EZ_EINVAL;
        bound += ez_compress_bound((size_t)(ends[j] - (j ? ends[j - 1] : 0)));
    }
    // checked before anything reaches the device: the kernel advances the handle's ring and table, so a
    // call that could not return its bytes must not run at all (a retry then sees the same history)
    if (cap < bound) return EZ_ENOSPC;
    {
        DeviceGuard g(w->device);
        if (!g.ok) return EZ_EDEVICE;
        const int z = writer_clean(w);
        if (z) return z;
    }
    if (k >= 1) {  // K1L on the handle's ring and table, when every Write qualifies
        const int e = writer_run_long(w, p, ends, k, out, cap, out_ends, bound);
        if (e >= 0) return e;
    }
    DeviceGuard g(w->device);
    if (!g.ok) return EZ_EDEVICE;
    const size_t o_meta = (n + 15) & ~(size_t)15, nm = 8 + 2 * k;  // meta words
    const size_t o_out = o_meta + nm * 8 + ((k > 1 ? k : 0) * 8);
    const size_t total = ((o_out + 15) & ~(size_t)15) + bound + 16;
    if (w->dev.ensure(total) || w->host.ensure(total)) return EZ_EDEVICE;
    const size_t o_o = (o_out + 15) & ~(size_t)15;
    uint8_t *H = w->host.as<uint8_t>(), *D = w->dev.as<uint8_t>();
    if (n) memcpy(H, p, n);
    uint64_t *m = (uint64_t *)(H + o_meta);
    m[0] = 0; m[1] = n; m[2] = o_o; m[3] = o_o + bound; m[4] = 0; m[5] = 0; m[6] = 0; m[7] = k;
    for (size_t j = 0; j < k; j++) m[8 + j] = ends[j];
    EZ_HIP(hipMemcpyAsync(D, H, o_meta + nm * 8, hipMemcpyHostToDevice, w->stream));
    uint64_t *dm = (uint64_t *)(D + o_meta);
    ez::CompressArgs a{};
    a.in = D;
    a.in_off = dm;
    a.out = D;
    a.out_off = dm + 2;
    a.out_size = dm + 4;
    a.status = (int32_t *)(dm + 5);
    a.count = 1;
    a.bs = w->bs;
    a.hs = w->hs;
    a.append_magic = w->append_magic;
    a.ver = w->ver;
    a.header = w->pristine ? 1 : 0;
    a.start = w->pos;
    a.ring = w->ring.as<uint8_t>();
    a.ht_global = w->ht.as<uint32_t>();
    a.max_len = n ? n : 1;
    if (k > 1) {  // the Writes' ends, and their output ends recorded by the kernel
        a.write_idx = dm + 6;
        a.write_end = dm + 8;
        a.max_writes = k;
        a.write_out = dm + 8 + k;
    }
    // from the launch on, the device history may already hold p: any failure restarts the stream
    // (as Go does after a failed sink write, writer.go:391-393), so later Writes stay exact
    w->tainted = true;
    hipError_t he = ez::launch_compress(a, w->stream);
    // status, sizes and output back at once (the bound, not the exact size: small Writes)
    if (he == hipSuccess)
        he = hipMemcpyAsync(H + o_meta, D + o_meta, o_o - o_meta + bound, hipMemcpyDeviceToHost, w->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(w->stream);
    if (he != hipSuccess) {
        (void)writer_zero(w);
        return EZ_EDEVICE;
    }
    int st = (int)(int32_t)(m[5] & 0xffffffffu);
    const size_t got = (size_t)m[4];
    if (!st && got > bound) st = EZ_ENOSPC;  // cannot happen (tests/test_bound.py)
    if (st) {
        // the device history already holds p while the stream position does not: start the stream
        // over, as Go does after a failed sink write (writer.go:391-393), so later Writes stay exact
        if (st == EZ_EINVAL) {
            // Encoder.Tag panics only for lengths of 2^32 - 8 past its Len4 base (writer.go:558-562),
            // which needs a Write at least that long; the only other panic is the distance check
            // (writer.go:308-310)
            const uint64_t tag_limit = ((uint64_t)1 << 32) - 8 + 65916;
            w->last_panic = EZ_PANIC_OFFSET;
            for (size_t j = 0; j < k; j++)
                if (ends[j] - (j ? ends[j - 1] : 0) >= tag_limit) w->last_panic = EZ_PANIC_LENGTH;
        }
        const int z = writer_zero(w);
        return z ? z : st;
    }
    if (got) memcpy(out, H + o_o, got);
    if (out_ends) {
        if (k > 1) for (size_t j = 0; j < k; j++) out_ends[j] = m[8 + k + j];
        else if (k == 1) out_ends[0] = got;
    }
    w->pos += (int64_t)n;
    w->pristine = false;
    w->tainted = false;
    return EZ_OK;
}

}  // namespace

extern "C" int ez_writer_write(ez_writer *w, const uint8_t *p, size_t n, uint8_t *out, size_t cap, size_t *out_n) {
    *out_n = 0;
    const uint64_t end = n;
    uint64_t oe = 0;
    const int e = writer_run(w, p, &end, 1, out, cap, &oe);
    if (!e) *out_n = (size_t)oe;
    return e;
}

extern "C" int ez_writer_write_batch(ez_writer *w, const uint8_t *p, const uint64_t *ends, size_t k, uint8_t *out, size_t cap,
                                     uint64_t *out_ends) {
    if (k == 0) return EZ_OK;
    if (!ends || !out_ends) return EZ_EINVAL;
    return writer_run(w, p, ends, k, out, cap, out_ends);
}

extern "C" int ez_writer_header(ez_writer *w, uint8_t *out, size_t cap, size_t *out_n) {
    *out_n = 0;
    if (w->tainted) {
        DeviceGuard g(w->device);
        if (!g.ok) return EZ_EDEVICE;
        const int z = writer_clean(w);
        if (z) return z;
    }
    if (!w->pristine) return EZ_OK;
    uint8_t h[16];
    const size_t k = header_bytes(h, w->append_magic, w->ver, w->bs);
    if (k > cap) return EZ_ENOSPC;
    memcpy(out, h, k);
    *out_n = k;
    w->pristine = false;
    return EZ_OK;
}

extern "C" int ez_writer_break(ez_writer *w, uint8_t *out, size_t cap, size_t *out_n) {
    *out_n = 0;
    if (w->tainted) {
        DeviceGuard g(w->device);
        if (!g.ok) return EZ_EDEVICE;
        const int z = writer_clean(w);
        if (z) return z;
    }
    uint8_t h[32];
    size_t k = 0;
    if (w->pristine) k = header_bytes(h, w->append_magic, w->ver, w->bs);
    h[k++] = 0x80;
    h[k++] = 0x18 | 7;  // Meta, MetaBreak|MetaLen0 (writer.go:363)
    if (k > cap) return EZ_ENOSPC;
    memcpy(out, h, k);
    *out_n = k;
    w->pristine = false;
    return EZ_OK;
}

extern "C" int ez_writer_reset(ez_writer *w) {
    DeviceGuard g(w->device);
    if (!g.ok) return EZ_EDEVICE;
    return writer_zero(w);
}

extern "C" int ez_writer_reset_size(ez_writer *w, int64_t block, int64_t htable) {
    if (!valid_writer_sizes(block, htable)) return EZ_EINVAL;
    DeviceGuard g(w->device);
    if (!g.ok) return EZ_EDEVICE;
    int e = writer_alloc(w, block, htable);
    if (e) return e;
    return writer_zero(w);
}

// ------------------------------------------------------------------ Reader handle

struct ez_reader {
    int device = 0;
    ez::DecodeState st{};
    int64_t limit = 0;
    int require_magic = 0, skip_meta = 0;
    DBuf in, obuf[2], dstate, meta;  // obuf: history + output, double-buffered (ez_reader_read)
    int cur = 0;
    hipStream_t stream = nullptr;
    // whole-stream decode (ez_reader_set_whole): the stream decoded once by the batch path into a_out
    // (device memory), the Reads served from it through a pinned staging window
    int whole = 0;             // the caller's b is the whole stream (NewReaderBytes / ResetBytes)
    int tried = 0;             // tried since the last reset
    int ahead_on = 0;          // Reads are served from a_out[a_at .. a_n)
    DBuf a_in, a_out, a_meta, a_ws, a_brk;  // kept across resets (grown, never shrunk)
    uint64_t a_n = 0, a_at = 0;             // bytes decoded; bytes served
    size_t a_blen = 0;                      // the input decoded (len(r.b) at the first Read)
    std::vector<uint64_t> brk;              // the Break metas' output positions, ascending
    size_t brk_next = 0;                    // the next one a Read has not reported
    int64_t end_bs = 0, end_pos = 0;        // the Reader's len(r.block) and r.pos after the stream
    uint8_t *stage = nullptr;               // pinned: srv[stage_at .. stage_at + stage_n)
    uint64_t stage_at = 0, stage_n = 0;
    const uint8_t *srv = nullptr;           // the device bytes the Reads are served from (a_out, or a read-ahead's)
    // read-ahead of a NewReader(io.Reader) handle (whole == 0, ez_reader_read): all the input buffered
    // at a Read decoded at once; its Reads are then served from srv[a_at .. a_n) (ahead_on stays 0)
    int s_on = 0;
    int64_t s_iend = 0;                     // the absolute input position the read-ahead consumed to
    int64_t s_skip = -1;                    // a read-ahead handed over at this absolute buffer end: none until more input
    int64_t s_count = 0;                    // read-aheads made (ez_reader_ahead_count)
    DBuf s_meta, s_ws;
};

extern "C" int ez_reader_new(int device, ez_reader **out) {
    *out = nullptr;
    DeviceGuard g(device);
    if (!g.ok) return EZ_EDEVICE;
    ez_reader *r = new ez_reader();
    r->device = device;
    if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
        delete r;
        return EZ_EDEVICE;
    }
    if (r->dstate.ensure(sizeof(ez::DecodeState)) || r->meta.ensure(64)) {
        ez_reader_free(r);
        return EZ_EDEVICE;
    }
    *out = r;
    return EZ_OK;
}

extern "C" void ez_reader_free(ez_reader *r) {
    if (!r) return;
    DeviceGuard g(r->device);
    r->in.release();
    r->obuf[0].release();
    r->obuf[1].release();
    r->dstate.release();
    r->meta.release();
    r->a_in.release();
    r->a_out.release();
    r->a_meta.release();
    r->a_ws.release();
    r->a_brk.release();
    r->s_meta.release();
    r->s_ws.release();
    if (r->stage) (void)hipHostFree(r->stage);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
}

extern "C" int ez_reader_configure(ez_reader *r, int64_t block_size_limit, int require_magic, int skip_meta) {
    r->limit = block_size_limit;
    r->require_magic = require_magic ? 1 : 0;
    r->skip_meta = skip_meta ? 1 : 0;
    return EZ_OK;
}

// ResetBytes reader.go:102-113: block = block[:0], pos = 0, state = 0
// (r.d.Ver is kept, as in the reference).
extern "C" int ez_reader_reset(ez_reader *r) {
    const int32_t ver = r->st.ver;
    r->st = ez::DecodeState{};
    r->st.ver = ver;
    r->tried = 0;
    r->ahead_on = 0;
    r->s_on = 0;
    r->s_skip = -1;
    r->a_n = r->a_at = 0;
    r->brk.clear();
    r->brk_next = 0;
    r->stage_n = 0;
    return EZ_OK;
}

extern "C" int ez_reader_set_whole(ez_reader *r, int whole) {
    r->whole = whole ? 1 : 0;
    return EZ_OK;
}

extern "C" int ez_reader_whole_decoded(const ez_reader *r) { return r->ahead_on; }

extern "C" int64_t ez_reader_ahead_count(const ez_reader *r) { return r->s_count; }

extern "C" int ez_reader_pending(const ez_reader *r) { return r->st.state != 0 ? 1 : 0; }

namespace {
// K2j's workspace for Reader handles, one per device: a whole-stream decode is synchronous, so the
// handles of a device take turns with it (a handle of its own would be allocated anew for every
// NewReaderBytes, tens of ms for a large stream)
struct ReaderJws {
    std::mutex mu;
    DBuf buf;
};
ReaderJws &reader_jws(int dev) {
    static std::mutex m;
    static std::map<int, ReaderJws *> all;
    std::lock_guard<std::mutex> lk(m);
    ReaderJws *&p = all[dev];
    if (!p) p = new ReaderJws();
    return *p;
}

constexpr size_t kAheadMax = ((size_t)1 << 30) - 64;  // the largest output slot (K2t takes slots below 2^30)
constexpr size_t kAheadBrk = (size_t)1 << 16;         // Break positions recorded (more: Read by Read)
constexpr size_t kStage = (size_t)4 << 20;            // the pinned staging window (host memory per Reader)

// Whole-stream decode (NewReaderBytes then Read to the end, the reference's common use): the batch
// path decodes b as one stream -- K2t, every lane of a wave on its tokens -- into a device slot, and the
// Reads are then served from that output.  The slot starts at 8 x b_len and grows 4x while K2t reports
// it too small (up to 1 GiB).  The decoders record every Break meta's output position, so the Reads stop
// at each with ErrBreak as Read by Read does (reader.go:312-313), and the Reader's state at the end
// (len(r.block), r.pos), so that input a caller supplies after the stream (a Reader set after
// NewReaderBytes) continues Read by Read.  It applies where it gives exactly the bytes and errors of
// Read-by-Read decoding: a clean end of stream (status OK), RequireMagic and SkipUnsupportedMeta off;
// anything else leaves the handle as it was and the exact decoder runs Read by Read.  Device buffers are
// kept in the handle, host memory is the 4 MiB staging window.  Returns 1 when the Reads are now
// served from the decoded bytes.
int reader_ahead(ez_reader *r, const uint8_t *b, size_t b_len) {
    r->tried = 1;
    if (b_len == 0 || b_len > ((size_t)1 << 28) || r->require_magic || r->skip_meta) return 0;
    const size_t ws = ez_decompress_workspace(1);
    constexpr size_t o_meta = 64;  // [in_off 2][out_off 2][out_size][status][end_state 2]
    if (r->a_in.ensure(b_len + 64) || r->a_meta.ensure(o_meta * 2) || r->a_ws.ensure(ws) || r->a_brk.ensure(8 * (kAheadBrk + 1)))
        return 0;
    if (!r->stage && hipHostMalloc((void **)&r->stage, kStage, hipHostMallocDefault) != hipSuccess) {
        r->stage = nullptr;
        return 0;
    }
    if (hipMemcpyAsync(r->a_in.p, b, b_len, hipMemcpyHostToDevice, r->stream) != hipSuccess) return 0;
    size_t cap = 8 * b_len + 4096 < kAheadMax ? 8 * b_len + 4096 : kAheadMax;
    for (;;) {
        if (r->a_out.ensure(cap + 64)) return 0;
        uint64_t m[8] = {0, (uint64_t)b_len, 0, (uint64_t)cap, 0, 0, (uint64_t)-1, (uint64_t)-1};
        uint64_t nbrk = 0;
        if (hipMemcpyAsync(r->a_meta.p, m, sizeof m, hipMemcpyHostToDevice, r->stream) != hipSuccess) return 0;
        if (hipMemsetAsync(r->a_brk.p, 0, 8, r->stream) != hipSuccess) return 0;
        uint64_t *dmw = r->a_meta.as<uint64_t>();
        ez::DecompressArgs a{};
        a.in = r->a_in.as<uint8_t>();
        a.in_off = dmw;
        a.out = r->a_out.as<uint8_t>();
        a.out_off = dmw + 2;
        a.out_size = dmw + 4;
        a.status = (int32_t *)(dmw + 5);
        a.end_state = (int64_t *)(dmw + 6);
        a.breaks = r->a_brk.as<uint64_t>();
        a.breaks_cap = kAheadBrk;
        a.count = 1;
        a.block_size_limit = r->limit;
        a.slow = r->a_ws.as<uint32_t>();
        a.max_out = cap;
        // one stream: K2j (chip-wide) for a long one, else the token-parallel wave
        a.force = b_len >= ((size_t)16 << 10) ? 'j' : 't';
        {
            ReaderJws &J = reader_jws(r->device);
            std::lock_guard<std::mutex> lk(J.mu);
            if (a.force == 'j') {
                const uint64_t need = ez::jump_workspace_bytes(1, b_len, cap);
                if (J.buf.ensure(need)) return 0;
                a.jws = J.buf.p;
                a.jws_cap = J.buf.cap;
            }
            if (ez::launch_decompress(a, r->stream) != hipSuccess) return 0;
            if (hipMemcpyAsync(m, r->a_meta.p, sizeof m, hipMemcpyDeviceToHost, r->stream) != hipSuccess) return 0;
            if (hipMemcpyAsync(&nbrk, r->a_brk.p, 8, hipMemcpyDeviceToHost, r->stream) != hipSuccess) return 0;
            if (hipStreamSynchronize(r->stream) != hipSuccess) return 0;
        }
        const int status = (int32_t)(m[5] & 0xffffffffu);
        if ((int64_t)m[6] == -2 && status == EZ_ENOSPC && cap < kAheadMax) {  // the slot was too small
            cap = cap < kAheadMax / 4 ? 4 * cap : kAheadMax;
            continue;
        }
        if (status != EZ_OK || m[4] > cap || nbrk > kAheadBrk || (int64_t)m[6] < 0) return 0;
        try {
            r->brk.resize((size_t)nbrk);
        } catch (...) {
            return 0;
        }
        if (nbrk && (hipMemcpy(r->brk.data(), r->a_brk.as<uint64_t>() + 1, 8 * nbrk, hipMemcpyDeviceToHost) != hipSuccess)) {
            r->brk.clear();
            return 0;
        }
        std::sort(r->brk.begin(), r->brk.end());
        r->brk_next = 0;
        r->a_n = m[4];
        r->a_at = 0;
        r->a_blen = b_len;
        r->end_bs = (int64_t)m[6];
        r->end_pos = (int64_t)m[7];
        r->stage_at = r->stage_n = 0;
        r->srv = r->a_out.as<uint8_t>();
        r->ahead_on = 1;
        return 1;
    }
}

// n bytes of the decoded stream from a_at into p (staged; a copy larger than the window goes direct)
int ahead_copy(ez_reader *r, uint8_t *p, size_t n) {
    while (n) {
        if (r->a_at < r->stage_at || r->a_at >= r->stage_at + r->stage_n) {
            const uint64_t left = r->a_n - r->a_at;
            if (n >= kStage) {
                if (hipMemcpy(p, r->srv + r->a_at, n, hipMemcpyDeviceToHost) != hipSuccess) return EZ_EDEVICE;
                r->a_at += n;
                return EZ_OK;
            }
            r->stage_at = r->a_at;
            r->stage_n = left < kStage ? left : kStage;
            if (hipMemcpy(r->stage, r->srv + r->a_at, r->stage_n, hipMemcpyDeviceToHost) != hipSuccess) {
                r->stage_n = 0;
                return EZ_EDEVICE;
            }
        }
        const uint64_t in_stage = r->stage_at + r->stage_n - r->a_at;
        const size_t k = n < in_stage ? n : (size_t)in_stage;
        memcpy(p, r->stage + (r->a_at - r->stage_at), k);
        p += k;
        n -= k;
        r->a_at += k;
    }
    return EZ_OK;
}

constexpr size_t kStreamMin = (size_t)8 << 10;  // buffered input a read-ahead takes at least

// Read-ahead of a NewReader(io.Reader) handle (the README's usage, reader.go:79-86, 116-141, 516-543):
// at a Read with nothing decoded ahead, every whole token of the buffered input b[i..b_len) is decoded
// at once on the device -- K2j continuing the stream from the handle's state: the window's history at
// the head of the decode buffer, a pending literal's bytes put in front, the chain stopping before a
// token the buffer ends inside of, whose literal bytes there are are output too (reader.go:166-168) --
// and the Reads are served from that output until it runs out.  Then Read asks for more input exactly
// where Read by Read would (the whole tokens are consumed, the state is the same), so the io.Reader
// sees the same calls and the caller the same bytes, Breaks and errors.  A buffer K2j hands over (an
// error, a MetaReset after output, a distance past the window, ...) is decoded Read by Read until more
// input arrives.  Returns 1 when the Reads are now served from the read-ahead.
int stream_ahead(ez_reader *r, const uint8_t *b, size_t b_len, size_t i, int64_t boff) {
    ez::DecodeState &st = r->st;
    const int64_t bend = boff + (int64_t)b_len;
    if (r->require_magic || r->skip_meta || b_len < i + kStreamMin || b_len > ((size_t)1 << 28) || bend == r->s_skip) return 0;
    if (st.state == 'c' || st.ver != 0 || st.bs > ((int64_t)1 << 30)) return 0;  // (mid-copy: after a Read that filled p)
    const size_t H = (size_t)st.hist, nin = b_len - i;
    // a pending literal (r.state 'l'): its next bytes are the input's first
    const size_t k = st.state == 'l' ? (st.len < (int64_t)nin ? (size_t)st.len : nin) : 0;
    const size_t n2 = nin - k;  // the input K2j decodes (none when the literal takes it all)
    const size_t ws = ez_decompress_workspace(1);
    if (r->in.ensure(n2 + 64) || r->s_meta.ensure(256) || r->s_ws.ensure(ws) || r->a_brk.ensure(8 * (kAheadBrk + 1))) return 0;
    if (!r->stage && hipHostMalloc((void **)&r->stage, kStage, hipHostMallocDefault) != hipSuccess) {
        r->stage = nullptr;
        return 0;
    }
    if (n2 && hipMemcpyAsync(r->in.p, b + i + k, n2, hipMemcpyHostToDevice, r->stream) != hipSuccess) return 0;
    size_t cap = n2 ? 8 * n2 + 4096 : 0;
    for (;;) {
        if (cap > kAheadMax) return 0;
        DBuf &cur = r->obuf[r->cur];
        if (cur.cap < H + k + cap + 64) {  // grow, keeping the history at the head
            DBuf nbuf;
            if (nbuf.ensure(H + k + cap + 64)) return 0;
            if (H && hipMemcpyAsync(nbuf.p, cur.p, H, hipMemcpyDeviceToDevice, r->stream) != hipSuccess) return 0;
            if (hipStreamSynchronize(r->stream) != hipSuccess) return 0;
            cur.release();
            cur = nbuf;
            nbuf.p = nullptr;
            nbuf.cap = 0;
        }
        uint8_t *o = cur.as<uint8_t>();
        if (k && hipMemcpyAsync(o + H, b + i, k, hipMemcpyHostToDevice, r->stream) != hipSuccess) return 0;
        // [in_off 2][out_off 2][out_size][status][end_state 5][slow count (u32)]
        uint64_t m[12] = {0, (uint64_t)n2, (uint64_t)(H + k), (uint64_t)(H + k + cap), 0, 0, 0, 0, 0, 0, 0, 0};
        uint64_t nbrk = 0;
        if (n2) {
            uint64_t *dm = r->s_meta.as<uint64_t>();
            if (hipMemcpyAsync(dm, m, sizeof m, hipMemcpyHostToDevice, r->stream) != hipSuccess) return 0;
            if (hipMemsetAsync(r->a_brk.p, 0, 8, r->stream) != hipSuccess) return 0;
            if (hipMemsetAsync(r->s_ws.p, 0, 4, r->stream) != hipSuccess) return 0;
            ez::DecompressArgs a{};
            a.in = r->in.as<uint8_t>();
            a.in_off = dm;
            a.out = o;
            a.out_off = dm + 2;
            a.out_size = dm + 4;
            a.status = (int32_t *)(dm + 5);
            a.end_state = (int64_t *)(dm + 6);
            a.breaks = r->a_brk.as<uint64_t>();
            a.breaks_cap = kAheadBrk;
            a.count = 1;
            a.block_size_limit = r->limit;
            a.slow = r->s_ws.as<uint32_t>();
            a.max_out = cap;
            a.in_bytes = n2;
            a.out_bytes = cap;
            a.c_on = 1;
            a.c_bsl = st.bs == 0 ? -1 : __builtin_ctzll((uint64_t)st.bs);
            a.c_hist = H + k;
            a.c_pos0 = st.pos + (int64_t)k;
            {
                ReaderJws &J = reader_jws(r->device);
                std::lock_guard<std::mutex> lk(J.mu);
                const uint64_t need = ez::jump_workspace_bytes(1, n2, cap + H + k + 16);
                if (J.buf.ensure(need)) return 0;
                a.jws = J.buf.p;
                a.jws_cap = J.buf.cap;
                if (ez::launch_decompress_jump(a, r->stream) != hipSuccess) return 0;
                if (hipMemcpyAsync(m, dm, sizeof m, hipMemcpyDeviceToHost, r->stream) != hipSuccess) return 0;
                if (hipMemcpyAsync(&nbrk, r->a_brk.p, 8, hipMemcpyDeviceToHost, r->stream) != hipSuccess) return 0;
                uint32_t slow = 0;
                if (hipMemcpyAsync(&slow, r->s_ws.p, 4, hipMemcpyDeviceToHost, r->stream) != hipSuccess) return 0;
                if (hipStreamSynchronize(r->stream) != hipSuccess) return 0;
                if (slow) {
                    if ((int64_t)m[6] == -2 && cap < kAheadMax) {  // the slot was too small
                        cap = cap < kAheadMax / 4 ? 4 * cap : kAheadMax;
                        continue;
                    }
                    r->s_skip = bend;  // handed over: Read by Read until more input arrives
                    return 0;
                }
            }
            if (nbrk > kAheadBrk) {
                r->s_skip = bend;
                return 0;
            }
        }
        // the chain's stop and a literal the input ends inside of
        const int64_t total = n2 ? (int64_t)m[4] : 0;
        const int64_t stop = n2 ? (int64_t)m[8] : 0, tj = n2 ? (int64_t)m[9] : 0, tL = n2 ? (int64_t)m[10] : 0;
        int64_t tail = 0;
        if (tj > 0) {
            tail = (int64_t)n2 - stop - tj < tL ? (int64_t)n2 - stop - tj : tL;
            if (tail > 0 &&
                hipMemcpyAsync(o + H + k + total, r->in.as<uint8_t>() + stop + tj, (size_t)tail, hipMemcpyDeviceToDevice, r->stream) != hipSuccess)
                return 0;
        }
        try {
            r->brk.resize((size_t)nbrk);
        } catch (...) {
            return 0;
        }
        if (nbrk && hipMemcpy(r->brk.data(), r->a_brk.as<uint64_t>() + 1, 8 * nbrk, hipMemcpyDeviceToHost) != hipSuccess) return 0;
        for (auto &x : r->brk) x += k;  // (positions in the served bytes: the pending literal's come first)
        std::sort(r->brk.begin(), r->brk.end());
        // the Reader's state after the last whole token (or inside the literal the input ends in)
        const int64_t out_n = (int64_t)k + total + tail;
        ez::DecodeState ns = st;
        if (n2) ns.bs = (int64_t)m[6];
        ns.pos = st.pos + out_n;
        if (n2 == 0) {  // the pending literal took the whole input
            ns.len = st.len - (int64_t)k;
            ns.state = ns.len == 0 ? 0 : 'l';
        } else if (tj > 0) {
            ns.state = 'l';
            ns.len = tL - tail;
        } else {
            ns.state = 0;
            ns.len = 0;
        }
        ns.hist = ns.bs == 0 ? 0 : (ns.pos < ns.bs ? ns.pos : ns.bs);
        // the next decode's history: the window's last hist bytes, at the head of the other buffer
        const size_t H2 = (size_t)ns.hist;
        if (H2 > H + (size_t)out_n) return 0;  // (cannot happen: the history is decoded output)
        DBuf &nxt = r->obuf[r->cur ^ 1];
        if (nxt.cap < H2 + 16) {
            if (hipStreamSynchronize(r->stream) != hipSuccess || nxt.ensure(H2 + 16)) return 0;
        }
        if (H2 && hipMemcpyAsync(nxt.p, o + H + out_n - H2, H2, hipMemcpyDeviceToDevice, r->stream) != hipSuccess) return 0;
        if (hipStreamSynchronize(r->stream) != hipSuccess) return 0;
        r->cur ^= 1;  // (the served bytes stay in this buffer; the next decode writes the other)
        st = ns;
        r->srv = o + H;
        r->a_n = (uint64_t)out_n;
        r->a_at = 0;
        r->brk_next = 0;
        r->stage_at = r->stage_n = 0;
        r->s_iend = boff + (int64_t)(n2 == 0 || tj > 0 ? b_len : i + k + (size_t)stop);
        r->s_on = 1;
        r->s_count++;
        return 1;
    }
}

// Input after the decoded stream (a Reader set after NewReaderBytes, so more() supplied more): the
// handle continues Read by Read from the Reader's state at the stream's end -- len(r.block), r.pos, no
// token pending, version 0 (the whole decode takes only those) -- with the window's history, the last
// min(r.pos, len(r.block)) decoded bytes, at the head of the decode buffer.
int ahead_leave(ez_reader *r) {
    ez::DecodeState st{};
    st.bs = r->end_bs;
    st.pos = r->end_pos;
    st.hist = st.bs == 0 ? 0 : (st.pos < st.bs ? st.pos : st.bs);
    const size_t H = (size_t)st.hist;
    if (H > r->a_n) return EZ_EDEVICE;  // (cannot happen: the history is decoded output)
    DBuf &cur = r->obuf[r->cur];
    if (cur.ensure(H + 16)) return EZ_EDEVICE;
    if (H && hipMemcpyAsync(cur.p, r->a_out.as<uint8_t>() + (r->a_n - H), H, hipMemcpyDeviceToDevice, r->stream) != hipSuccess)
        return EZ_EDEVICE;
    if (hipStreamSynchronize(r->stream) != hipSuccess) return EZ_EDEVICE;
    r->st = st;
    r->ahead_on = 0;
    return EZ_OK;
}
}  // namespace

// Input is uploaded in windows from b[i] on, not the whole of b per call: a Read loop over one large
// NewReaderBytes buffer then moves each input byte to the device about once.  A window that ends inside
// a token makes the decoder stop there with EZ_ESHORTBUF and nothing of that token consumed
// (reader.go:218-270), so the next window resumes at exactly that token; a token longer than the window
// with no progress doubles the window.  The decoded block history sits in front of the output in one of
// two device buffers; after a call the last min(pos, bs) bytes are copied once into the head of the
// other buffer, which the next call decodes into.
extern "C" int ez_reader_read(ez_reader *r, const uint8_t *b, size_t b_len, size_t i, int64_t boff, uint8_t *p,
                              size_t p_len, size_t *n, size_t *i_out, int64_t *detail) {
    *n = 0;
    *i_out = i;
    if (detail) *detail = 0;
    if (p_len == 0) return EZ_OK;  // Read(p) with len(p) == 0 returns at once (reader.go:119)
    DeviceGuard g(r->device);
    if (!g.ok) return EZ_EDEVICE;
    // a fresh handle over a whole stream: decode it once (reader_ahead), then serve every Read from it
    if (!r->ahead_on && r->whole && !r->tried && i == 0 && boff == 0 && r->st.bs == 0 && r->st.pos == 0 && r->st.state == 0)
        (void)reader_ahead(r, b, b_len);
    if (r->ahead_on && r->a_at == r->a_n && r->brk_next == r->brk.size() && (uint64_t)boff + b_len > r->a_blen) {
        // the stream is served and input follows it: Read by Read from the Reader's state at its end
        if (ahead_leave(r) != EZ_OK) return EZ_EDEVICE;
    }
    // NewReader(io.Reader): the buffered input decoded ahead, the Reads served from it
    if (!r->whole && !r->s_on) (void)stream_ahead(r, b, b_len, i, boff);
    if (r->s_on) {
        const bool at_brk = r->brk_next < r->brk.size();
        const uint64_t lim = at_brk ? r->brk[r->brk_next] : r->a_n;
        const uint64_t left = lim - r->a_at;
        const size_t m = p_len < left ? p_len : (size_t)left;
        if (m && ahead_copy(r, p, m) != EZ_OK) return EZ_EDEVICE;
        *n = m;
        *i_out = (size_t)(r->s_iend - boff);  // (only read back when this returns ErrShortBuffer)
        if (m == p_len) return EZ_OK;
        if (at_brk) {
            r->brk_next++;
            return EZ_EBREAK;
        }
        r->s_on = 0;  // served: Read asks for more input where Read by Read would
        return EZ_ESHORTBUF;
    }
    if (r->ahead_on) {
        // up to the next Break (reader.go:312-313: Read returns the bytes before it with ErrBreak, and a
        // Read that starts at it returns 0 bytes with ErrBreak) or the stream's end
        const bool at_brk = r->brk_next < r->brk.size();
        const uint64_t lim = at_brk ? r->brk[r->brk_next] : r->a_n;
        const uint64_t left = lim - r->a_at;
        const size_t m = p_len < left ? p_len : (size_t)left;
        if (m && ahead_copy(r, p, m) != EZ_OK) return EZ_EDEVICE;
        *n = m;
        if (m == p_len) return EZ_OK;  // (the input position is reported when the output is done)
        if (at_brk) {
            r->brk_next++;
            return EZ_EBREAK;
        }
        *i_out = b_len;  // the stream's end: Read asks for more input and gets EOF
        return EZ_ESHORTBUF;
    }
    const size_t H = (size_t)r->st.hist;
    DBuf &cur = r->obuf[r->cur];
    if (cur.cap < H + p_len + 16) {  // grow, keeping the history at the head
        DBuf nb;
        if (nb.ensure(H + p_len + 16)) return EZ_EDEVICE;
        if (H) EZ_HIP(hipMemcpyAsync(nb.p, cur.p, H, hipMemcpyDeviceToDevice, r->stream));
        EZ_HIP(hipStreamSynchronize(r->stream));
        cur.release();
        cur = nb;
        nb.p = nullptr;
        nb.cap = 0;
    }
    if (r->meta.ensure(64)) return EZ_EDEVICE;
    size_t win = p_len * 2 + 64 < ((size_t)1 << 16) ? ((size_t)1 << 16) : p_len * 2 + 64;
    size_t at = i, got = 0;
    int err = EZ_OK;
    for (;;) {
        const size_t take = b_len - at < win ? b_len - at : win;
        if (r->in.ensure(take + 16)) return EZ_EDEVICE;
        if (take) EZ_HIP(hipMemcpyAsync(r->in.p, b + at, take, hipMemcpyHostToDevice, r->stream));
        r->st.i = 0;
        EZ_HIP(hipMemcpyAsync(r->dstate.p, &r->st, sizeof(r->st), hipMemcpyHostToDevice, r->stream));
        uint64_t m[4] = {0, (uint64_t)take, (uint64_t)(H + got), (uint64_t)(H + p_len)};
        EZ_HIP(hipMemcpyAsync(r->meta.p, m, sizeof(m), hipMemcpyHostToDevice, r->stream));
        ez::DecompressArgs a{};
        uint64_t *dm = r->meta.as<uint64_t>();
        a.in = r->in.as<uint8_t>();
        a.in_off = dm;
        a.out = cur.as<uint8_t>();
        a.out_off = dm + 2;
        a.out_size = nullptr;
        a.status = nullptr;
        a.count = 1;
        a.block_size_limit = r->limit;
        a.require_magic = r->require_magic;
        a.skip_unsupported_meta = r->skip_meta;
        a.handle = 1;
        a.boff = boff + (int64_t)at;  // absolute offset of the window's first byte
        a.st = r->dstate.as<ez::DecodeState>();
        EZ_HIP(ez::launch_decompress(a, r->stream));
        EZ_HIP(hipMemcpyAsync(&r->st, r->dstate.p, sizeof(r->st), hipMemcpyDeviceToHost, r->stream));
        EZ_HIP(hipStreamSynchronize(r->stream));
        err = r->st.err;
        const size_t used = (size_t)r->st.i, made = (size_t)r->st.n;
        at += used;
        got += made;
        // the window, not the input, ran short: go on with the next one
        if (err == EZ_ESHORTBUF && take < b_len - (at - used) && got < p_len) {
            if (used == 0 && made == 0) win *= 2;
            continue;
        }
        break;
    }
    const size_t H2 = (size_t)r->st.hist;
    if (got) EZ_HIP(hipMemcpyAsync(p, cur.as<uint8_t>() + H, got, hipMemcpyDeviceToHost, r->stream));
    if (H2) {  // the next call decodes into the other buffer, behind this block's last H2 bytes
        DBuf &nxt = r->obuf[r->cur ^ 1];
        if (nxt.cap < H2 + 16) {
            EZ_HIP(hipStreamSynchronize(r->stream));
            if (nxt.ensure(H2 + 16)) return EZ_EDEVICE;
        }
        EZ_HIP(hipMemcpyAsync(nxt.p, cur.as<uint8_t>() + H + got - H2, H2, hipMemcpyDeviceToDevice, r->stream));
        r->cur ^= 1;
    }
    EZ_HIP(hipStreamSynchronize(r->stream));
    *n = got;
    *i_out = at;
    if (detail) *detail = r->st.detail;
    return err;
}

// ------------------------------------------------------------------ batches

static int compress_batch_impl(int64_t block, int64_t htable, int flags, const ez_batch *b, const uint64_t *write_idx,
                               const uint64_t *write_end, uint64_t max_writes, void *hip_stream) {
    if (!valid_writer_sizes(block, htable)) return EZ_EINVAL;
    if (device_count() <= 0) return EZ_EDEVICE;
    ez::CompressArgs a{};
    a.in = b->in;
    a.in_off = b->in_off;
    a.out = b->out;
    a.out_off = b->out_off;
    a.out_size = b->out_size;
    a.status = b->status;
    a.count = b->count;
    a.bs = block;
    a.hs = htable;
    a.append_magic = (flags & EZ_F_NO_MAGIC) ? 0 : 1;
    a.ver = 0;
    a.header = 1;
    a.start = 0;
    a.ring = nullptr;
    a.max_len = b->max_len;
    a.write_idx = write_idx;
    a.write_end = write_end;
    a.max_writes = max_writes;
    // multi-Write streams: K1s when it takes them (fresh streams, 2 x stream <= block), else the
    // general kernel (one wave per stream, the history read from the stream's earlier Writes)
    if (write_idx && b->count == 0) return EZ_OK;
    const bool split_mw = write_idx && ez::split_stride_words(a) != 0;
    auto words_of = [&](const ez::CompressArgs &x) { return split_mw ? ez::split_scratch_words(x) : ez::compress_scratch_words(x); };
    uint64_t words = words_of(a);
    // the scratch of this (device, stream) stays leased through the launches: another host thread
    // growing it meanwhile would free what these kernels were given
    ez::CacheLease lease;
    if (words) {
        int dev = 0;
        EZ_HIP(hipGetDevice(&dev));
        lease = k1_cache().acquire(dev, hip_stream);
        if (!lease->ensure((size_t)words * 4)) {
            // K1c's logs (about 13 bytes per input byte) may not fit where K1L's records do: K1L alone
            ez::CompressArgs b = a;
            b.no_k1c = 1;
            const uint64_t w2 = words_of(b);
            if (w2 >= words || !lease->ensure((size_t)w2 * 4)) return EZ_EDEVICE;
            a = b;
        }
        a.ht_global = (uint32_t *)lease->p;
    }
    if (split_mw) EZ_HIP(ez::launch_compress_split(a, a.ht_global, (hipStream_t)hip_stream));
    else EZ_HIP(ez::launch_compress(a, (hipStream_t)hip_stream));
    return EZ_OK;
}

extern "C" int ez_compress_batch(int64_t block, int64_t htable, int flags, const ez_batch *b, void *hip_stream) {
    return compress_batch_impl(block, htable, flags, b, nullptr, nullptr, 0, hip_stream);
}

extern "C" int ez_compress_batch_writes(int64_t block, int64_t htable, int flags, const ez_batch *b, const uint64_t *write_idx,
                                        const uint64_t *write_end, uint64_t max_writes, void *hip_stream) {
    if (!write_idx || !write_end || max_writes == 0) return EZ_EINVAL;
    return compress_batch_impl(block, htable, flags, b, write_idx, write_end, max_writes, hip_stream);
}

extern "C" size_t ez_pack_workspace(uint64_t count) { return ez::pack_workspace(count); }

extern "C" int ez_pack_batch(const uint8_t *slots, const uint64_t *slot_off, const uint64_t *sizes, uint64_t count,
                             uint8_t *packed, uint64_t *packed_off, void *workspace, void *hip_stream) {
    if (device_count() <= 0) return EZ_EDEVICE;
    EZ_HIP(ez::launch_pack(slots, slot_off, sizes, count, packed, packed_off, workspace, (hipStream_t)hip_stream));
    return EZ_OK;
}

extern "C" int ez_compress_kernel(int64_t block, int64_t htable, uint64_t max_len, uint64_t count) {
    if (!valid_writer_sizes(block, htable)) return -EZ_EINVAL;
    if (device_count() <= 0) return -EZ_EDEVICE;
    ez::CompressArgs a{};
    a.count = count;
    a.bs = block;
    a.hs = htable;
    a.max_len = max_len;
    a.append_magic = 1;
    a.header = 1;
    return (int)ez::compress_variant(a);
}

extern "C" int ez_select_compress_kernel(int kind) {
    if (kind != 0 && !strchr("sSwxl", kind)) return EZ_EINVAL;
    ez::select_split_table(kind == 'S');
    ez::select_compress_variant(kind == 'S' ? 's' : kind);
    return EZ_OK;
}

extern "C" int ez_select_decompress_kernel(int kind) {
    if (kind != 0 && kind != 'r' && kind != 'w' && kind != 't' && kind != 'j') return EZ_EINVAL;
    ez::select_decompress_variant(kind);
    return EZ_OK;
}

extern "C" int ez_decompress_kernel_last(void) { return ez::last_decompress_variant(); }

extern "C" int ez_compress_k1c_stats(int enable, uint64_t *counts) {
    ez::k1c_stats(enable, counts);
    return EZ_OK;
}

extern "C" size_t ez_decompress_workspace(uint64_t count) {
    return (size_t)ez::decompress_workspace_words(count) * sizeof(uint32_t);
}

extern "C" int ez_decompress_batch(int64_t block_size_limit, const ez_batch *b, void *workspace, void *hip_stream) {
    if (device_count() <= 0) return EZ_EDEVICE;
    ez::DecompressArgs a{};
    a.in = b->in;
    a.in_off = b->in_off;
    a.out = b->out;
    a.out_off = b->out_off;
    a.out_size = b->out_size;
    a.status = b->status;
    a.count = b->count;
    a.block_size_limit = block_size_limit;
    a.handle = 0;
    a.slow = (uint32_t *)workspace;
    a.max_out = b->max_len;  // decompress: the largest output slot, if the caller knows it
    a.in_bytes = b->in_bytes;  // the batch's extents, if the caller knows them
    a.out_bytes = b->out_bytes;
    EZ_HIP(ez::launch_decompress(a, (hipStream_t)hip_stream));
    return EZ_OK;
}

// ------------------------------------------------------------------ host batches over several devices

namespace {
// Contiguous whole-stream shards of a batch, balanced by bytes: shard k is streams [first[k],
// first[k+1]) with first[k] the first stream starting at or after k / nshard of the batch's bytes.
std::vector<uint64_t> shard_bounds(const uint64_t *off, uint64_t count, int nshard) {
    std::vector<uint64_t> first((size_t)nshard + 1, count);
    first[0] = 0;
    const uint64_t total = off[count] - off[0];
    uint64_t s = 0;
    for (int k = 1; k < nshard; k++) {
        const uint64_t target = off[0] + (uint64_t)((unsigned __int128)total * (uint64_t)k / (uint64_t)nshard);
        while (s < count && off[s] < target) s++;
        first[(size_t)k] = s;
    }
    return first;
}

int resolve_devices(const int *devices, int ndev, std::vector<int> &out) {
    const int have = device_count();
    if (have <= 0) return EZ_EDEVICE;
    if (!devices || ndev <= 0) {
        for (int d = 0; d < have; d++) out.push_back(d);
        return EZ_OK;
    }
    for (int k = 0; k < ndev; k++) {
        if (devices[k] < 0 || devices[k] >= have) return EZ_EINVAL;
        out.push_back(devices[k]);
    }
    return EZ_OK;
}

// A shard's HIP stream, timing events and grow-only device buffers, pooled per device between calls:
// the K1 / K2j scratch caches are keyed by (device, stream), so pooled streams reuse their entries
// instead of leaving one behind per call, and repeated calls do not re-allocate (ez_release_cached
// frees the idle ones).
struct ShardRes {
    int dev = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the shard's device work
    DBuf in, in_off, out, out_off, size, status, ws, packed, packed_off;
    void release_bufs() {
        for (DBuf *b : {&in, &in_off, &out, &out_off, &size, &status, &ws, &packed, &packed_off}) b->release();
    }
};

class ShardPool {
  public:
    // an idle resource of dev, or a new one (the caller's thread is bound to dev); nullptr on failure
    ShardRes *take(int dev) {
        {
            std::lock_guard<std::mutex> lk(m_);
            auto &v = idle_[dev];
            if (!v.empty()) {
                ShardRes *r = v.back();
                v.pop_back();
                return r;
            }
        }
        ShardRes *r = new ShardRes();
        r->dev = dev;
        if (hipStreamCreateWithFlags(&r->st, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&r->ev0) != hipSuccess ||
            hipEventCreate(&r->ev1) != hipSuccess) {
            if (r->ev0) (void)hipEventDestroy(r->ev0);
            if (r->st) (void)hipStreamDestroy(r->st);
            delete r;
            return nullptr;
        }
        return r;
    }
    void give(ShardRes *r) {
        std::lock_guard<std::mutex> lk(m_);
        idle_[r->dev].push_back(r);
    }
    // free the idle resources' buffers on dev (all devices for dev < 0); streams and events stay
    void trim(int dev) {
        std::lock_guard<std::mutex> lk(m_);
        for (auto &kv : idle_) {
            if (dev >= 0 && kv.first != dev) continue;
            if (hipSetDevice(kv.first) != hipSuccess) continue;
            for (ShardRes *r : kv.second) r->release_bufs();
        }
    }

  private:
    std::mutex m_;
    std::map<int, std::vector<ShardRes *>> idle_;
};
ShardPool &shard_pool() {
    static ShardPool *p = new ShardPool();  // (never destroyed: no HIP calls after the runtime's teardown)
    return *p;
}

// one shard of a multi-device call (its host thread runs it on a pooled resource)
struct Shard {
    int dev = 0;
    uint64_t first = 0, count = 0;
    ShardRes *r = nullptr;
    uint64_t total = 0, base = 0;  // compress: packed bytes of the shard, its place in the global packing
    int err = EZ_OK;
    ~Shard() {
        if (r) shard_pool().give(r);
    }
};

// the per-shard device intervals of the last multi-device call (ez_multi_last_shards)
struct ShardTime {
    int dev;
    double t0, t1;
};
std::mutex g_times_mu;
std::vector<ShardTime> g_times;

// run f(shard) on one host thread per shard (each binds its device and takes a pooled resource
// first), join them, then record their device intervals
template <class F>
int each_shard(std::vector<std::unique_ptr<Shard>> &sh, F f, bool record = true) {
    std::vector<std::thread> th;
    for (auto &p : sh) {
        Shard *x = p.get();
        if (x->count == 0) continue;
        th.emplace_back([x, &f]() {
            if (hipSetDevice(x->dev) != hipSuccess) {
                x->err = EZ_EDEVICE;
                return;
            }
            if (!x->r && !(x->r = shard_pool().take(x->dev))) {
                x->err = EZ_EDEVICE;
                return;
            }
            if (x->err != EZ_OK) return;
            if (hipEventRecord(x->r->ev0, x->r->st) != hipSuccess) {
                x->err = EZ_EDEVICE;
                return;
            }
            x->err = f(*x);
            if (x->err == EZ_OK && (hipEventRecord(x->r->ev1, x->r->st) != hipSuccess || hipEventSynchronize(x->r->ev1) != hipSuccess))
                x->err = EZ_EDEVICE;
        });
    }
    for (auto &t : th) t.join();
    for (auto &p : sh)
        if (p->err != EZ_OK) return p->err;
    if (!record) return EZ_OK;
    // device intervals, in ms from the earliest shard start on the same device
    std::vector<ShardTime> tv;
    for (auto &p : sh) {
        if (!p->r || p->count == 0) continue;
        const Shard *ref = nullptr;
        for (auto &q : sh) {  // the shard on this device whose start is earliest
            if (!q->r || q->count == 0 || q->dev != p->dev) continue;
            if (!ref) {
                ref = q.get();
                continue;
            }
            float e = 0.f;
            if (hipSetDevice(p->dev) == hipSuccess && hipEventElapsedTime(&e, ref->r->ev0, q->r->ev0) == hipSuccess && e < 0.f) ref = q.get();
        }
        float a = 0.f, b = 0.f;
        if (hipSetDevice(p->dev) != hipSuccess || hipEventElapsedTime(&a, ref->r->ev0, p->r->ev0) != hipSuccess ||
            hipEventElapsedTime(&b, ref->r->ev0, p->r->ev1) != hipSuccess)
            a = b = -1.f;
        tv.push_back(ShardTime{p->dev, (double)a, (double)b});
    }
    std::lock_guard<std::mutex> lk(g_times_mu);
    g_times.swap(tv);
    return EZ_OK;
}
}  // namespace

// Introspection (tests, measurement): the shards of the last multi-device call and their device
// intervals (ms from the earliest shard start on the same device; -1 if not measurable)
extern "C" int ez_multi_last_shards(int *dev, double *t0, double *t1, int cap) {
    std::lock_guard<std::mutex> lk(g_times_mu);
    const int n = (int)g_times.size();
    for (int k = 0; k < n && k < cap; k++) {
        if (dev) dev[k] = g_times[(size_t)k].dev;
        if (t0) t0[k] = g_times[(size_t)k].t0;
        if (t1) t1[k] = g_times[(size_t)k].t1;
    }
    return n;
}

#define EZ_SHARD_HIP(x)                          \
    do {                                         \
        if ((x) != hipSuccess) return EZ_EDEVICE; \
    } while (0)

extern "C" int ez_compress_batch_multi(int64_t block, int64_t htable, int flags, const uint8_t *in, const uint64_t *in_off,
                                       uint64_t count, const int *devices, int ndev, uint8_t *packed, uint64_t packed_cap,
                                       uint64_t *packed_off, int32_t *status) {
    if (!valid_writer_sizes(block, htable) || !in_off || !packed_off) return EZ_EINVAL;
    std::vector<int> devs;
    int e = resolve_devices(devices, ndev, devs);
    if (e != EZ_OK) return e;
    packed_off[0] = 0;
    if (count == 0) return EZ_OK;
    DeviceGuard keep(-1);  // (the shards' buffers are freed on this thread, each on its device)
    try {
        const std::vector<uint64_t> first = shard_bounds(in_off, count, (int)devs.size());
        std::vector<std::unique_ptr<Shard>> sh;
        for (size_t k = 0; k < devs.size(); k++) {
            sh.emplace_back(new Shard());
            sh[k]->dev = devs[k];
            sh[k]->first = first[k];
            sh[k]->count = first[k + 1] - first[k];
        }
        // phase 1: per shard, upload, K1 into bound-sized slots, K3 into a packed shard; its sizes back
        e = each_shard(sh, [&](Shard &x) -> int {
            const uint64_t c = x.count, base = in_off[x.first], nb = in_off[x.first + c] - base;
            std::vector<uint64_t> ioff(c + 1), ooff(c + 1);
            uint64_t mx = 0;
            ooff[0] = 0;
            for (uint64_t t = 0; t <= c; t++) ioff[t] = in_off[x.first + t] - base;
            for (uint64_t t = 0; t < c; t++) {
                const uint64_t n = ioff[t + 1] - ioff[t];
                mx = n > mx ? n : mx;
                ooff[t + 1] = ooff[t] + ((ez_compress_bound(n) + 15) & ~15ull);
            }
            if (x.r->in.ensure(nb + 64) || x.r->in_off.ensure(8 * (c + 1)) || x.r->out.ensure(ooff[c] + 64) || x.r->out_off.ensure(8 * (c + 1)) ||
                x.r->size.ensure(8 * c) || x.r->status.ensure(4 * c) || x.r->ws.ensure(ez_pack_workspace(c) + 64) || x.r->packed.ensure(ooff[c] + 64) ||
                x.r->packed_off.ensure(8 * (c + 1)))
                return EZ_EDEVICE;
            if (nb) EZ_SHARD_HIP(hipMemcpyAsync(x.r->in.p, in + base, nb, hipMemcpyHostToDevice, x.r->st));
            EZ_SHARD_HIP(hipMemcpyAsync(x.r->in_off.p, ioff.data(), 8 * (c + 1), hipMemcpyHostToDevice, x.r->st));
            EZ_SHARD_HIP(hipMemcpyAsync(x.r->out_off.p, ooff.data(), 8 * (c + 1), hipMemcpyHostToDevice, x.r->st));
            ez_batch b{x.r->in.as<uint8_t>(), x.r->in_off.as<uint64_t>(), x.r->out.as<uint8_t>(), x.r->out_off.as<uint64_t>(),
                       x.r->size.as<uint64_t>(), x.r->status.as<int32_t>(), c, mx};
            int r = ez_compress_batch(block, htable, flags, &b, x.r->st);
            if (r != EZ_OK) return r;
            r = ez_pack_batch(x.r->out.as<uint8_t>(), x.r->out_off.as<uint64_t>(), x.r->size.as<uint64_t>(), c, x.r->packed.as<uint8_t>(),
                              x.r->packed_off.as<uint64_t>(), x.r->ws.p, x.r->st);
            if (r != EZ_OK) return r;
            // the shard's packed offsets straight into the caller's array (rebased below; its last one,
            // the shard's total, is the next shard's first entry and comes back separately)
            EZ_SHARD_HIP(hipMemcpyAsync(packed_off + x.first, x.r->packed_off.p, 8 * c, hipMemcpyDeviceToHost, x.r->st));
            EZ_SHARD_HIP(hipMemcpyAsync(&x.total, x.r->packed_off.as<uint64_t>() + c, 8, hipMemcpyDeviceToHost, x.r->st));
            if (status) EZ_SHARD_HIP(hipMemcpyAsync(status + x.first, x.r->status.p, 4 * c, hipMemcpyDeviceToHost, x.r->st));
            EZ_SHARD_HIP(hipStreamSynchronize(x.r->st));
            return EZ_OK;
        });
        if (e != EZ_OK) return e;
        // the global packing: shard k starts where shard k-1 ends (a host exclusive scan of the totals)
        uint64_t at = 0;
        for (auto &x : sh) {
            x->base = at;
            at += x->total;
            for (uint64_t t = 0; t < x->count; t++) packed_off[x->first + t] += x->base;
        }
        packed_off[count] = at;
        if (at > packed_cap) return EZ_ENOSPC;
        // phase 2: every shard's packed bytes down to its place
        return each_shard(sh, [&](Shard &x) -> int {
            if (x.total) EZ_SHARD_HIP(hipMemcpyAsync(packed + x.base, x.r->packed.p, x.total, hipMemcpyDeviceToHost, x.r->st));
            EZ_SHARD_HIP(hipStreamSynchronize(x.r->st));
            return EZ_OK;
        }, false);
    } catch (...) {
        return EZ_EDEVICE;  // (host allocation failure: nothing unwinds across the C-ABI)
    }
}

extern "C" int ez_decompress_batch_multi(int64_t block_size_limit, const uint8_t *in, const uint64_t *in_off, uint64_t count,
                                         const int *devices, int ndev, uint8_t *out, const uint64_t *out_off, uint64_t *out_size,
                                         int32_t *status) {
    if (!in_off || !out_off || !out_size) return EZ_EINVAL;
    std::vector<int> devs;
    int e = resolve_devices(devices, ndev, devs);
    if (e != EZ_OK) return e;
    if (count == 0) return EZ_OK;
    DeviceGuard keep(-1);
    try {
        const std::vector<uint64_t> first = shard_bounds(in_off, count, (int)devs.size());
        std::vector<std::unique_ptr<Shard>> sh;
        for (size_t k = 0; k < devs.size(); k++) {
            sh.emplace_back(new Shard());
            sh[k]->dev = devs[k];
            sh[k]->first = first[k];
            sh[k]->count = first[k + 1] - first[k];
        }
        return each_shard(sh, [&](Shard &x) -> int {
            const uint64_t c = x.count, ib = in_off[x.first], nb = in_off[x.first + c] - ib;
            const uint64_t ob = out_off[x.first], no = out_off[x.first + c] - ob;
            std::vector<uint64_t> ioff(c + 1), ooff(c + 1);
            uint64_t mx = 0;
            for (uint64_t t = 0; t <= c; t++) {
                ioff[t] = in_off[x.first + t] - ib;
                ooff[t] = out_off[x.first + t] - ob;
                if (t) mx = ooff[t] - ooff[t - 1] > mx ? ooff[t] - ooff[t - 1] : mx;
            }
            if (x.r->in.ensure(nb + 64) || x.r->in_off.ensure(8 * (c + 1)) || x.r->out.ensure(no + 64) || x.r->out_off.ensure(8 * (c + 1)) ||
                x.r->size.ensure(8 * c) || x.r->status.ensure(4 * c) || x.r->ws.ensure(ez_decompress_workspace(c) + 64))
                return EZ_EDEVICE;
            if (nb) EZ_SHARD_HIP(hipMemcpyAsync(x.r->in.p, in + ib, nb, hipMemcpyHostToDevice, x.r->st));
            EZ_SHARD_HIP(hipMemcpyAsync(x.r->in_off.p, ioff.data(), 8 * (c + 1), hipMemcpyHostToDevice, x.r->st));
            EZ_SHARD_HIP(hipMemcpyAsync(x.r->out_off.p, ooff.data(), 8 * (c + 1), hipMemcpyHostToDevice, x.r->st));
            // (the largest slot and the extents given: the decoder route needs no device read-back)
            ez_batch b{x.r->in.as<uint8_t>(), x.r->in_off.as<uint64_t>(), x.r->out.as<uint8_t>(), x.r->out_off.as<uint64_t>(),
                       x.r->size.as<uint64_t>(), x.r->status.as<int32_t>(), c, mx ? mx : 1, nb, no};
            const int r = ez_decompress_batch(block_size_limit, &b, x.r->ws.p, x.r->st);
            if (r != EZ_OK) return r;
            if (no) EZ_SHARD_HIP(hipMemcpyAsync(out + ob, x.r->out.p, no, hipMemcpyDeviceToHost, x.r->st));
            EZ_SHARD_HIP(hipMemcpyAsync(out_size + x.first, x.r->size.p, 8 * c, hipMemcpyDeviceToHost, x.r->st));
            if (status) EZ_SHARD_HIP(hipMemcpyAsync(status + x.first, x.r->status.p, 4 * c, hipMemcpyDeviceToHost, x.r->st));
            EZ_SHARD_HIP(hipStreamSynchronize(x.r->st));
            return EZ_OK;
        });
    } catch (...) {
        return EZ_EDEVICE;
    }
}

// Frees the device scratch the batch calls keep between calls (no reference counterpart; like a
// caching allocator's empty_cache): the K1 / K1c scratch and K2j workspaces per (device, HIP stream),
// the multi-device calls' pooled shard buffers and the Reader handles' shared K2j workspace, on
// `device` (< 0: every device).  Scratch a call is using at that moment is kept.
extern "C" int ez_release_cached(int device) {
    const int have = device_count();
    if (have <= 0) return EZ_EDEVICE;
    if (device >= have) return EZ_EINVAL;
    DeviceGuard keep(-1);
    for (int d = device < 0 ? 0 : device; d < (device < 0 ? have : device + 1); d++) {
        if (hipSetDevice(d) != hipSuccess) return EZ_EDEVICE;
        k1_cache().trim(d);
        ez::jump_cache().trim(d);
        ReaderJws &J = reader_jws(d);
        if (J.mu.try_lock()) {
            J.buf.release();
            J.mu.unlock();
        }
    }
    shard_pool().trim(device);
    return EZ_OK;
}
