/*
 * synth.c — seeded synthetic inputs for tests and bench.py (not the codec).
 *
 * ez_synth_logs: tlwire-like log events mirroring the framing the
 * reference's file tests split on (eazy_test.go:1273-1282):
 *   bf 62 "_t" c2 1b <8-byte BE ns timestamp, +U(1,1e6)>
 *   62 "_m" <str "message" from 6 constants>
 *   65 "level" <str>  62 "ip" <str 10.0.x.y>  64 "path" <str /api/...>
 *   65 "trace" <str 16 hex>  63 "dur" <str N "us">  ff
 * concatenated into one buffer of exactly n bytes.
 */
#include <stdint.h>
#include <string.h>

static uint64_t xs(uint64_t *s) { /* xorshift64* */
    uint64_t x = *s;
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    *s = x;
    return x * 0x2545F4914F6CDD1DULL;
}
static uint64_t rnd(uint64_t *s, uint64_t n) { return xs(s) % n; }

static size_t put(uint8_t *b, size_t k, const void *p, size_t n) { memcpy(b + k, p, n); return k + n; }
static size_t put_str(uint8_t *b, size_t k, const char *p, size_t n) {
    if (n < 24) b[k++] = (uint8_t)(0x60 + n);
    else { b[k++] = 0x78; b[k++] = (uint8_t)n; }
    return put(b, k, p, n);
}

static const char *MSGS[] = {"request handled", "cache miss", "db query done", "user login", "retrying upstream",
                             "connection reset by peer"};
static const char *LEVELS[] = {"info", "info", "info", "debug", "warn", "error"};
static const char *PATHS[] = {"/api/v1/users/", "/api/v1/orders/", "/api/v2/items/", "/healthz", "/api/v1/search?q=",
                              "/static/app.js?v="};

/* one event into e (<= 256 bytes); returns its length */
static size_t event(uint8_t *e, uint64_t *s, uint64_t *ts) {
    char tmp[64];
    size_t k = 0;
    const uint8_t hdr[6] = {0xbf, 0x62, '_', 't', 0xc2, 0x1b};
    k = put(e, k, hdr, 6);
    *ts += 1 + rnd(s, 1000000);
    for (int j = 7; j >= 0; j--) e[k++] = (uint8_t)(*ts >> (8 * j));
    k = put_str(e, k, "_m", 2);
    const char *m = MSGS[rnd(s, 6)];
    k = put_str(e, k, m, strlen(m));
    k = put_str(e, k, "level", 5);
    const char *lv = LEVELS[rnd(s, 6)];
    k = put_str(e, k, lv, strlen(lv));
    k = put_str(e, k, "ip", 2);
    int n = 0;
    {
        unsigned a = (unsigned)rnd(s, 4), c = (unsigned)rnd(s, 256);
        char *p = tmp;
        memcpy(p, "10.0.", 5); p += 5;
        p += (a >= 10 ? 2 : 1); { unsigned v = a; char *q = p; do { *--q = (char)('0' + v % 10); v /= 10; } while (v); }
        *p++ = '.';
        { unsigned v = c, d = v >= 100 ? 3 : v >= 10 ? 2 : 1; char *q = p + d; p += d; do { *--q = (char)('0' + v % 10); v /= 10; } while (v); }
        n = (int)(p - tmp);
    }
    k = put_str(e, k, tmp, (size_t)n);
    k = put_str(e, k, "path", 4);
    {
        const char *pp = PATHS[rnd(s, 6)];
        size_t l = strlen(pp);
        memcpy(tmp, pp, l);
        unsigned id = (unsigned)rnd(s, 100000);
        char num[12]; int d = 0;
        do { num[d++] = (char)('0' + id % 10); id /= 10; } while (id);
        while (d) tmp[l++] = num[--d];
        n = (int)l;
    }
    k = put_str(e, k, tmp, (size_t)n);
    k = put_str(e, k, "trace", 5);
    {
        static const char hx[] = "0123456789abcdef";
        uint64_t t = xs(s);
        for (int j = 0; j < 16; j++) tmp[j] = hx[(t >> (4 * j)) & 15];
    }
    k = put_str(e, k, tmp, 16);
    k = put_str(e, k, "dur", 3);
    {
        unsigned v = (unsigned)rnd(s, 5001);
        char num[12]; int d = 0, l = 0;
        do { num[d++] = (char)('0' + v % 10); v /= 10; } while (v);
        while (d) tmp[l++] = num[--d];
        tmp[l++] = 'u'; tmp[l++] = 's';
        n = l;
    }
    k = put_str(e, k, tmp, (size_t)n);
    e[k++] = 0xff;
    return k;
}

/* fill out[0..n) with concatenated events (the last one truncated) */
void ez_synth_logs(uint64_t seed, uint8_t *out, uint64_t n) {
    uint64_t s = seed * 0x9E3779B97F4A7C15ULL + 0x1234567ULL;
    if (!s) s = 1;
    uint64_t ts = 1700000000000000000ULL + seed * 1000003ULL;
    uint8_t e[256];
    uint64_t k = 0;
    while (k < n) {
        size_t l = event(e, &s, &ts);
        if (l > n - k) l = (size_t)(n - k);
        memcpy(out + k, e, l);
        k += l;
    }
}

/* fp32 ~ N(0, sigma) (Irwin-Hall approximation), little-endian bytes */
void ez_synth_f32(uint64_t seed, float sigma, float *out, uint64_t count) {
    uint64_t s = seed * 0x9E3779B97F4A7C15ULL + 99;
    if (!s) s = 1;
    for (uint64_t i = 0; i < count; i++) {
        double acc = 0;
        for (int j = 0; j < 12; j++) acc += (double)(xs(&s) >> 11) * (1.0 / 9007199254740992.0);
        out[i] = (float)((acc - 6.0) * sigma);
    }
}
