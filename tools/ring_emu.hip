// Host emulation of the K2r decoder's per-lane code (ez_decompress_ring.hip):
// the same source, compiled for the CPU, run stream by stream.
//   ring_emu <in.bin> <offs.bin (u64 count+1)> <cap per stream> <out.bin> <sizes.bin (u64, ~0 = handed over)>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../eazy_amd/csrc/ez_decompress_ring.hip"

static std::vector<uint8_t> slurp(const char *f) {
    FILE *fp = std::fopen(f, "rb");
    std::vector<uint8_t> v;
    if (!fp) return v;
    std::fseek(fp, 0, SEEK_END);
    v.resize(std::ftell(fp));
    std::fseek(fp, 0, SEEK_SET);
    if (!v.empty() && std::fread(v.data(), 1, v.size(), fp) != v.size()) v.clear();
    std::fclose(fp);
    return v;
}

int main(int argc, char **argv) {
    if (argc < 6) return 2;
    const bool hw = argc < 7 || atoi(argv[6]) != 0;  // the aligned header window (default) or the per-token load
    auto in = slurp(argv[1]);
    auto ob = slurp(argv[2]);
    const uint64_t *offs = (const uint64_t *)ob.data();
    const uint64_t count = ob.size() / 8 - 1, cap = (uint64_t)atoll(argv[3]);
    std::vector<uint64_t> out_off(count + 1), size(count);
    for (uint64_t s = 0; s <= count; s++) out_off[s] = s * cap;
    std::vector<uint8_t> out(out_off[count] + 64);
    std::vector<int32_t> st(count);
    ez::DecompressArgs a{};
    a.in = in.data();
    a.in_off = offs;
    a.out = out.data();
    a.out_off = out_off.data();
    a.out_size = size.data();
    a.status = st.data();
    a.count = count;
    alignas(16) static uint8_t ring[1024];
    for (uint64_t s = 0; s < count; s++)
        if (!(hw ? ez::ring_one<true>(a, s, ring + 16) : ez::ring_one<false>(a, s, ring + 16))) size[s] = ~0ull;  // front guard
#ifndef __HIP_DEVICE_COMPILE__
    std::fprintf(stderr, "iterations per stream %.1f\n", (double)ez::g_ring_iters / (double)(count ? count : 1));
    const double c = (double)(count ? count : 1);
    std::fprintf(stderr, "per stream: live steps %.1f, inner moves HBM %.1f pattern %.1f ring %.1f; pairs %.1f, lone literals %.1f, lone copies %.1f\n",
                 ez::g_ring_stat[0] / c, ez::g_ring_stat[1] / c, ez::g_ring_stat[2] / c, ez::g_ring_stat[3] / c, ez::g_ring_stat[4] / c,
                 ez::g_ring_stat[5] / c, ez::g_ring_stat[6] / c);
#endif
    FILE *fo = std::fopen(argv[4], "wb");
    for (uint64_t s = 0; s < count; s++)
        if (size[s] != ~0ull) std::fwrite(out.data() + out_off[s], 1, size[s], fo);
    std::fclose(fo);
    FILE *fs = std::fopen(argv[5], "wb");
    std::fwrite(size.data(), 8, count, fs);
    std::fclose(fs);
    return 0;
}
