// Host emulation of the lane-per-stream kernels' per-lane code (K1 lane):
// the same source, compiled for the CPU, run stream by stream.  Debug aid:
//   lane_emu <in.bin> <offs.bin (u64 count+1)> <block> <htable> <out.bin> <sizes.bin>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../eazy_amd/csrc/ez_compress_lane.hip"

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
    if (argc < 7) return 2;
    auto in = slurp(argv[1]);
    auto ob = slurp(argv[2]);
    const uint64_t *offs = (const uint64_t *)ob.data();
    const uint64_t count = ob.size() / 8 - 1;
    in.resize(in.size() + 64);
    std::vector<uint64_t> out_off(count + 1, 0), size(count);
    for (uint64_t s = 0; s < count; s++) out_off[s + 1] = out_off[s] + ((offs[s + 1] - offs[s]) * 5 / 4 + 48) / 16 * 16;
    std::vector<uint8_t> out(out_off[count] + 64);
    std::vector<int32_t> st(count);
    ez::CompressArgs a{};
    a.in = in.data();
    a.in_off = offs;
    a.out = out.data();
    a.out_off = out_off.data();
    a.out_size = size.data();
    a.status = st.data();
    a.count = count;
    a.bs = atoll(argv[3]);
    a.hs = atoll(argv[4]);
    a.append_magic = 1;
    std::vector<uint16_t> ht(a.hs);
    for (uint64_t s = 0; s < count; s++) ez::lane_one(a, ht.data(), s);
    FILE *fo = std::fopen(argv[5], "wb");
    for (uint64_t s = 0; s < count; s++) std::fwrite(out.data() + out_off[s], 1, size[s], fo);
    std::fclose(fo);
    FILE *fs = std::fopen(argv[6], "wb");
    std::fwrite(size.data(), 8, count, fs);
    std::fclose(fs);
    return 0;
}
