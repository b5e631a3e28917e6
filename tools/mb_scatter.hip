// microbenchmark: cost of per-lane scattered dependent loads/stores (one stream per lane)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef uint4 __attribute__((aligned(1))) uint4_u;

template <int MODE>
__global__ void chain(const uint8_t *base, uint8_t *outb, int iters, int lanes, long long *cyc, unsigned *sink) {
    const int lane = threadIdx.x & 63;
    const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= lanes) return;
    const uint8_t *p = base + s * 4096;
    uint8_t *o = outb + s * 4096;
    unsigned x = (unsigned)(s * 2654435761u);
    long long t0 = clock64();
    for (int k = 0; k < iters; k++) {
        unsigned off = (x * 16u + (unsigned)k * 48u) & 4080u;
        if (MODE == 0) {  // 16B aligned dependent load
            uint4 v = *(const uint4 *)(p + off);
            x ^= v.x + v.w;
        } else if (MODE == 1) {  // 16B unaligned dependent load
            uint4 v = *(const uint4_u *)(p + off + (x & 7) % 8);
            x ^= v.x + v.w;
        } else if (MODE == 2) {  // 4B dependent load
            x ^= *(const unsigned *)(p + off);
        } else if (MODE == 3) {  // 16B load + 16B store (decoder-like)
            uint4 v = *(const uint4 *)(p + off);
            *(uint4 *)(o + ((k * 16) & 4080)) = v;
            x ^= v.x + v.w;
        } else if (MODE == 4) {  // 2 independent 16B loads then use
            uint4 v = *(const uint4 *)(p + off);
            uint4 w = *(const uint4 *)(p + ((off + 1024) & 4080));
            x ^= v.x + w.w;
        }
    }
    long long t1 = clock64();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    sink[s] = x;
}

int main(int argc, char **argv) {
    const long nstreams = 262144;
    uint8_t *base, *outb;
    hipMalloc(&base, nstreams * 4096);
    hipMalloc(&outb, nstreams * 4096);
    hipMemset(base, 1, nstreams * 4096);
    long long *cyc;
    unsigned *sink;
    hipMalloc(&cyc, 65536 * 8);
    hipMalloc(&sink, nstreams * 4);
    const int iters = 2000;
    int waves_list[] = {1, 16, 256, 1024, 2048, 4096};
    int lanes_list[] = {1, 8, 64};
    for (int mode = 0; mode < 5; mode++)
        for (int lanes : lanes_list)
            for (int waves : waves_list) {
                if (lanes != 64 && waves > 16) continue;
                auto run = [&]() {
                    switch (mode) {
                        case 0: hipLaunchKernelGGL(chain<0>, dim3(waves), dim3(64), 0, 0, base, outb, iters, lanes, cyc, sink); break;
                        case 1: hipLaunchKernelGGL(chain<1>, dim3(waves), dim3(64), 0, 0, base, outb, iters, lanes, cyc, sink); break;
                        case 2: hipLaunchKernelGGL(chain<2>, dim3(waves), dim3(64), 0, 0, base, outb, iters, lanes, cyc, sink); break;
                        case 3: hipLaunchKernelGGL(chain<3>, dim3(waves), dim3(64), 0, 0, base, outb, iters, lanes, cyc, sink); break;
                        case 4: hipLaunchKernelGGL(chain<4>, dim3(waves), dim3(64), 0, 0, base, outb, iters, lanes, cyc, sink); break;
                    }
                };
                run();
                hipDeviceSynchronize();
                hipEvent_t e0, e1;
                hipEventCreate(&e0);
                hipEventCreate(&e1);
                hipEventRecord(e0);
                run();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                std::vector<long long> c(waves);
                hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost);
                double avg = 0;
                for (auto v : c) avg += v;
                avg /= waves;
                printf("mode %d lanes %2d waves %4d: %.3f ms, %.0f cycles/iter (clock64)\n", mode, lanes, waves, ms, avg / iters);
            }
    return 0;
}
