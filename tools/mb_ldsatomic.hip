// micro-test: order of same-address LDS atomics within one wave instruction
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned *out, int mode) {
    __shared__ unsigned t[64];
    int l = threadIdx.x;
    if (l < 64) t[l] = 0;
    __syncthreads();
    unsigned a = mode == 0 ? 0 : (l % 3);   // address
    unsigned v = mode == 2 ? (unsigned)(100 - l) : (unsigned)(l + 1);
    unsigned old = atomicMax(&t[a], v);
    out[l] = old;
    __syncthreads();
    if (l < 4) out[64 + l] = t[l];
}
int main() {
    unsigned *d, h[68];
    hipMalloc(&d, 68 * 4);
    for (int mode = 0; mode < 3; mode++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h, d, 68 * 4, hipMemcpyDeviceToHost);
        printf("mode %d:", mode);
        for (int i = 0; i < 68; i++) printf(" %u", h[i]);
        printf("\n");
    }
    return 0;
}
