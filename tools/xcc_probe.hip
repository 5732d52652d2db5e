#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
}
int main() {
    unsigned* d; hipMalloc(&d, 4096 * 4);
    hipLaunchKernelGGL(k, dim3(4096), dim3(64), 0, 0, d);
    unsigned h[4096]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int cnt[16] = {0}; int mism = 0;
    for (int i = 0; i < 4096; ++i) { cnt[h[i] & 15]++; if ((h[i] & 7) != ((h[0] + i) & 7)) ++mism; }
    for (int i = 0; i < 16; ++i) printf("%d ", cnt[i]);
    printf("\nfirst: %u %u %u %u %u %u %u %u %u; mismatch vs (b + c) %% 8: %d\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], mism);
    return 0;
}
