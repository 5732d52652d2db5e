// Which XCDs a CU-masked stream's workgroups land on (hipExtStreamCreateWithCUMask): the mask's bit layout against
// the XCC id each workgroup reads (s_getreg XCC_ID). Prints, per mask, the histogram of XCC ids and of (XCC, CU).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void probe(unsigned* out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);   // HW_REG_XCC_ID
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
    // hold the CU a little so that the workgroups spread
    for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(1);
}

int main() {
    int dev = 0;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, dev);
    const int ncu = prop.multiProcessorCount;
    printf("CUs %d\n", ncu);
    const int words = (ncu + 31) / 32;
    const int nblk = 4096;
    unsigned* d;
    hipMalloc(&d, 2 * nblk * sizeof(unsigned));
    const char* names[] = {"first half", "i % 8 < 4", "even", "i % 16 < 8", "first quarter"};
    for (int m = 0; m < 5; ++m) {
        std::vector<uint32_t> mask(words, 0u);
        for (int i = 0; i < ncu; ++i) {
            bool on = false;
            if (m == 0) on = i < ncu / 2;
            if (m == 1) on = (i % 8) < 4;
            if (m == 2) on = (i % 2) == 0;
            if (m == 3) on = (i % 16) < 8;
            if (m == 4) on = i < ncu / 4;
            if (on) mask[i / 32] |= 1u << (i % 32);
        }
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, words, mask.data()) != hipSuccess) { printf("mask %d: create failed\n", m); continue; }
        hipMemset(d, 0xff, 2 * nblk * sizeof(unsigned));
        hipLaunchKernelGGL(probe, dim3(nblk), dim3(64), 0, s, d);
        hipStreamSynchronize(s);
        std::vector<unsigned> h(2 * nblk);
        hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
        int cnt[16] = {0};
        std::vector<int> cus(16 * 64, 0);
        for (int b = 0; b < nblk; ++b) {
            const unsigned x = h[2 * b] & 15u, hw = h[2 * b + 1];
            cnt[x]++;
            const unsigned cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
            cus[x * 64 + ((se * 2 + sh) * 16 + cu) % 64] = 1;
        }
        printf("mask %-14s xcc histogram:", names[m]);
        for (int x = 0; x < 8; ++x) printf(" %d", cnt[x]);
        printf(" | distinct CUs per xcc:");
        for (int x = 0; x < 8; ++x) {
            int n = 0;
            for (int c = 0; c < 64; ++c) n += cus[x * 64 + c];
            printf(" %d", n);
        }
        printf("\n");
        hipStreamDestroy(s);
    }
    hipFree(d);
    return 0;
}
