// VALU issue-rate probe for gfx950 (the SALU filler is s_movk_i32: it must not write SCC, which the loop branch reads): how many wave64 VALU instructions per second the chip sustains
// with W waves per SIMD, for independent v_add_f32 / v_pk_add_f32 / v_fma_f32 streams and for a
// VALU stream interleaved with SALU. Used to read the render kernel's PMC instruction counts as a
// fraction of the issue ceiling. Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP2(x) x x

template <int KIND>
__global__ __launch_bounds__(256) void probe(float* out, int iters) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float b = 1e-7f;
    int s = 0;
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0) {   // 16 independent v_add_f32 per iteration
            asm volatile(REP2("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n"
                              "v_add_f32 %3, %3, %8\n v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n"
                              "v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        } else if (KIND == 1) {   // 16 v_pk_add_f32 on 4 independent register pairs
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
            const f2 q = {b, b};
            asm volatile(REP8("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n"
                              "v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n")
                         : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(q));
            a0 = p0.x; a1 = p0.y; a2 = p1.x; a3 = p1.y; a4 = p2.x; a5 = p2.y; a6 = p3.x; a7 = p3.y;
        } else if (KIND == 2) {   // 16 v_fma_f32
            asm volatile(REP2("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n"
                              "v_fma_f32 %3, %3, %8, %8\n v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n"
                              "v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        } else {           // 16 v_add_f32 + 8 s_add_u32
            asm volatile(REP2("v_add_f32 %0, %0, %9\n s_movk_i32 %8, 0x1\n v_add_f32 %1, %1, %9\n"
                              "v_add_f32 %2, %2, %9\n s_movk_i32 %8, 0x1\n v_add_f32 %3, %3, %9\n"
                              "v_add_f32 %4, %4, %9\n s_movk_i32 %8, 0x1\n v_add_f32 %5, %5, %9\n"
                              "v_add_f32 %6, %6, %9\n s_movk_i32 %8, 0x1\n v_add_f32 %7, %7, %9\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+s"(s)
                         : "v"(b));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)s;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float) * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    const char* names[] = {"v_add_f32", "v_pk_add_f32", "v_fma_f32", "v_add_f32+salu"};
    for (int kind = 0; kind < 4; ++kind)
        for (int wps : {1, 2, 4, 5, 8}) {   // waves per SIMD: blocks of 4 waves, one block per SIMD-quad
            const int blocks = cus * wps;
            auto run = [&]() {
                if (kind == 0) probe<0><<<blocks, 256>>>(out, iters);
                if (kind == 1) probe<1><<<blocks, 256>>>(out, iters);
                if (kind == 2) probe<2><<<blocks, 256>>>(out, iters);
                if (kind == 3) probe<3><<<blocks, 256>>>(out, iters);
            };
            run();
            hipEventRecord(e0);
            run();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double winstr = (double)blocks * 4 * iters * (kind == 1 ? 32 : 16);
            printf("%-16s waves/SIMD %d: %.3f ms, %.1f G wave-VALU/s, %.2f VALU per SIMD-cycle at 2.4 GHz\n",
                   names[kind], wps, ms, winstr / ms / 1e6, winstr / (ms * 1e-3) / (cus * 4.0 * 2.4e9));
        }
    return 0;
}
