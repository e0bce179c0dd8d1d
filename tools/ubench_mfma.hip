// Microbenchmark: v_mfma_i32_32x32x32_i8 on MI355X.
//   mode 0: 4 independent accumulators per wave (throughput)
//   mode 1: one dependent accumulator chain (srcC = previous result)
//   mode 2: chains of 3 dependent MFMAs from a fixed C, each followed by
//           8 VALU reads of the result (the scan filter's shape)
// Reports wave-MFMAs per microsecond per CU and cycles per MFMA per SIMD
// (at an assumed 2.4 GHz), for 1..4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/ubench_mfma.hip -o tools/bin/ubench_mfma
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256) void kern(int *out, int seed, int iters) {
    const int l = threadIdx.x;
    v4i a = {seed ^ l, seed + l, seed * 3, l}, b = {l, seed, seed ^ 5, 7};
    v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
    unsigned acc = 0xffff;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
        } else if (MODE == 1) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c0, 0, 0, 0);
        } else {
            v16i d = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
            d = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, d, 0, 0, 0);
#pragma unroll
            for (int v = 0; v < 16; v += 2) {
                const unsigned short x = (unsigned short)d[v], y = (unsigned short)d[v + 1];
                acc = __builtin_elementwise_min(__builtin_elementwise_min((unsigned short)acc, x), y);
            }
            a.x += (int)acc;
        }
    }
    int r = (int)acc;
    for (int v = 0; v < 16; ++v) r ^= c0[v] ^ c1[v] ^ c2[v] ^ c3[v];
    out[blockIdx.x * blockDim.x + l] = r;
}

template <int MODE>
void run(int *d, int cus, int wps, int iters) {
    const int per_block = 4;                 // waves per block (one per SIMD)
    const int blocks = cus * wps;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<MODE><<<blocks, 64 * per_block>>>(d, 7, iters);
    hipEventRecord(e0);
    kern<MODE><<<blocks, 64 * per_block>>>(d, 7, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double mf = (double)blocks * per_block * iters * (MODE == 2 ? 3 : 4);
    const double per_cu_us = mf / cus / (ms * 1e3);
    const double cyc = 2.4e3 / (per_cu_us / 4.0);
    printf("mode %d  waves/SIMD %d  %.1f wave-MFMA/us/CU  %.1f cycles/MFMA/SIMD\n", MODE, wps, per_cu_us, cyc);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int *d;
    if (hipMalloc(&d, 64 * 4 * cus * 8 * sizeof(int))) return 2;
    for (int w = 1; w <= 4; ++w) run<0>(d, cus, w, 20000);
    for (int w = 1; w <= 4; ++w) run<1>(d, cus, w, 20000);
    for (int w = 1; w <= 4; ++w) run<2>(d, cus, w, 20000);
    return 0;
}
