// Layout check for v_mfma_i32_32x32x32_i8 on gfx950 (exact integer data,
// asymmetric operands).  Assumed maps, the ones the MFMA scan relies on:
//   A: lane l (i = l&31, h = l>>5) byte j  = A[i][16h + j]
//   B: lane l (c = l&31, h = l>>5) byte j  = B[16h + j][c]
//   D: lane l reg v = D[(v&3) + 8(v>>2) + 4(l>>5)][l&31]
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/mfma_i8_check tools/mfma_i8_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const int8_t *A, const int8_t *B, int32_t *D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    union { v4i v; int8_t b[16]; } a, b;
    for (int j = 0; j < 16; ++j) {
        a.b[j] = A[r * 32 + 16 * h + j];
        b.b[j] = B[(16 * h + j) * 32 + r];
    }
    v16i c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a.v, b.v, c, 0, 0, 0);
    for (int v = 0; v < 16; ++v) D[((v & 3) + 8 * (v >> 2) + 4 * h) * 32 + r] = c[v];
}

int main() {
    int8_t A[1024], B[1024];
    int32_t D[1024], R[1024];
    srand(7);
    for (int i = 0; i < 1024; ++i) { A[i] = (int8_t)(rand() & 0xff); B[i] = (int8_t)(rand() & 0xff); }
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            int s = 0;
            for (int q = 0; q < 32; ++q) s += A[i * 32 + q] * B[q * 32 + j];
            R[i * 32 + j] = s;
        }
    int8_t *dA, *dB;
    int32_t *dD;
    if (hipMalloc(&dA, 1024) || hipMalloc(&dB, 1024) || hipMalloc(&dD, 4096)) return 2;
    hipMemcpy(dA, A, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    if (hipMemcpy(D, dD, 4096, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    int bad = 0;
    for (int i = 0; i < 1024; ++i) bad += D[i] != R[i];
    printf("mfma_i32_32x32x32_i8 layout check: %d / 1024 mismatches\n", bad);
    return bad != 0;
}
