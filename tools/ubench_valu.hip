// Microbenchmark: issue throughput of the VALU instructions the scan and BLAKE3
// kernels use, on MI355X.  Each lane runs 8 independent chains (ILP 8) of one
// instruction (or 1 dependent chain, "dep"), at 1 / 2 / 4 waves per SIMD.
// Reports wave-instructions per ns per SIMD and the shader clock measured in
// the kernel (s_memtime / s_memrealtime at 100 MHz), hence cycles per
// wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o build/ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP8(INSN)                                                                    \
    asm volatile(INSN " %0, %0, %8\n\t" INSN " %1, %1, %8\n\t" INSN " %2, %2, %8\n\t" \
                 INSN " %3, %3, %8\n\t" INSN " %4, %4, %8\n\t" INSN " %5, %5, %8\n\t" \
                 INSN " %6, %6, %8\n\t" INSN " %7, %7, %8"                             \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(k))
#define OP8_3(INSN)                                                                              \
    asm volatile(INSN " %0, %0, %8, %0\n\t" INSN " %1, %1, %8, %1\n\t" INSN " %2, %2, %8, %2\n\t" \
                 INSN " %3, %3, %8, %3\n\t" INSN " %4, %4, %8, %4\n\t" INSN " %5, %5, %8, %5\n\t" \
                 INSN " %6, %6, %8, %6\n\t" INSN " %7, %7, %8, %7"                                 \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(k))
#define ROT8(N)                                                                                    \
    asm volatile("v_alignbit_b32 %0, %0, %0, " #N "\n\tv_alignbit_b32 %1, %1, %1, " #N "\n\t"      \
                 "v_alignbit_b32 %2, %2, %2, " #N "\n\tv_alignbit_b32 %3, %3, %3, " #N "\n\t"      \
                 "v_alignbit_b32 %4, %4, %4, " #N "\n\tv_alignbit_b32 %5, %5, %5, " #N "\n\t"      \
                 "v_alignbit_b32 %6, %6, %6, " #N "\n\tv_alignbit_b32 %7, %7, %7, " #N              \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7))
#define DEP8(INSN)                                                                   \
    asm volatile(INSN " %0, %0, %1\n\t" INSN " %0, %0, %1\n\t" INSN " %0, %0, %1\n\t" \
                 INSN " %0, %0, %1\n\t" INSN " %0, %0, %1\n\t" INSN " %0, %0, %1\n\t" \
                 INSN " %0, %0, %1\n\t" INSN " %0, %0, %1"                             \
                 : "+v"(a0) : "v"(k))

#define SDWA8(INSN)                                                                                    \
    asm volatile(INSN " %0, %0, %8 src1_sel:BYTE_1\n\t" INSN " %1, %1, %8 src1_sel:BYTE_1\n\t"             \
                 INSN " %2, %2, %8 src1_sel:BYTE_1\n\t" INSN " %3, %3, %8 src1_sel:BYTE_1\n\t"             \
                 INSN " %4, %4, %8 src1_sel:BYTE_1\n\t" INSN " %5, %5, %8 src1_sel:BYTE_1\n\t"             \
                 INSN " %6, %6, %8 src1_sel:BYTE_1\n\t" INSN " %7, %7, %8 src1_sel:BYTE_1"                   \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(k))

constexpr int NOPS = 15;
const char *names[NOPS] = {"v_add_u32", "v_xor_b32", "v_add3_u32", "v_alignbit_b32(12)", "v_pk_add_u16",
                           "v_pk_mad_u16", "v_pk_min_u16", "v_perm_b32", "v_dot4_u32_u8", "v_lshl_add_u32",
                           "dep v_add_u32", "dep v_xor_b32", "v_add_u32_e64", "v_add_u32_sdwa", "v_min_u16"};

template <int OP>
__global__ __launch_bounds__(256) void kern(unsigned *out, unsigned long long *clk, unsigned seed, int iters) {
    unsigned a0 = seed ^ threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7, k = seed * 3 + 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) OP8("v_add_u32");
        if (OP == 1) OP8("v_xor_b32");
        if (OP == 2) OP8_3("v_add3_u32");
        if (OP == 3) ROT8(12);
        if (OP == 4) OP8("v_pk_add_u16");
        if (OP == 5) OP8_3("v_pk_mad_u16");
        if (OP == 6) OP8("v_pk_min_u16");
        if (OP == 7) OP8_3("v_perm_b32");
        if (OP == 8) OP8_3("v_dot4_u32_u8");
        if (OP == 9) OP8_3("v_lshl_add_u32");
        if (OP == 10) DEP8("v_add_u32");
        if (OP == 11) DEP8("v_xor_b32");
        if (OP == 12) OP8("v_add_u32_e64");
        if (OP == 13) SDWA8("v_add_u32_sdwa");
        if (OP == 14) OP8("v_min_u16");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int OP>
void run(unsigned *d, unsigned long long *clk, int cus, int per_simd, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = cus * per_simd;                  // 256 threads = one wave per SIMD per block
    kern<OP><<<blocks, 256>>>(d, clk, 7, iters);
    hipEventRecord(e0);
    kern<OP><<<blocks, 256>>>(d, clk, 7, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    hipMemcpy(c, clk, sizeof c, hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;      // memrealtime: 100 MHz
    const double winsts = (double)blocks * 4 * iters * 8;                 // wave-instructions
    const double per_simd_ns = winsts / (cus * 4.0) / (ms * 1e6);
    printf("%-20s waves/SIMD %d: %.3f wave-instr/ns/SIMD  clock %.2f GHz  -> %.2f cycles per wave-instr per SIMD\n",
           names[OP], per_simd, per_simd_ns, ghz, ghz / per_simd_ns);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int OP>
void all(unsigned *d, unsigned long long *clk, int cus) {
    for (int w : {1, 2, 3, 4}) run<OP>(d, clk, cus, w, 20000);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *d;
    unsigned long long *clk;
    hipMalloc(&d, (size_t)cus * 4 * 256 * 4);
    hipMalloc(&clk, 16);
    all<0>(d, clk, cus); all<1>(d, clk, cus); all<2>(d, clk, cus); all<3>(d, clk, cus);
    all<4>(d, clk, cus); all<5>(d, clk, cus); all<6>(d, clk, cus); all<7>(d, clk, cus);
    all<8>(d, clk, cus); all<9>(d, clk, cus); all<10>(d, clk, cus); all<11>(d, clk, cus);
    all<12>(d, clk, cus); all<13>(d, clk, cus); all<14>(d, clk, cus);
    hipFree(d);
    hipFree(clk);
    return 0;
}
