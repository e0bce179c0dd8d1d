// Microbenchmark: issue throughput of the VALU instructions the scan kernel
// uses, on MI355X.  Each lane runs 8 independent chains (ILP 8) of one
// instruction; reports instructions per cycle per CU at the measured clock-free
// rate (wave-instructions / s / CU).
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

template <int OP>
__global__ __launch_bounds__(256) void kern(unsigned *out, unsigned seed, int iters) {
    unsigned a0 = seed ^ threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7, k = seed * 3 + 1;
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) OP8("v_add_u32");
        if (OP == 1) OP8("v_pk_add_u16");
        if (OP == 2) OP8_3("v_pk_mad_u16");
        if (OP == 3) OP8("v_pk_min_u16");
        if (OP == 4) OP8_3("v_perm_b32");
        if (OP == 5) OP8_3("v_dot4_u32_u8");
        if (OP == 6) OP8("v_pk_sub_i16");
        if (OP == 7) OP8_3("v_lshl_add_u32");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
double run(unsigned *d, int blocks, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<OP><<<blocks, 256>>>(d, 7, iters);
    hipEventRecord(e0);
    kern<OP><<<blocks, 256>>>(d, 7, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double winsts = (double)blocks * 4 * iters * 8;        // wave-instructions
    return winsts / (ms * 1e-3);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char *names[] = {"v_add_u32", "v_pk_add_u16", "v_pk_mad_u16", "v_pk_min_u16",
                           "v_perm_b32", "v_dot4_u32_u8", "v_pk_sub_i16", "v_lshl_add_u32"};
    unsigned *d;
    const int iters = 20000;
    for (int wpc : {4, 8, 16}) {
        const int blocks = cus * wpc / 4;
        hipMalloc(&d, (size_t)blocks * 256 * 4);
        double r[8] = {run<0>(d, blocks, iters), run<1>(d, blocks, iters), run<2>(d, blocks, iters),
                       run<3>(d, blocks, iters), run<4>(d, blocks, iters), run<5>(d, blocks, iters),
                       run<6>(d, blocks, iters), run<7>(d, blocks, iters)};
        for (int i = 0; i < 8; i++)
            std::printf("waves/CU %2d  %-16s %8.3f Twave-inst/s  = %.3f wave-inst/ns/CU\n", wpc, names[i],
                        r[i] / 1e12, r[i] / 1e9 / cus);
        hipFree(d);
    }
    return 0;
}
