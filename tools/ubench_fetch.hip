// Calibration of rocprofv3 FETCH_SIZE for the access patterns of this repo's
// kernels (MI355X_MICROARCH.md: "calibrate on a known byte count in your own
// access pattern").  Each kernel reads every byte of a 4 GiB buffer exactly once
// (known algorithmic bytes), so FETCH_SIZE * 1024 / bytes is the counter's scale
// for that pattern:
//   contig  : 1 KiB contiguous per wave instruction (16 B per lane) -- the scan's
//             LDS-DMA tiles and the read probe
//   leafpat : the BLAKE3 leaf's cooperative loader: per 64-byte block step, wave
//             instruction i reads 16 contiguous 64-byte runs, one per task
//             (tasks 16i..16i+15 of the wave's 64 tasks, 4 KiB apart)
//   run128  : 128-byte runs (whole lines), one per 8 lanes, runs 4 KiB apart
//   leaf_u  : leafpat with the wave's tasks starting 37 bytes past a line (a
//             chunk at an arbitrary batch offset): each 64-byte run spans two
//             64-byte sectors, the second re-read by the next block step
//   leafdma / leafdma_u : the same two patterns issued as global_load_lds_dwordx4
//             (the leaf kernel's actual instruction)
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_fetch.hip -o build/ubench_fetch
//   rocprofv3 --pmc FETCH_SIZE -- ./build/ubench_fetch
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void contig(const u32x4 *__restrict__ p, size_t nvec, unsigned *sink) {
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256)
        acc ^= __builtin_nontemporal_load(p + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345u) sink[blockIdx.x] = 1;
}

// one wave = 64 tasks x 4 KiB (256 KiB); 64 block steps of 64 B per task
__global__ __launch_bounds__(256) void leafpat(const unsigned char *__restrict__ p, size_t items, unsigned *sink) {
    const int lane = threadIdx.x & 63;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < items; w += (size_t)gridDim.x * 4) {
        const unsigned char *base = p + w * 262144;
        for (int t = 0; t < 64; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = 16 * i + (lane >> 2);
                acc ^= *(const u32x4 *)(base + (size_t)q * 4096 + t * 64 + (lane & 3) * 16);
            }
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345u) sink[blockIdx.x] = 1;
}

__global__ __launch_bounds__(256) void leaf_u(const unsigned char *__restrict__ p, size_t items, unsigned *sink) {
    const int lane = threadIdx.x & 63;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < items; w += (size_t)gridDim.x * 4) {
        const unsigned char *base = p + w * 262144 + 37;
        for (int t = 0; t < 64; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = 16 * i + (lane >> 2);
                u32x4 v;
                __builtin_memcpy(&v, base + (size_t)q * 4096 + t * 64 + (lane & 3) * 16, 16);
                acc ^= v;
            }
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345u) sink[blockIdx.x] = 1;
}

__device__ __forceinline__ void dma16(const unsigned char *gsrc, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}

template <int OFF>
__global__ __launch_bounds__(256) void leafdma(const unsigned char *__restrict__ p, size_t items, unsigned *sink) {
    __shared__ __attribute__((aligned(16))) unsigned stage[4 * 1024];
    const int lane = threadIdx.x & 63;
    const unsigned lds = (unsigned)__builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)(stage + (threadIdx.x >> 6) * 1024));
    unsigned acc = 0;
    for (size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < items; w += (size_t)gridDim.x * 4) {
        const unsigned char *base = p + w * 262144 + OFF;
        for (int t = 0; t < 64; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = 16 * i + (lane >> 2);
                dma16(base + (size_t)q * 4096 + t * 64 + (lane & 3) * 16, lds + i * 1024);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= stage[(threadIdx.x >> 6) * 1024 + lane * 16];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    if (acc == 0x12345u) sink[blockIdx.x] = 1;
}

// leafdma with 128 bytes per task per step (two BLAKE3 blocks per issue round),
// task stride STRIDE (4096 = the leaf; 4096+256 tests L2 set aliasing)
template <int OFF, int STRIDE>
__global__ __launch_bounds__(256) void dma128(const unsigned char *__restrict__ p, size_t items, unsigned *sink) {
    __shared__ __attribute__((aligned(16))) unsigned stage[8 * 1024];
    const int lane = threadIdx.x & 63;
    const unsigned lds = (unsigned)__builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)(stage + (threadIdx.x >> 6) * 2048));
    unsigned acc = 0;
    for (size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < items; w += (size_t)gridDim.x * 4) {
        const unsigned char *base = p + w * 64 * STRIDE + OFF;
        for (int t = 0; t < (STRIDE < 4096 ? STRIDE : 4096) / 128; ++t) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int q = 8 * i + (lane >> 3);
                dma16(base + (size_t)q * STRIDE + t * 128 + (lane & 7) * 16, lds + i * 1024);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= stage[(threadIdx.x >> 6) * 2048 + lane * 32];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    if (acc == 0x12345u) sink[blockIdx.x] = 1;
}

template <int OFF, int STRIDE>
__global__ __launch_bounds__(256) void dma64s(const unsigned char *__restrict__ p, size_t items, unsigned *sink) {
    __shared__ __attribute__((aligned(16))) unsigned stage[4 * 1024];
    const int lane = threadIdx.x & 63;
    const unsigned lds = (unsigned)__builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)(stage + (threadIdx.x >> 6) * 1024));
    unsigned acc = 0;
    for (size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < items; w += (size_t)gridDim.x * 4) {
        const unsigned char *base = p + w * 64 * STRIDE + OFF;
        for (int t = 0; t < (STRIDE < 4096 ? STRIDE : 4096) / 64; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = 16 * i + (lane >> 2);
                dma16(base + (size_t)q * STRIDE + t * 64 + (lane & 3) * 16, lds + i * 1024);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= stage[(threadIdx.x >> 6) * 1024 + lane * 16];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    if (acc == 0x12345u) sink[blockIdx.x] = 1;
}

// 128-byte runs (whole cache lines) 4 KiB apart: per 128-byte step, wave
// instruction i reads 8 runs of 128 B, one per task (tasks 8i..8i+7)
__global__ __launch_bounds__(256) void run128(const unsigned char *__restrict__ p, size_t items, unsigned *sink) {
    const int lane = threadIdx.x & 63;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); w < items; w += (size_t)gridDim.x * 4) {
        const unsigned char *base = p + w * 262144;
        for (int t = 0; t < 32; ++t) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int q = 8 * i + (lane >> 3);
                acc ^= *(const u32x4 *)(base + (size_t)q * 4096 + t * 128 + (lane & 7) * 16);
            }
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345u) sink[blockIdx.x] = 1;
}

int main() {
    const size_t bytes = 4ull << 30;
    unsigned char *p;
    unsigned *sink;
    if (hipMalloc(&p, bytes + 4096) != hipSuccess || hipMalloc(&sink, 1 << 20) != hipSuccess) return 1;
    (void)hipMemset(p, 1, bytes + 4096);
    (void)hipDeviceSynchronize();
    const size_t items = bytes / 262144;
    hipLaunchKernelGGL(contig, dim3(2048), dim3(256), 0, 0, (const u32x4 *)p, bytes / 16, sink);
    hipLaunchKernelGGL(leafpat, dim3(2048), dim3(256), 0, 0, p, items, sink);
    hipLaunchKernelGGL(run128, dim3(2048), dim3(256), 0, 0, p, items, sink);
    hipLaunchKernelGGL(leaf_u, dim3(2048), dim3(256), 0, 0, p, items, sink);
    hipLaunchKernelGGL(leafdma<0>, dim3(2048), dim3(256), 0, 0, p, items, sink);
    hipLaunchKernelGGL(leafdma<37>, dim3(2048), dim3(256), 0, 0, p, items, sink);
    // padded strides cover less than 4 GiB: items scaled so the bytes stay inside the buffer
    const size_t items_pad = bytes / (64 * (4096 + 256)) - 1;
    hipLaunchKernelGGL((dma64s<0, 4096 + 256>), dim3(2048), dim3(256), 0, 0, p, items_pad, sink);
    hipLaunchKernelGGL((dma128<0, 4096>), dim3(2048), dim3(256), 0, 0, p, items, sink);
    hipLaunchKernelGGL((dma128<37, 4096>), dim3(2048), dim3(256), 0, 0, p, items, sink);
    hipLaunchKernelGGL((dma128<37, 4096 + 256>), dim3(2048), dim3(256), 0, 0, p, items_pad, sink);
    // 1 KiB / 2 KiB task strides (one / two leaves per lane task): items scaled to the same 4 GiB
    hipLaunchKernelGGL((dma128<37, 1024>), dim3(2048), dim3(256), 0, 0, p, items * 4 - 1, sink);
    hipLaunchKernelGGL((dma128<37, 2048>), dim3(2048), dim3(256), 0, 0, p, items * 2 - 1, sink);
    hipLaunchKernelGGL((dma64s<37, 1024>), dim3(2048), dim3(256), 0, 0, p, items * 4 - 1, sink);
    printf("padded-stride kernels read %zu bytes (%.4f of 4 GiB)\n", items_pad * 64 * 4096, items_pad * 64 * 4096.0 / bytes);
    (void)hipDeviceSynchronize();
    printf("bytes per kernel: %zu (%.3f GiB)\n", bytes, bytes / 1073741824.0);
    (void)hipFree(p);
    (void)hipFree(sink);
    return 0;
}
