// Global->LDS copy throughput probe (tools/, not part of the library).  512 workgroups of 4 waves
// each copy R rounds of N KiB per wave from a buffer of S bytes (wrapping) into LDS, waiting for
// every round (s_waitcnt vmcnt(0) + barrier) like qgemm's chunk pipeline.  Modes:
//   0: global_load_lds_dwordx4 (LDS DMA)      1: global_load_dwordx4 + ds_write_b128
// Prints GB/s into LDS for several footprints S (L2-resident .. HBM-sized).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(3))) void lds_void_t;

template <int MODE, int N>
__global__ __launch_bounds__(256) void k_copy(const uint8_t * src, size_t S, int R, int * sink) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[2][4 * N * 1024];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    size_t off = ((size_t)blockIdx.x * 4 * N * 1024 * 7) % S;
    int acc = 0;
    for (int r = 0; r < R; r++) {
        uint8_t * dst = buf[r & 1] + wave * N * 1024;
#pragma unroll
        for (int i = 0; i < N; i++) {
            const uint8_t * g = src + (off + (size_t)(wave * N + i) * 1024 + lane * 16) % S;
            if constexpr (MODE == 0) {
                const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long)(lds_void_t *)(dst + i * 1024));
                asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(g) : "m0");
            } else {
                const int4 v = *(const int4 *)g;
                *(int4 *)(dst + i * 1024 + lane * 16) = v;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        acc += buf[r & 1][threadIdx.x * 16];
        off = (off + (size_t)4 * N * 1024 * 512) % S;
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

template <int MODE, int N>
static void run(const uint8_t * src, size_t S, int * sink) {
    const int R = 64;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_copy<MODE, N>), dim3(512), dim3(256), 0, 0, src, S, R, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < 5; i++) hipLaunchKernelGGL((k_copy<MODE, N>), dim3(512), dim3(256), 0, 0, src, S, R, sink);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / 5, bytes = 512.0 * 4 * N * 1024 * R;
    printf("mode %d  N %2d KiB/wave/round  S %6.1f MB  %8.1f us  %7.1f GB/s  %6.2f us/round\n", MODE, N, S / 1e6, us,
           bytes / us * 1e-3, us / R);
}

int main() {
    const size_t SMAX = 512ull << 20;
    uint8_t * src;
    int * sink;
    CK(hipMalloc(&src, SMAX + 4096));
    CK(hipMemset(src, 1, SMAX + 4096));
    CK(hipMalloc(&sink, 4));
    for (size_t S : {(size_t)2 << 20, (size_t)32 << 20, SMAX}) {
        run<0, 2>(src, S, sink);
        run<0, 4>(src, S, sink);
        run<0, 8>(src, S, sink);
        run<1, 2>(src, S, sink);
        run<1, 4>(src, S, sink);
        run<1, 8>(src, S, sink);
    }
    return 0;
}
