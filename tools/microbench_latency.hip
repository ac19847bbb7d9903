// Latency microbenchmark for the decode building blocks (tools/, not part of the library):
// empty kernel, single-workgroup LayerNorm (fp64 vs fp32 reductions), shuffle reductions.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_empty(float * p) { if (threadIdx.x == 1000) p[0] = 1; }

template <typename T>
__device__ T wsum(T v) { for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o); return v; }

template <typename T>
__device__ T bsum(T v, T * sh) {
    v = wsum(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    T r = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) r += sh[w];
    __syncthreads();
    return r;
}

template <typename T>
__global__ void k_ln(const float * x, float * y, int C) {
    __shared__ T sh[8];
    T s = 0;
    for (int c = threadIdx.x; c < C; c += blockDim.x) s += (T)x[c];
    s = bsum(s, sh);
    float mean = (float)(s / (T)C);
    T s2 = 0;
    for (int c = threadIdx.x; c < C; c += blockDim.x) { float v = x[c] - mean; s2 += (T)(v * v); }
    s2 = bsum(s2, sh);
    float sc = 1.0f / sqrtf((float)(s2 / (T)C) + 1e-5f);
    for (int c = threadIdx.x; c < C; c += blockDim.x) y[c] = (x[c] - mean) * sc;
}

__global__ void k_stream(const int4 * w, int4 * out, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    int4 acc = make_int4(0, 0, 0, 0);
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) { int4 v = w[i]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
    if (acc.x == 0x12345678) out[0] = acc;
}

struct BigArg {
    int v[512];
};

// N dependent scalar loads from the kernel-argument segment
template <int N>
__global__ void k_karg_chain(BigArg a, int * out) {
    int i = a.v[0];
#pragma unroll
    for (int k = 1; k < N; k++) i = a.v[i & 511];
    if (threadIdx.x == 0 && i == -7) out[0] = i;
}

// N dependent scalar loads from a device buffer
template <int N>
__global__ void k_dev_chain(const int * __restrict__ p, int * out) {
    int i = p[0];
#pragma unroll
    for (int k = 1; k < N; k++) i = p[i & 511];
    if (threadIdx.x == 0 && i == -7) out[0] = i;
}

// N dependent per-lane vector loads from a buffer the previous kernel wrote
template <int N>
__global__ void k_vec_chain(int * p, int * out) {
    int i = p[threadIdx.x & 63];
#pragma unroll
    for (int k = 1; k < N; k++) i = p[(i + threadIdx.x) & 511];
    if (blockIdx.x == 0 && threadIdx.x < 64) p[threadIdx.x] = i & 7;  // write for the next launch
    if (i == -7) out[0] = i;
}

int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    float *x, *y;
    CK(hipMalloc(&x, 1 << 20));
    CK(hipMalloc(&y, 1 << 20));
    CK(hipMemset(x, 0, 1 << 20));
    int4 * big;
    size_t nbig = (size_t)64 << 20;  // 1 GiB of int4
    CK(hipMalloc(&big, nbig * 16));
    CK(hipMemset(big, 1, nbig * 16));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char * name, auto launch, int reps) {
        for (int i = 0; i < 10; i++) launch();
        hipStreamSynchronize(st);
        // graph of `reps` launches
        hipGraph_t g; hipGraphExec_t ge;
        hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
        for (int i = 0; i < reps; i++) launch();
        hipStreamEndCapture(st, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        hipGraphLaunch(ge, st);
        hipStreamSynchronize(st);
        hipEventRecord(a, st);
        hipGraphLaunch(ge, st);
        hipEventRecord(b, st);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("%-40s %8.2f us/launch (graph of %d)\n", name, ms * 1000 / reps, reps);
        hipGraphExecDestroy(ge); hipGraphDestroy(g);
    };
    {
        BigArg ba;
        for (int i = 0; i < 512; i++) ba.v[i] = (i * 7 + 3) & 511;
        int * dv;
        CK(hipMalloc(&dv, 4096));
        CK(hipMemcpy(dv, ba.v, 2048, hipMemcpyHostToDevice));
        int * ob;
        CK(hipMalloc(&ob, 4096));
        for (int grid : {1, 256, 1024}) {
            char nm[64];
            snprintf(nm, sizeof nm, "kernarg chain 1 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_karg_chain<1>, dim3(grid), dim3(256), 0, st, ba, ob); }, 500);
            snprintf(nm, sizeof nm, "kernarg chain 4 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_karg_chain<4>, dim3(grid), dim3(256), 0, st, ba, ob); }, 500);
            snprintf(nm, sizeof nm, "kernarg chain 8 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_karg_chain<8>, dim3(grid), dim3(256), 0, st, ba, ob); }, 500);
            snprintf(nm, sizeof nm, "devbuf chain 1 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_dev_chain<1>, dim3(grid), dim3(256), 0, st, dv, ob); }, 500);
            snprintf(nm, sizeof nm, "devbuf chain 4 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_dev_chain<4>, dim3(grid), dim3(256), 0, st, dv, ob); }, 500);
            snprintf(nm, sizeof nm, "devbuf chain 8 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_dev_chain<8>, dim3(grid), dim3(256), 0, st, dv, ob); }, 500);
            snprintf(nm, sizeof nm, "vector chain 1 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_vec_chain<1>, dim3(grid), dim3(256), 0, st, dv, ob); }, 500);
            snprintf(nm, sizeof nm, "vector chain 4 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_vec_chain<4>, dim3(grid), dim3(256), 0, st, dv, ob); }, 500);
            snprintf(nm, sizeof nm, "vector chain 8 grid %d", grid);
            timeit(nm, [&]() { hipLaunchKernelGGL(k_vec_chain<8>, dim3(grid), dim3(256), 0, st, dv, ob); }, 500);
        }
    }
    timeit("empty 1 WG", [&]() { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, y); }, 1000);
    timeit("empty 256 WG", [&]() { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, st, y); }, 1000);
    timeit("empty 2048 WG", [&]() { hipLaunchKernelGGL(k_empty, dim3(2048), dim3(256), 0, st, y); }, 1000);
    timeit("LN fp64 C=2048 1 WG", [&]() { hipLaunchKernelGGL(k_ln<double>, dim3(1), dim3(256), 0, st, x, y, 2048); }, 1000);
    timeit("LN fp32 C=2048 1 WG", [&]() { hipLaunchKernelGGL(k_ln<float>, dim3(1), dim3(256), 0, st, x, y, 2048); }, 1000);
    timeit("LN fp64 C=2048 256 WG", [&]() { hipLaunchKernelGGL(k_ln<double>, dim3(256), dim3(256), 0, st, x, y, 2048); }, 1000);
    for (size_t mb : {1, 2, 4, 8, 16, 64, 256}) {
        size_t n = mb * 65536;  // int4 count for mb MiB
        char nm[64];
        for (int grid : {256, 1024, 4096}) {
            snprintf(nm, sizeof nm, "stream %zu MiB grid %d", mb, grid);
            // distinct windows per launch so L2/MALL reuse does not help
            size_t off = 0;
            timeit(nm, [&]() { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, st, big + off, (int4 *)y, n); off = (off + n) % (nbig - n); }, 100);
        }
    }
    return 0;
}
