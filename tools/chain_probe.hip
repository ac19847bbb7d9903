// Decode-chain floor probe (tools/, not part of the library).  Times a hipGraph of N dependent
// synthetic Q4_0 x Q8 matvec launches (the shape of one decode step: each wave owns 2 rows of
// K = 2048, one 16-byte weight unit per lane per row, activation read from the buffer the previous
// launch wrote), with the weights rotated through R copies so that they come cold from HBM
// (R large), warm from the Infinity Cache (R*bytes < 256 MB) or warm from L2 (R = 1).
// Also: the same chain with trivial kernels (the launch floor).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/chain_probe tools/chain_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <string.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_flush(const int4 * p, size_t n, float * out) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i].x;
    if (acc == 0x12345678) out[0] = 1;
}
__global__ void k_triv(float * p) { if (threadIdx.x == 1000) p[0] = 1; }

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_add(float v) {
    const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, false);
    return v + __builtin_bit_cast(float, o);
}
__device__ __forceinline__ float wave_sum63(float v) {
    v = dpp_add<0xB1, 0xF>(v);
    v = dpp_add<0x4E, 0xF>(v);
    v = dpp_add<0x141, 0xF>(v);
    v = dpp_add<0x140, 0xF>(v);
    v = dpp_add<0x142, 0xA>(v);
    v = dpp_add<0x143, 0xC>(v);
    return v;
}

// W: [M][64] 16-byte units (K = 2048 Q4 nibbles), sc: [M][64] fp16 scales
// act: int8[2048] + float d[64]
template <int R>
__global__ __launch_bounds__(256) void k_syn(const int4 * __restrict__ W, const unsigned short * __restrict__ sc,
                                             const int8_t * __restrict__ act, const float * __restrict__ ad,
                                             float * __restrict__ y, int8_t * __restrict__ act_out, int M) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row0 = (blockIdx.x * 4 + wave) * R;
    int4 w[R];
    unsigned short s[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int row = min(row0 + r, M - 1);
        w[r] = W[(size_t)row * 64 + lane];
        s[r] = sc[(size_t)row * 64 + lane];
    }
    const int4 xl = *(const int4 *)(act + lane * 32);
    const int4 xh = *(const int4 *)(act + lane * 32 + 16);
    const float d = ad[lane];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int q[4] = {w[r].x, w[r].y, w[r].z, w[r].w};
        const int xs[8] = {xl.x, xl.y, xl.z, xl.w, xh.x, xh.y, xh.z, xh.w};
        int acc = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            acc = __builtin_amdgcn_sdot4((q[j] & 0x0f0f0f0f) - 0x08080808, xs[j], acc, false);
            acc = __builtin_amdgcn_sdot4(((q[j] >> 4) & 0x0f0f0f0f) - 0x08080808, xs[4 + j], acc, false);
        }
        const float f = wave_sum63(__half2float(__ushort_as_half(s[r])) * d * (float)acc);
        if (lane == 63 && row0 + r < M) {
            y[row0 + r] = f;
            if (row0 + r < 2048) act_out[row0 + r] = (int8_t)((int)f & 0x7f);
        }
    }
}

// The same body behind a k_mv-like group argument: 8 entries of 304 bytes by value, the entry
// found by a loop over block0 (dependent scalar loads), then its pointers loaded.
struct SynEnt {
    const int4 * W;
    const unsigned short * sc;
    const int8_t * act;
    const float * ad;
    float * y;
    int8_t * act_out;
    int M;
    int block0;
    char pad[304 - 56];
};
struct SynGrp {
    SynEnt e[8];
    int n;
};
template <int R>
__global__ __launch_bounds__(256) void k_syn_grp(SynGrp g) {
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const SynEnt & E = g.e[e];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int M = E.M;
    const int row0 = (((int)blockIdx.x - E.block0) * 4 + wave) * R;
    int4 w[R];
    unsigned short s[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int row = min(row0 + r, M - 1);
        w[r] = E.W[(size_t)row * 64 + lane];
        s[r] = E.sc[(size_t)row * 64 + lane];
    }
    const int4 xl = *(const int4 *)(E.act + lane * 32);
    const int4 xh = *(const int4 *)(E.act + lane * 32 + 16);
    const float d = E.ad[lane];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int q[4] = {w[r].x, w[r].y, w[r].z, w[r].w};
        const int xs[8] = {xl.x, xl.y, xl.z, xl.w, xh.x, xh.y, xh.z, xh.w};
        int acc = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            acc = __builtin_amdgcn_sdot4((q[j] & 0x0f0f0f0f) - 0x08080808, xs[j], acc, false);
            acc = __builtin_amdgcn_sdot4(((q[j] >> 4) & 0x0f0f0f0f) - 0x08080808, xs[4 + j], acc, false);
        }
        const float f = wave_sum63(__half2float(__ushort_as_half(s[r])) * d * (float)acc);
        if (lane == 63 && row0 + r < M) {
            E.y[row0 + r] = f;
            if (row0 + r < 2048) E.act_out[row0 + r] = (int8_t)((int)f & 0x7f);
        }
    }
}

int main(int argc, char ** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 168;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    float * y;
    int8_t * act[2];
    float * ad;
    CK(hipMalloc(&y, 1 << 20));
    for (int i = 0; i < 2; i++) {
        CK(hipMalloc(&act[i], 4096));
        CK(hipMemset(act[i], 1, 4096));
    }
    CK(hipMalloc(&ad, 4096));
    CK(hipMemset(ad, 0, 4096));
    int4 * flush;
    CK(hipMalloc(&flush, (size_t)512 << 20));
    CK(hipMemset(flush, 0, (size_t)512 << 20));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time_graph = [&](auto && body, const char * name, double bytes_per_kernel) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        body();
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 3; i++) CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        const int reps = 10;
        float ms = 0;
        for (int i = 0; i < reps; i++) {
            // evict the Infinity Cache between replays (untimed): read 512 MiB elsewhere
            hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, st, flush, (size_t)(512 << 20) / 16, y);
            CK(hipEventRecord(a, st));
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float t;
            CK(hipEventElapsedTime(&t, a, b));
            ms += t;
        }
        const double us = ms * 1e3 / reps / N;
        printf("%-44s %8.2f us/kernel  %8.1f GB/s\n", name, us, bytes_per_kernel / (us * 1e3));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    };
    time_graph([&] { for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_triv, dim3(256), dim3(256), 0, st, y); },
               "trivial 256x256", 0);
    time_graph([&] { for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_triv, dim3(1024), dim3(256), 0, st, y); },
               "trivial 1024x256", 0);
    const size_t total = (size_t)1 << 30;  // 1 GiB of weights + scales
    char * pool;
    CK(hipMalloc(&pool, total));
    CK(hipMemset(pool, 0x35, total));
    for (int M : {1024, 2048, 4096, 8192}) {
        const size_t wbytes = (size_t)M * 64 * 16, sbytes = (size_t)M * 64 * 2;
        const size_t per = wbytes + sbytes;
        const double algo = (double)M * 64 * 18;
        for (size_t rot_bytes : {total, (size_t)96 << 20, per}) {
            const int R = (int)(rot_bytes / per);
            char name[128];
            snprintf(name, sizeof name, "M=%d R2 copies=%d (%s)", M, R,
                     R == 1 ? "L2" : rot_bytes == total ? "HBM" : "MALL");
            time_graph([&] {
                for (int i = 0; i < N; i++) {
                    char * base = pool + (size_t)(i % R) * per;
                    hipLaunchKernelGGL(k_syn<2>, dim3((M + 7) / 8), dim3(256), 0, st, (const int4 *)base,
                                       (const unsigned short *)(base + wbytes), act[i & 1], ad, y, act[(i + 1) & 1], M);
                }
            }, name, algo);
        }
        for (int ne : {1, 4}) {
            const int R = (int)(total / per);
            char name[128];
            snprintf(name, sizeof name, "M=%d group of %d, copies=%d (HBM)", M, ne, R);
            time_graph([&] {
                for (int i = 0; i < N; i++) {
                    char * base = pool + (size_t)(i % R) * per;
                    SynGrp g;
                    memset(&g, 0, sizeof g);
                    g.n = ne;
                    const int Me = M / ne;
                    for (int j = 0; j < ne; j++) {
                        g.e[j].W = (const int4 *)(base + (size_t)j * Me * 64 * 16);
                        g.e[j].sc = (const unsigned short *)(base + wbytes + (size_t)j * Me * 64 * 2);
                        g.e[j].act = act[i & 1];
                        g.e[j].ad = ad;
                        g.e[j].y = y + j * Me;
                        g.e[j].act_out = act[(i + 1) & 1];
                        g.e[j].M = Me;
                        g.e[j].block0 = j * ((Me + 7) / 8);
                    }
                    hipLaunchKernelGGL(k_syn_grp<2>, dim3(ne * ((Me + 7) / 8)), dim3(256), 0, st, g);
                }
            }, name, algo);
        }
        {
            const int R = (int)(total / per);
            char name[128];
            snprintf(name, sizeof name, "M=%d R4 copies=%d (HBM)", M, R);
            time_graph([&] {
                for (int i = 0; i < N; i++) {
                    char * base = pool + (size_t)(i % R) * per;
                    hipLaunchKernelGGL(k_syn<4>, dim3((M + 15) / 16), dim3(256), 0, st, (const int4 *)base,
                                       (const unsigned short *)(base + wbytes), act[i & 1], ad, y, act[(i + 1) & 1], M);
                }
            }, name, algo);
        }
    }
    return 0;
}
