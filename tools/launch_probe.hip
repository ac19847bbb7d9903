// Launch-chain probe (tools/, not part of the library): what a short dependent matvec-like
// kernel costs inside a hipGraph chain on gfx950, split into inter-kernel gap, first-load
// latency and tail, for cold (HBM) weight slices.  Variants: empty kernel; weight pointer in
// preloaded kernarg SGPRs; weight pointer behind a dependent kernarg load (large by-value
// struct, like MVGroup); weight pointer behind a dependent load from a device table.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=16 tools/launch_probe.hip -o tools/bin/launch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Big {
    int pad[760];
    const int4 * w;
    float * out;
    int units;
};

__device__ __forceinline__ int4 ldnt(const int4 * p) {
    int4 v;
    v.x = __builtin_nontemporal_load(&p->x);
    v.y = __builtin_nontemporal_load(&p->y);
    v.z = __builtin_nontemporal_load(&p->z);
    v.w = __builtin_nontemporal_load(&p->w);
    return v;
}

template <int U>
__device__ __forceinline__ void body(const int4 * w, float * out, unsigned long long * st) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t row = (size_t)blockIdx.x * 4 + wave;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ldnt(w + (row * U + u) * 64 + lane);
    int s = 0;
#pragma unroll
    for (int u = 0; u < U; u++) s += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) out[row] = (float)s;
    if (st && threadIdx.x == 0) {
        st[blockIdx.x * 4 + 0] = t0;
        st[blockIdx.x * 4 + 1] = t1;
        st[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memrealtime();
    }
}

__global__ void k_empty(float * out) {
    if (threadIdx.x == 1000) out[0] = 1.0f;
}

template <int U>
__global__ __launch_bounds__(256) void k_pre(const int4 * w, float * out, unsigned long long * st) { body<U>(w, out, st); }

template <int U>
__global__ __launch_bounds__(256) void k_big(int e, Big g) { body<U>(g.w, g.out, nullptr); }

template <int U>
__global__ __launch_bounds__(256) void k_tab(const int4 * const * tab, int i, float * out) { body<U>(tab[i], out, nullptr); }

int main() {
    const size_t BUF = (size_t)1536 << 20;
    int4 * buf;
    CK(hipMalloc(&buf, BUF));
    CK(hipMemset(buf, 0x5a, BUF));
    float * out;
    CK(hipMalloc(&out, 1 << 24));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int N = 200;
    unsigned long long * stamps;
    CK(hipMalloc(&stamps, (size_t)N * 4096 * 4 * 8));
    const int4 ** dtab;
    CK(hipMalloc(&dtab, N * sizeof(void *)));

    auto run = [&](const char * name, int wgs, int U, int kind, bool cold, bool stamp) {
        const size_t per = (size_t)wgs * 4 * U * 1024;
        std::vector<const int4 *> ptrs(N);
        for (int i = 0; i < N; i++) ptrs[i] = cold ? buf + ((per * i) % (BUF - per)) / 16 : buf;
        CK(hipMemcpy(dtab, ptrs.data(), N * sizeof(void *), hipMemcpyHostToDevice));
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < N; i++) {
            unsigned long long * sp = stamp ? stamps + (size_t)i * wgs * 4 : nullptr;
            float * o = out + (size_t)(i % 4) * 65536;
            if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(wgs), dim3(256), 0, st, o);
#define DISPATCH(UU)                                                                                  \
    else if (U == UU) {                                                                               \
        if (kind == 1) hipLaunchKernelGGL(k_pre<UU>, dim3(wgs), dim3(256), 0, st, ptrs[i], o, sp);    \
        if (kind == 2) {                                                                              \
            Big bg;                                                                                   \
            bg.w = ptrs[i];                                                                           \
            bg.out = o;                                                                               \
            bg.units = UU;                                                                            \
            hipLaunchKernelGGL(k_big<UU>, dim3(wgs), dim3(256), 0, st, i & 1, bg);                   \
        }                                                                                             \
        if (kind == 3) hipLaunchKernelGGL(k_tab<UU>, dim3(wgs), dim3(256), 0, st, (const int4 * const *)dtab, i, o); \
    }
            DISPATCH(1) DISPATCH(2) DISPATCH(4) DISPATCH(8)
        }
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        float best = 1e30f;
        for (int r = 0; r < 3; r++) {
            CK(hipEventRecord(a, st));
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = std::min(best, ms);
        }
        const double us = best * 1000.0 / N;
        printf("%-34s WGs %5d U %d %6.2f MB/launch: %6.2f us/launch  %7.0f GB/s\n", name, wgs, U,
               kind ? per / 1e6 : 0.0, us, kind ? per / us / 1e3 : 0.0);
        if (stamp) {
            std::vector<unsigned long long> h((size_t)N * wgs * 4);
            CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> gap, lat50, lat90, spread, tail, dur;
            unsigned long long prev_end = 0;
            for (int i = 20; i < N - 20; i++) {
                const unsigned long long * p = &h[(size_t)i * wgs * 4];
                unsigned long long s0 = ~0ull, s1 = 0, e = 0;
                std::vector<double> l;
                for (int w = 0; w < wgs; w++) {
                    s0 = std::min(s0, p[w * 4]);
                    s1 = std::max(s1, p[w * 4]);
                    e = std::max(e, p[w * 4 + 2]);
                    l.push_back((p[w * 4 + 1] - p[w * 4]) * 0.01);
                }
                std::sort(l.begin(), l.end());
                if (prev_end) gap.push_back(((double)s0 - (double)prev_end) * 0.01);
                lat50.push_back(l[l.size() / 2]);
                lat90.push_back(l[l.size() * 9 / 10]);
                spread.push_back((s1 - s0) * 0.01);
                dur.push_back((e - s0) * 0.01);
                const unsigned long long * q = &h[(size_t)(i - 1) * wgs * 4];
                (void)q;
                prev_end = e;
            }
            auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
            printf("    stamps: gap(prev last end -> first start) %.2f us, start spread %.2f, load latency p50 %.2f p90 %.2f, "
                   "first start -> last end %.2f us\n", med(gap), med(spread), med(lat50), med(lat90), med(dur));
        }
    };
    run("empty", 256, 1, 0, true, false);
    run("empty", 1024, 1, 0, true, false);
    for (int U : {1, 2, 4, 8}) run("preloaded ptr, cold", 256, U, 1, true, true);
    for (int U : {1, 2}) run("preloaded ptr, warm (same slice)", 256, U, 1, false, true);
    run("preloaded ptr, cold", 1024, 2, 1, true, true);
    run("preloaded ptr, cold", 2048, 1, 1, true, true);
    for (int U : {1, 2, 8}) run("ptr behind kernarg load (3 KB arg)", 256, U, 2, true, false);
    for (int U : {1, 2, 8}) run("ptr behind device table load", 256, U, 3, true, false);
    return 0;
}
