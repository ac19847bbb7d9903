// Real-k_mv chain probe (tools/, not part of the library): a hipGraph of N dependent launches of
// the library's decode matvec (launch_mv_group) on a Wo-like / FFN-v-like / rkvg-like group,
// weights rotated through copies so they come cold from HBM (Infinity Cache flushed between
// replays), beside the same chain of the minimal synthetic kernel (tools/chain_probe.hip).
// Build: hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -DRWKV_BUILD
//        -mllvm -amdgpu-kernarg-preload-count=16 -Irwkv.cppy_amd/csrc -Iinclude -o tools/mv_chain
//        tools/mv_chain.hip rwkv.cppy_amd/build/mv_*.hip.o
#include "kernels_decode.hip"


#include <string.h>
#include <stdlib.h>
#include <vector>

using namespace rwkvmi;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_flush(const int4 * p, size_t n, float * out) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i].x;
    if (acc == 0x12345678) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_syn(const int4 * __restrict__ W, const unsigned short * __restrict__ sc,
                                             const int8_t * __restrict__ act, const float * __restrict__ ad,
                                             float * __restrict__ y, int M) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row0 = (blockIdx.x * 4 + wave) * 2;
    int4 w[2];
    unsigned short s[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int row = min(row0 + r, M - 1);
        w[r] = W[(size_t)row * 64 + lane];
        s[r] = sc[(size_t)row * 64 + lane];
    }
    const int4 xl = *(const int4 *)(act + lane * 32);
    const int4 xh = *(const int4 *)(act + lane * 32 + 16);
    const float d = ad[lane];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int q[4] = {w[r].x, w[r].y, w[r].z, w[r].w};
        const int xs[8] = {xl.x, xl.y, xl.z, xl.w, xh.x, xh.y, xh.z, xh.w};
        int acc = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            acc = __builtin_amdgcn_sdot4((q[j] & 0x0f0f0f0f) - 0x08080808, xs[j], acc, false);
            acc = __builtin_amdgcn_sdot4(((q[j] >> 4) & 0x0f0f0f0f) - 0x08080808, xs[4 + j], acc, false);
        }
        const float f = wave_sum63(__half2float(__ushort_as_half(s[r])) * d * (float)acc);
        if (lane == 63 && row0 + r < M) y[row0 + r] = y[row0 + r] + f;
    }
}

int main(int argc, char ** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 168;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    float * y;
    CK(hipMalloc(&y, 1 << 22));
    CK(hipMemset(y, 0, 1 << 22));
    int4 * flush;
    CK(hipMalloc(&flush, (size_t)512 << 20));
    CK(hipMemset(flush, 0, (size_t)512 << 20));
    const size_t total = (size_t)1 << 30;
    char * pool;
    CK(hipMalloc(&pool, total));
    CK(hipMemset(pool, 0x35, total));
    // activation buffers (Q8_0, K up to 8192), two, ping-pong
    ActBuf act[2];
    for (int i = 0; i < 2; i++) {
        memset(&act[i], 0, sizeof(ActBuf));
        act[i].fmt = A_Q8_0;
        char * p;
        CK(hipMalloc(&p, 1 << 20));
        CK(hipMemset(p, 0, 1 << 20));
        act[i].q = (int8_t *)p;
        act[i].d = (float *)(p + 65536);
        act[i].qsum = (int *)(p + 65536 * 2);
        act[i].s = (float *)(p + 65536 * 3);
    }
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
        for (int i = 0; i < 2; i++) CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        const int reps = 8;
        float ms = 0;
        for (int i = 0; i < reps; i++) {
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
        printf("%-52s %8.2f us/kernel  %8.1f GB/s\n", name, us, bytes_per_kernel / (us * 1e3));
        fflush(stdout);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    };
    struct Shape {
        const char * name;
        int n;         // entries
        int M[5], K;
        int epi;
    };
    const Shape shapes[] = {
        {"Wo   2048x2048 EPI_ADD", 1, {2048}, 2048, EPI_ADD},
        {"Wo   2048x2048 EPI_STORE", 1, {2048}, 2048, EPI_STORE},
        {"FFNv 2048x7168 EPI_ADD", 1, {2048}, 7168, EPI_ADD},
        {"rkvg 4x2048+64 x2048", 5, {2048, 2048, 2048, 2048, 64}, 2048, EPI_STORE},
        {"one  8256x2048", 1, {8256}, 2048, EPI_STORE},
    };
    for (const Shape & sh : shapes) {
        const int K = sh.K, nb = K / 32;
        int Mt = 0;
        for (int i = 0; i < sh.n; i++) Mt += sh.M[i];
        const size_t per = (size_t)Mt * nb * 18;
        const int R = (int)(total / per);
        std::vector<MVGroup> groups(N);
        for (int i = 0; i < N; i++) {
            char * base = pool + (size_t)(i % R) * per;
            MVGroup & g = groups[i];
            memset(&g, 0, sizeof g);
            g.n = sh.n;
            size_t off = 0;
            for (int j = 0; j < sh.n; j++) {
                MVEntry & e = g.e[j];
                e.W.type = W_Q4_0;
                e.W.M = sh.M[j];
                e.W.K = K;
                e.W.qs = (const uint8_t *)(base + off);
                e.W.sc = base + off + (size_t)sh.M[j] * nb * 16;
                off += (size_t)sh.M[j] * nb * 18;
                e.src = SRC_ACT;
                e.act = act[i & 1];
                e.act.K = K;
                e.y = y + j * 8192;
                e.epi = sh.epi;
                e.act_out.fmt = -1;
            }
        }
        char name[128];
        snprintf(name, sizeof name, "k_mv %s (HBM)", sh.name);
        time_graph([&] {
            for (int i = 0; i < N; i++) launch_mv_group(st, groups[i]);
        }, name, (double)per);
        if (K == 2048) {
            snprintf(name, sizeof name, "k_syn M=%d K=2048 (HBM)", Mt);
            time_graph([&] {
                for (int i = 0; i < N; i++) {
                    char * base = pool + (size_t)(i % R) * per;
                    hipLaunchKernelGGL(k_syn, dim3((Mt + 7) / 8), dim3(256), 0, st, (const int4 *)base,
                                       (const unsigned short *)(base + (size_t)Mt * nb * 16), act[i & 1].q, act[i & 1].d, y, Mt);
                }
            }, name, (double)per);
        }
    }
    return 0;
}
