// Sequence-GEMM probe (tools/, not part of the library): times launch_qgemm (int8 MFMA) and
// launch_mm_group (k_mm) on the v6-1B6 layer shapes at T = 1024 with random Q4_0 weights.
#include "kernels.hip"
#include "qgemm.hip"

#include <string.h>
#include <vector>

using namespace rwkvmi;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static void * dalloc(size_t n) {
    void * p;
    CK(hipMalloc(&p, n));
    std::vector<uint8_t> h(n);
    uint32_t s = 777u + (uint32_t)n;
    for (size_t i = 0; i < n; i++) {
        s = s * 1664525u + 1013904223u;
        h[i] = (uint8_t)(s >> 24);
    }
    CK(hipMemcpy(p, h.data(), n, hipMemcpyHostToDevice));
    return p;
}

static DMat qmat(int M, int K) {
    DMat m;
    memset(&m, 0, sizeof m);
    m.type = W_Q4_0;
    m.M = M;
    m.K = K;
    const size_t nb = (size_t)M * K / 32;
    m.qs = (const uint8_t *)dalloc(nb * 16);
    std::vector<__half> d(nb, __float2half(0.01f));
    void * p;
    CK(hipMalloc(&p, nb * 2));
    CK(hipMemcpy(p, d.data(), nb * 2, hipMemcpyHostToDevice));
    m.sc = p;
    m.gt = (const uint8_t *)dalloc((size_t)(M + 63) / 64 * (K / 32) * qg_w_bytes(W_Q4_0));
    return m;
}

static ActBuf act(int T, int K) {
    ActBuf a;
    memset(&a, 0, sizeof a);
    a.fmt = A_Q8_0;
    a.K = K;
    a.q = (int8_t *)dalloc((size_t)T * K);
    std::vector<float> d((size_t)T * K / 32, 0.02f);
    CK(hipMalloc(&a.d, d.size() * 4));
    CK(hipMemcpy(a.d, d.data(), d.size() * 4, hipMemcpyHostToDevice));
    a.qsum = (int *)dalloc((size_t)T * K / 32 * 4);
    a.tq = (uint8_t *)dalloc((size_t)(T + 63) / 64 * (K / 32) * qg_a_bytes(false));
    return a;
}

int main(int argc, char ** argv) {
    const int npath = argc > 1 ? atoi(argv[1]) : 3;
    const int T = 1024;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    struct Shape { const char * name; int M, K; };
    Shape shapes[] = {{"4x C x C (r,k,v,g)", 4 * 2048, 2048}, {"FFN k+r (9216 x 2048)", 9216, 2048},
                      {"FFN v (2048 x 7168)", 2048, 7168}, {"Wo (2048 x 2048)", 2048, 2048}};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto & s : shapes) {
        DMat W = qmat(s.M, s.K);
        ActBuf x = act(T, s.K);
        float * y;
        CK(hipMalloc(&y, (size_t)T * s.M * 4));
        std::vector<float> ref((size_t)T * s.M), out(ref.size());
        for (int path = 0; path < npath; path++) {
            MMGroup g;
            memset(&g, 0, sizeof g);
            g.n = 1;
            g.T = T;
            g.e[0].W = W;
            g.e[0].in = x;
            g.e[0].in.tiled = path < 2 ? 1 : 0;
            g.e[0].y = y;
            g.e[0].ldy = s.M;
            g.e[0].epi = EPI_STORE;
            g_qgemm_generic = path == 1;
            auto run = [&]() { return path == 2 ? launch_mm_group(st, g, W_Q4_0) : launch_qgemm(st, g, W_Q4_0); };
            if (!run()) return 1;
            CK(hipStreamSynchronize(st));
            const int reps = path == 2 ? 1 : 5;
            CK(hipEventRecord(a, st));
            for (int i = 0; i < reps; i++) run();
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            CK(hipMemcpy(out.data(), y, out.size() * 4, hipMemcpyDeviceToHost));
            if (path == 0) ref = out;
            const bool same = !memcmp(ref.data(), out.data(), out.size() * 4);
            const double us = ms * 1e3 / reps, ops = 2.0 * s.M * s.K * T;
            unsigned long long h = 1469598103934665603ull;
            for (float f : out) h = (h ^ __builtin_bit_cast(uint32_t, f)) * 1099511628211ull;
            printf("%-26s %-14s %9.1f us  %7.1f TOPS  %s  hash %016llx\n", s.name, path == 2 ? "k_mm" : path ? "qgemm-generic" : "qgemm",
                   us, ops / us * 1e-6, path && path < 2 ? (same ? "bit-identical" : "DIFFERENT") : "", h);
        }
    }
    return 0;
}
