// Float-matmul probe (tools/, not part of the library): times launch_fmm_group (k_fmm, f32 MFMA) on
// the shapes it serves -- the batched F16 head, the v7 LoRA stages, an FP16 model's layer matmul --
// with random F16 weights and activations, and prints an output hash (for A/B of variants).
#include "mv_fmfma.hip"
#include "qgemm.hip"

#include <string.h>
#include <vector>

using namespace rwkvmi;

#define CK(x) do { hipError_t ck_ = (x); if (ck_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(ck_), __LINE__); exit(1); } } while (0)

static void * dhalf(size_t n, uint32_t seed) {
    std::vector<__half> h(n);
    uint32_t s = seed;
    for (size_t i = 0; i < n; i++) {
        s = s * 1664525u + 1013904223u;
        h[i] = __float2half(((float)(s >> 8) / 16777216.0f - 0.5f) * 0.25f);
    }
    void * p;
    CK(hipMalloc(&p, n * 2 + 64));
    CK(hipMemcpy(p, h.data(), n * 2, hipMemcpyHostToDevice));
    return p;
}

int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    struct Shape { const char * name; int M, K, T; };
    Shape shapes[] = {{"head B=128 (65536x2048)", 65536, 2048, 128}, {"head B=64", 65536, 2048, 64},
                      {"v7 LoRA-1 (576x2560) T=1024", 576, 2560, 1024}, {"v7 LoRA-2 (2560x96) T=1024", 2560, 96, 1024},
                      {"v7 g LoRA-2 (2560x320) T=1024", 2560, 320, 1024}, {"FP16 layer (2048x2048) T=1024", 2048, 2048, 1024},
                      {"K sweep 2560x32", 2560, 32, 1024}, {"K sweep 2560x128", 2560, 128, 1024},
                      {"K sweep 2560x512", 2560, 512, 1024}, {"K sweep 2560x1024", 2560, 1024, 1024},
                      {"T sweep 2560x96 T=256", 2560, 96, 256}, {"M sweep 640x96 T=1024", 640, 96, 1024}};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto & s : shapes) {
        MMGroup g;
        memset(&g, 0, sizeof g);
        g.n = 1;
        g.T = s.T;
        g.fmm = 1;
        MMEntry & e = g.e[0];
        e.W.type = W_F16;
        e.W.M = s.M;
        e.W.K = s.K;
        e.W.qs = (const uint8_t *)dhalf((size_t)s.M * s.K, 7u + s.M);
        e.in.fmt = A_F16;
        e.in.K = s.K;
        e.in.h = (__half *)dhalf((size_t)s.T * s.K, 11u + s.K);
        CK(hipMalloc(&e.y, (size_t)s.T * s.M * 4));
        e.ldy = s.M;
        e.epi = EPI_STORE;
        bool launched = false;
        if (!launch_fmm_group(st, g, W_F16, &launched) || !launched) { printf("%s: not launched\n", s.name); continue; }
        CK(hipStreamSynchronize(st));
        const int reps = 10;
        CK(hipEventRecord(a, st));
        for (int i = 0; i < reps; i++) launch_fmm_group(st, g, W_F16, &launched);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        std::vector<float> out((size_t)s.T * s.M);
        CK(hipMemcpy(out.data(), e.y, out.size() * 4, hipMemcpyDeviceToHost));
        unsigned long long h = 1469598103934665603ull;
        for (float f : out) h = (h ^ __builtin_bit_cast(uint32_t, f)) * 1099511628211ull;
        const double us = ms * 1e3 / reps, fl = 2.0 * s.M * s.K * s.T;
        printf("%-32s %9.1f us  %6.1f TFLOP/s  hash %016llx\n", s.name, us, fl / us * 1e-6, h);
        CK(hipFree((void *)e.W.qs));
        CK(hipFree(e.in.h));
        CK(hipFree(e.y));
    }
    return 0;
}
