// Decode-matvec probe (tools/, not part of the library): builds the v6-1B6 matvec shapes with
// random Q4_0 / F16 weights, times each launch shape inside a hipGraph and records per-
// workgroup phase timestamps (s_memrealtime, 100 MHz) of one launch: start, input ready,
// dots reduced, end.  Build: see tools/gpu_probe.sh.
#include "kernels_decode.hip"

namespace rwkvmi {
template bool launch_mv_shape<-1>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
template bool launch_mv_shape<W_F16>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
template bool launch_mv_shape<W_Q4_0>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
template bool launch_mv_shape<W_Q4_1>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
template bool launch_mv_shape<W_Q5_0>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
template bool launch_mv_shape<W_Q5_1>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
template bool launch_mv_shape<W_Q8_0>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
}  // namespace rwkvmi

#include <algorithm>
#include <string.h>
#include <stdlib.h>
#include <vector>

using namespace rwkvmi;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static void * dalloc(size_t n, int fill = -1) {
    void * p;
    CK(hipMalloc(&p, n));
    std::vector<uint8_t> h(n);
    uint32_t s = 12345u + (uint32_t)n;
    for (size_t i = 0; i < n; i++) {
        s = s * 1664525u + 1013904223u;
        h[i] = fill >= 0 ? (uint8_t)fill : (uint8_t)(s >> 24);
    }
    CK(hipMemcpy(p, h.data(), n, hipMemcpyHostToDevice));
    return p;
}

static DMat mat(int type, int M, int K) {
    DMat m;
    m.type = type;
    m.M = M;
    m.K = K;
    m.qh = nullptr;
    m.sc = nullptr;
    if (type == W_F16) {
        std::vector<__half> h((size_t)M * K);
        for (size_t i = 0; i < h.size(); i++) h[i] = __float2half(((int)(i * 2654435761u % 2001) - 1000) * 1e-4f);
        void * p;
        CK(hipMalloc(&p, h.size() * 2));
        CK(hipMemcpy(p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
        m.qs = (const uint8_t *)p;
    } else {
        const size_t nb = (size_t)M * K / 32;
        m.qs = (const uint8_t *)dalloc(nb * 16);
        std::vector<__half> d(nb);
        for (size_t i = 0; i < nb; i++) d[i] = __float2half(0.01f);
        void * p;
        CK(hipMalloc(&p, nb * 2));
        CK(hipMemcpy(p, d.data(), nb * 2, hipMemcpyHostToDevice));
        m.sc = p;
    }
    return m;
}

static ActBuf act(int fmt, int K) {
    ActBuf a;
    memset(&a, 0, sizeof a);
    a.fmt = fmt;
    a.K = K;
    if (fmt == A_Q8_0) {
        a.q = (int8_t *)dalloc(K);
        a.d = (float *)dalloc(K / 32 * 4, 0);
        a.qsum = (int *)dalloc(K / 32 * 4, 0);
    } else if (fmt == A_F16) {
        a.h = (__half *)dalloc(K * 2, 0);
    } else {
        a.f = (float *)dalloc(K * 4, 0);
    }
    return a;
}

static float * fvec(int n, float v) {
    std::vector<float> h(n, v);
    for (int i = 0; i < n; i++) h[i] = v + 0.001f * (i % 17);
    float * p;
    CK(hipMalloc(&p, n * 4));
    CK(hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice));
    return p;
}

int main() {
    const int C = 2048, F = 7168, V = 65536;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    unsigned long long * probe;
    const int maxwg = 1 << 16;
    CK(hipMalloc(&probe, (size_t)maxwg * 8 * 8));
    float * x = fvec(C, 0.5f), * carry = fvec(C, 0.25f), * lnw = fvec(C, 1.0f), * lnb = fvec(C, 0.0f), * mu = fvec(C, 0.3f);
    float * y = fvec(V, 0.0f), * y2 = fvec(C, 0.0f), * cout = fvec(C, 0.0f);
    auto lnmix = [&](MVEntry & e, int form) {
        e.src = SRC_LNMIX;
        e.x = x;
        e.carry = carry;
        e.lnw = lnw;
        e.lnb = lnb;
        e.mu = mu;
        e.form = form;
        e.carry_out = cout;
    };
    struct Case {
        const char * name;
        MVGroup g;
        double bytes;
    };
    std::vector<Case> cases;
    auto entry = [](const DMat & W, float * out, int epi) {
        MVEntry e;
        memset(&e, 0, sizeof e);
        e.W = W;
        e.y = out;
        e.epi = epi;
        e.act_out.fmt = -1;
        return e;
    };
    auto qbytes = [](int M, int K) { return (double)M * K / 32 * 18; };
    {
        Case c{"rkvg+dw1 SRC_ACT 4x2048x2048+64", {}, 0};
        ActBuf a = act(A_Q8_0, C);
        for (int i = 0; i < 4; i++) {
            c.g.e[i] = entry(mat(W_Q4_0, C, C), y + i * C, EPI_STORE);
            c.g.e[i].src = SRC_ACT;
            c.g.e[i].act = a;
            c.bytes += qbytes(C, C);
        }
        c.g.e[4] = entry(mat(W_Q4_0, 64, C), y + 4 * C, EPI_TANH);
        c.g.e[4].src = SRC_ACT;
        c.g.e[4].act = a;
        c.bytes += qbytes(64, C);
        c.g.n = 5;
        cases.push_back(c);
    }
    {
        Case c{"W1 LNMIX 160x2048", {}, qbytes(160, C)};
        c.g.e[0] = entry(mat(W_Q4_0, 160, C), y, EPI_TANH);
        lnmix(c.g.e[0], 1);
        c.g.n = 1;
        cases.push_back(c);
    }
    {
        Case c{"Wo SRC_F32 2048x2048", {}, qbytes(C, C)};
        c.g.e[0] = entry(mat(W_Q4_0, C, C), y2, EPI_ADD);
        c.g.e[0].src = SRC_F32;
        c.g.e[0].f = x;
        c.g.n = 1;
        cases.push_back(c);
    }
    {
        Case c{"FFN k(emit)+r LNMIX 7168+2048 x2048", {}, qbytes(F, C) + qbytes(C, C)};
        c.g.e[0] = entry(mat(W_Q4_0, F, C), nullptr, EPI_RELU_SQ);
        lnmix(c.g.e[0], 1);
        c.g.e[0].emit = 1;
        c.g.e[0].act_out = act(A_Q8_0, F);
        c.g.e[1] = entry(mat(W_Q4_0, C, C), y, EPI_STORE);
        lnmix(c.g.e[1], 1);
        c.g.n = 2;
        cases.push_back(c);
    }
    {
        Case c{"FFN v SRC_ACT 2048x7168", {}, qbytes(C, F)};
        c.g.e[0] = entry(mat(W_Q4_0, C, F), y2, EPI_ADD);
        c.g.e[0].src = SRC_ACT;
        c.g.e[0].act = act(A_Q8_0, F);
        c.g.n = 1;
        cases.push_back(c);
    }
    {
        Case c{"head F16 LN 65536x2048", {}, (double)V * C * 2};
        c.g.e[0] = entry(mat(W_F16, V, C), y, EPI_STORE);
        lnmix(c.g.e[0], 2);
        c.g.e[0].carry_out = nullptr;
        c.g.n = 1;
        cases.push_back(c);
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto & c : cases) {
        unsigned long long * none = nullptr;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_probe), &none, sizeof none));
        for (int i = 0; i < 5; i++)
            if (!launch_mv_group(st, c.g)) return 1;
        CK(hipStreamSynchronize(st));
        const int reps = 50;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < reps; i++) launch_mv_group(st, c.g);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(a, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1000 / reps;
        // probe one launch (after a warm one)
        int nwg = 0;
        {
            MVGroup gg = c.g;
            launch_mv_group(st, gg);
            for (int i = 0; i < gg.n; i++) {
                const int RW = gg.e[i].emit ? 32 : 8;
                nwg = gg.e[i].block0 + (gg.e[i].W.M + RW - 1) / RW;
            }
            if (gg.stride > 0) nwg = gg.stride;
        }
        CK(hipMemset(probe, 0, (size_t)nwg * 64));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_probe), &probe, sizeof probe));
        launch_mv_group(st, c.g);
        CK(hipStreamSynchronize(st));
        std::vector<unsigned long long> h((size_t)nwg * 8);
        CK(hipMemcpy(h.data(), probe, h.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, tend = 0;
        std::vector<double> st0, d01, d12, d23, d04, d45, d56, d61;
        for (int w = 0; w < nwg; w++) {
            const unsigned long long * p = &h[(size_t)w * 8];
            t0 = std::min(t0, p[0]);
            tend = std::max(tend, p[3]);
        }
        for (int w = 0; w < nwg; w++) {
            const unsigned long long * p = &h[(size_t)w * 8];
            st0.push_back((p[0] - t0) * 0.01);
            d01.push_back((double)(p[1] - p[0]) * 0.01);
            d12.push_back((double)(p[2] - p[1]) * 0.01);
            d23.push_back((double)(p[3] - p[2]) * 0.01);
            if (p[4]) {
                d04.push_back((double)(p[4] - p[0]) * 0.01);
                if (p[5]) d45.push_back((double)(p[5] - p[4]) * 0.01);
                d56.push_back((double)(p[6] - (p[5] ? p[5] : p[4])) * 0.01);
                d61.push_back((double)(p[1] - p[6]) * 0.01);
            }
        }
        auto pct = [](std::vector<double> v, double q) {
            std::sort(v.begin(), v.end());
            return v[(size_t)(q * (v.size() - 1))];
        };
        printf("%-40s %7.2f us/launch (graph) %7.0f GB/s | WGs %d span %.2f us\n", c.name, us, c.bytes / us * 1e-3, nwg,
               (tend - t0) * 0.01);
        printf("    start offset  p50 %.2f p90 %.2f max %.2f\n", pct(st0, 0.5), pct(st0, 0.9), pct(st0, 1.0));
        printf("    input ready   p50 %.2f p90 %.2f max %.2f\n", pct(d01, 0.5), pct(d01, 0.9), pct(d01, 1.0));
        if (!d04.empty()) {
            printf("      LN stats(+loads) p50 %.2f p90 %.2f max %.2f\n", pct(d04, 0.5), pct(d04, 0.9), pct(d04, 1.0));
            if (!d45.empty()) printf("      LN stats    p50 %.2f p90 %.2f max %.2f\n", pct(d45, 0.5), pct(d45, 0.9), pct(d45, 1.0));
            printf("      mix+quant   p50 %.2f p90 %.2f max %.2f\n", pct(d56, 0.5), pct(d56, 0.9), pct(d56, 1.0));
            printf("      barrier     p50 %.2f p90 %.2f max %.2f\n", pct(d61, 0.5), pct(d61, 0.9), pct(d61, 1.0));
        }
        printf("    dots+reduce   p50 %.2f p90 %.2f max %.2f\n", pct(d12, 0.5), pct(d12, 0.9), pct(d12, 1.0));
        printf("    epilogue      p50 %.2f p90 %.2f max %.2f\n", pct(d23, 0.5), pct(d23, 0.9), pct(d23, 1.0));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
