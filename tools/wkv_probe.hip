// WKV6 sequence-kernel probe (tools/, not part of the library): times launch_wkv6 (head size 64,
// T = 1024, H = 32, per-token decay) for each workgroup width g_wkv6_nwv and checks that the
// variants agree bit for bit.
// Build: hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -DRWKV_BUILD
//        -Irwkv.cppy_amd/csrc -Iinclude -o tools/bin/wkv_probe tools/wkv_probe.hip
#include "kernels.hip"

#include <stdlib.h>
#include <string.h>
#include <vector>

namespace rwkvmi { extern int g_wkv6_nwv; }
using namespace rwkvmi;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main() {
    const int T = 1024, H = 32, S = 64, C = H * S;
    std::vector<float> hk((size_t)T * C), hv(hk.size()), hr(hk.size()), hw(hk.size()), hu(C), hs((size_t)H * S * S);
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX - 0.5f; };
    for (size_t i = 0; i < hk.size(); i++) {
        hk[i] = rnd(); hv[i] = rnd(); hr[i] = rnd(); hw[i] = 0.9f + 0.1f * rnd();
    }
    for (auto & x : hu) x = rnd();
    for (auto & x : hs) x = rnd();
    float *k, *v, *r, *w, *u, *s0, *s1, *y;
    const size_t tb = hk.size() * 4;
    CK(hipMalloc(&k, tb)); CK(hipMalloc(&v, tb)); CK(hipMalloc(&r, tb)); CK(hipMalloc(&w, tb)); CK(hipMalloc(&y, tb));
    CK(hipMalloc(&u, C * 4)); CK(hipMalloc(&s0, hs.size() * 4)); CK(hipMalloc(&s1, hs.size() * 4));
    CK(hipMemcpy(k, hk.data(), tb, hipMemcpyHostToDevice)); CK(hipMemcpy(v, hv.data(), tb, hipMemcpyHostToDevice));
    CK(hipMemcpy(r, hr.data(), tb, hipMemcpyHostToDevice)); CK(hipMemcpy(w, hw.data(), tb, hipMemcpyHostToDevice));
    CK(hipMemcpy(u, hu.data(), C * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(s0, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> ref, out((size_t)T * C), sref, sout(hs.size());
    for (int nwv : {4, 2, 1}) {
        g_wkv6_nwv = nwv;
        for (int i = 0; i < 2; i++) launch_wkv6(st, T, H, S, k, v, r, u, w, 1, s0, s1, y);
        CK(hipEventRecord(a, st));
        const int reps = 10;
        for (int i = 0; i < reps; i++) launch_wkv6(st, T, H, S, k, v, r, u, w, 1, s0, s1, y);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        CK(hipMemcpy(out.data(), y, tb, hipMemcpyDeviceToHost));
        CK(hipMemcpy(sout.data(), s1, hs.size() * 4, hipMemcpyDeviceToHost));
        bool same = true;
        if (ref.empty()) { ref = out; sref = sout; }
        else same = !memcmp(ref.data(), out.data(), tb) && !memcmp(sref.data(), sout.data(), hs.size() * 4);
        printf("wkv6 T=%d nwv=%d: %8.1f us  %s\n", T, nwv, ms * 1e3 / reps, same ? "bit-identical" : "DIFFERENT");
    }
    return 0;
}
