// arith_probe.hip -- pins the gfx950 arithmetic the bit-exact oracle variant must reproduce:
// v_dot2_f32_f16 rounding (one rounding of the exact sum, or two), f32 sqrt / division
// rounding under hipcc's default float mode.  Inputs are generated on the host, results are
// written raw to the output file and compared offline (tools/arith_check.py).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/arith_probe.hip -o tools/bin/arith_probe
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

__global__ void k_probe(int n, const uint32_t * a, const uint32_t * b, const float * c, const float * x,
                        const float * y, float * o_dot, float * o_sqrt, float * o_div, float * o_rcp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    o_dot[i] = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, a[i]), __builtin_bit_cast(half2_t, b[i]), c[i], false);
    o_sqrt[i] = sqrtf(fabsf(x[i]));
    o_div[i] = x[i] / y[i];
    o_rcp[i] = 1.0f / y[i];
}

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return (uint32_t)(s >> 11);
}

int main(int argc, char ** argv) {
    const int n = 1 << 20;
    std::vector<uint32_t> a(n), b(n);
    std::vector<float> c(n), x(n), y(n);
    for (int i = 0; i < n; i++) {
        // halves with a narrow exponent band so products and c overlap and cancel often
        auto h = [](int emin, int ebits) {
            const uint32_t e = (uint32_t)(emin + (int)(rnd() % ebits));
            return (uint16_t)(((rnd() & 1) << 15) | (e << 10) | (rnd() & 0x3ff));
        };
        const int mode = i & 3;
        a[i] = (uint32_t)h(10, 10) | ((uint32_t)h(10, 10) << 16);
        b[i] = (uint32_t)h(10, 10) | ((uint32_t)h(10, 10) << 16);
        uint32_t cb = ((rnd() & 1) << 31) | ((uint32_t)(110 + rnd() % 30) << 23) | (rnd() & 0x7fffff);
        if (mode == 1) cb = 0;
        memcpy(&c[i], &cb, 4);
        uint32_t xb = (rnd() & 0x807fffff) | ((uint32_t)(60 + rnd() % 130) << 23);
        uint32_t yb = (rnd() & 0x807fffff) | ((uint32_t)(60 + rnd() % 130) << 23);
        memcpy(&x[i], &xb, 4);
        memcpy(&y[i], &yb, 4);
    }
    uint32_t *da, *db;
    float *dc, *dx, *dy, *o[4];
    hipMalloc(&da, n * 4);
    hipMalloc(&db, n * 4);
    hipMalloc(&dc, n * 4);
    hipMalloc(&dx, n * 4);
    hipMalloc(&dy, n * 4);
    for (auto & p : o) hipMalloc(&p, n * 4);
    hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dc, c.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dy, y.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(n / 256), dim3(256), 0, 0, n, da, db, dc, dx, dy, o[0], o[1], o[2], o[3]);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    FILE * f = fopen(argc > 1 ? argv[1] : "arith_probe.bin", "wb");
    fwrite(a.data(), 4, n, f);
    fwrite(b.data(), 4, n, f);
    fwrite(c.data(), 4, n, f);
    fwrite(x.data(), 4, n, f);
    fwrite(y.data(), 4, n, f);
    std::vector<float> h(n);
    for (auto & p : o) {
        hipMemcpy(h.data(), p, n * 4, hipMemcpyDeviceToHost);
        fwrite(h.data(), 4, n, f);
    }
    fclose(f);
    printf("arith_probe: %d cases written\n", n);
    return 0;
}
