// Packed vs scalar f32 arithmetic on gfx950 (tools/, not part of the library): v_pk_{mul,add,fma}_f32
// against v_{mul,add,fma}_f32 on the same operands, counting bitwise mismatches, over random normal
// values and over the operand ranges of the sequence-GEMM epilogue.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void k_pk(const float * a, const float * b, const float * c, float * out, int n) {
    const int i = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
    if (i + 1 >= n) return;
    const f2 x = {a[i], a[i + 1]}, y = {b[i], b[i + 1]}, z = {c[i], c[i + 1]};
    const f2 m = x * y;
    const f2 s = x + z;
    const f2 f = __builtin_elementwise_fma(x, y, z);
    const f2 g = __builtin_elementwise_fma(x * y, z, s);  // the GEMM's fma(dw*dx, s, acc) shape
    out[6 * (size_t)i + 0] = m.x, out[6 * (size_t)i + 1] = m.y;
    out[6 * (size_t)i + 2] = s.x, out[6 * (size_t)i + 3] = s.y;
    out[6 * (size_t)i + 4] = f.x, out[6 * (size_t)i + 5] = f.y;
    out[6 * (size_t)n + 2 * (size_t)i] = g.x, out[6 * (size_t)n + 2 * (size_t)i + 1] = g.y;
}

__global__ void k_sc(const float * a, const float * b, const float * c, float * out, int n) {
    const int i = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
    if (i + 1 >= n) return;
    for (int e = 0; e < 2; e++) {
        const float x = a[i + e], y = b[i + e], z = c[i + e];
        const float m = x * y, s = x + z, f = fmaf(x, y, z), g = fmaf(x * y, z, s);
        out[6 * (size_t)i + 0 + e] = m;
        out[6 * (size_t)i + 2 + e] = s;
        out[6 * (size_t)i + 4 + e] = f;
        out[6 * (size_t)n + 2 * (size_t)i + e] = g;
    }
}

int main() {
    const int n = 1 << 22;
    std::vector<float> a(n), b(n), c(n);
    uint64_t s = 88172645463325252ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (int i = 0; i < n; i++) {
        const int mode = i % 4;
        if (mode == 0) {  // random bit patterns with moderate exponents
            uint32_t u = (uint32_t)rnd();
            u = (u & 0x807fffffu) | ((uint32_t)(100 + rnd() % 56) << 23);
            memcpy(&a[i], &u, 4);
            u = (uint32_t)rnd();
            u = (u & 0x807fffffu) | ((uint32_t)(100 + rnd() % 56) << 23);
            memcpy(&b[i], &u, 4);
            u = (uint32_t)rnd();
            u = (u & 0x807fffffu) | ((uint32_t)(100 + rnd() % 56) << 23);
            memcpy(&c[i], &u, 4);
        } else if (mode == 1) {  // GEMM epilogue: fp16 d, Q8 d, integer block sums
            a[i] = (float)((int)(rnd() % 2000) + 1) * 1e-5f;
            b[i] = (float)((int)(rnd() % 2000) + 1) * 3e-5f;
            c[i] = (float)((int)(rnd() % 8001) - 4000);
        } else if (mode == 2) {  // tiny values (denormal products / sums)
            a[i] = ldexpf((float)(rnd() % 1000 + 1), -80);
            b[i] = ldexpf((float)(rnd() % 1000 + 1), -60);
            c[i] = -ldexpf((float)(rnd() % 1000 + 1), -135);
        } else {  // cancellation
            a[i] = (float)(rnd() % 100000) * 1e-3f;
            b[i] = 1.0f + (float)(rnd() % 1000) * 1e-7f;
            c[i] = -a[i];
        }
    }
    float *da, *db, *dc, *o1, *o2;
    hipMalloc(&da, n * 4), hipMalloc(&db, n * 4), hipMalloc(&dc, n * 4);
    hipMalloc(&o1, (size_t)8 * n * 4), hipMalloc(&o2, (size_t)8 * n * 4);
    hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dc, c.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_pk, dim3(n / 512), dim3(256), 0, 0, da, db, dc, o1, n);
    hipLaunchKernelGGL(k_sc, dim3(n / 512), dim3(256), 0, 0, da, db, dc, o2, n);
    std::vector<uint32_t> h1((size_t)8 * n), h2((size_t)8 * n);
    hipMemcpy(h1.data(), o1, h1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(h2.data(), o2, h2.size() * 4, hipMemcpyDeviceToHost);
    const char * names[4] = {"mul", "add", "fma", "fma(mul)"};
    for (int op = 0; op < 4; op++)
        for (int mode = 0; mode < 4; mode++) {
            long bad = 0, tot = 0;
            long shown = 0;
            for (int i = 0; i < n; i++) {
                if (i % 4 != mode) continue;
                const size_t k = op < 3 ? 6 * (size_t)(i & ~1) + 2 * op + (i & 1) : 6 * (size_t)n + i;
                tot++;
                if (h1[k] != h2[k]) {
                    if (shown++ < 2) {
                        float f1, f2_;
                        memcpy(&f1, &h1[k], 4), memcpy(&f2_, &h2[k], 4);
                        printf("   %s mode %d: a=%a b=%a c=%a packed=%a scalar=%a\n", names[op], mode, a[i], b[i], c[i], f1, f2_);
                    }
                    bad++;
                }
            }
            printf("%-9s mode %d: %ld / %ld differ\n", names[op], mode, bad, tot);
        }
    return 0;
}
