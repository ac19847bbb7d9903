// MFMA issue-rate probe: int8 16x16x32 (CDNA3 form) vs 16x16x64 / 32x32x32 (gfx950 forms), wall
// clock over a full-chip grid, 4 independent accumulators per wave.  Prints TOPS per form.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v16i __attribute__((ext_vector_type(16)));
constexpr int IT = 2048;
__global__ __launch_bounds__(256) void k16x32(const v2i* a, v4i* o) {
    v2i x = a[threadIdx.x], y = a[threadIdx.x + 256];
    v4i c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < IT; i++) {
        long xx = __builtin_bit_cast(long, x), yy = __builtin_bit_cast(long, y);
        c0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(xx, yy, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(xx, yy, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x32_i8(xx, yy, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x32_i8(xx, yy, c3, 0, 0, 0);
    }
    o[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3;
}
__global__ __launch_bounds__(256) void k16x64(const v4i* a, v4i* o) {
    v4i x = a[threadIdx.x], y = a[threadIdx.x + 256];
    v4i c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < IT; i++) {
        c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, c3, 0, 0, 0);
    }
    o[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3;
}
__global__ __launch_bounds__(256) void k32x32(const v4i* a, v16i* o) {
    v4i x = a[threadIdx.x], y = a[threadIdx.x + 256];
    v16i c0 = {}, c1 = {};
    for (int i = 0; i < IT; i++) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(x, y, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(x, y, c1, 0, 0, 0);
    }
    o[blockIdx.x * 256 + threadIdx.x] = c0 + c1;
}
int main() {
    const int G = 256 * 8;
    void *a, *o;
    hipMalloc(&a, 1 << 16);
    hipMemset(a, 0x35, 1 << 16);
    hipMalloc(&o, (size_t)G * 256 * 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int f = 0; f < 3; f++) {
        double ops = 0;
        float best = 1e30f;
        for (int r = 0; r < 4; r++) {
            hipEventRecord(e0);
            if (f == 0) { k16x32<<<G, 256>>>((const v2i*)a, (v4i*)o); ops = 4.0 * IT * 16 * 16 * 32 * 2; }
            if (f == 1) { k16x64<<<G, 256>>>((const v4i*)a, (v4i*)o); ops = 4.0 * IT * 16 * 16 * 64 * 2; }
            if (f == 2) { k32x32<<<G, 256>>>((const v4i*)a, (v16i*)o); ops = 2.0 * IT * 32 * 32 * 32 * 2; }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r && ms < best) best = ms;
        }
        const double tot = ops * G * 4;  // 4 waves per workgroup
        printf("%s: %.3f ms  %.1f TOPS\n", f == 0 ? "i32_16x16x32_i8" : f == 1 ? "i32_16x16x64_i8" : "i32_32x32x32_i8", best,
               tot / best / 1e9);
    }
    return 0;
}
