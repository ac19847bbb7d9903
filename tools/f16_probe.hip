// f16_probe.hip -- f32 -> f16 -> f32 round trip on the device (__float2half as the kernels use it)
// over values that land in the f16 subnormal and normal ranges; compared offline with numpy.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <vector>

__global__ void k_rt(int n, const float * x, float * y) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = __half2float(__float2half(x[i]));
}

int main(int argc, char ** argv) {
    const int n = 1 << 20;
    std::vector<float> x(n), y(n);
    uint64_t s = 12345;
    for (int i = 0; i < n; i++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t e = 95 + (uint32_t)((s >> 33) % 40);  // 2^-32 .. 2^7
        const uint32_t b = ((uint32_t)(s >> 20) & 1u) << 31 | e << 23 | ((uint32_t)(s >> 8) & 0x7fffff);
        memcpy(&x[i], &b, 4);
    }
    float *dx, *dy;
    if (hipMalloc(&dx, n * 4) != hipSuccess || hipMalloc(&dy, n * 4) != hipSuccess) return 1;
    if (hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_rt, dim3(n / 256), dim3(256), 0, 0, n, dx, dy);
    if (hipMemcpy(y.data(), dy, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    FILE * f = fopen(argc > 1 ? argv[1] : "f16_probe.bin", "wb");
    fwrite(x.data(), 4, n, f);
    fwrite(y.data(), 4, n, f);
    fclose(f);
    printf("f16_probe: %d values\n", n);
    return 0;
}
