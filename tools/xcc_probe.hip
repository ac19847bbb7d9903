// Which XCC runs each workgroup (tools/, not part of the library): HW_REG_XCC_ID via asm and via
// the builtin, for two back-to-back launches of 64 workgroups.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_xcc(unsigned * out) {
    if (threadIdx.x) return;
    unsigned a, b = __builtin_amdgcn_s_getreg((3 << 11) | 20);
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(a));
    out[blockIdx.x * 2] = a;
    out[blockIdx.x * 2 + 1] = b;
}

int main() {
    unsigned * d;
    unsigned h[2][128];
    hipMalloc(&d, 2 * 128 * 4);
    for (int l = 0; l < 2; l++) {
        hipLaunchKernelGGL(k_xcc, dim3(64 + 3 * l), dim3(64), 0, 0, d + 0);
        hipMemcpy(h[l], d, 128 * 4, hipMemcpyDeviceToHost);
        printf("launch %d asm:", l);
        for (int i = 0; i < 24; i++) printf(" %u", h[l][2 * i]);
        printf("\n         builtin:");
        for (int i = 0; i < 24; i++) printf(" %u", h[l][2 * i + 1]);
        printf("\n");
    }
    return 0;
}
