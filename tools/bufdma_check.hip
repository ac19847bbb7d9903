// Checks the LDS placement rule of buffer_load_dwordx4 ... offen offset:N lds (tools/, not a test):
// expects LDS[M0 + N + 16*lane] <- mem[base + soffset + voffset + N].
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const unsigned * src, unsigned * out) {
    __shared__ __attribute__((aligned(16))) unsigned buf[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) buf[i] = 0xDEADBEEFu;
    __syncthreads();
    v4i r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned long)src);
    r.y = __builtin_amdgcn_readfirstlane((int)((unsigned long)src >> 32));
    r.z = -1;
    r.w = 0x00020000;
    const unsigned v = threadIdx.x * 16;
    const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long)(__attribute__((address_space(3))) void *)buf) + 512;
    const unsigned so = 4096;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen offset:1024 lds" ::"v"(v), "s"(m), "s"(r), "s"(so) : "memory", "m0");
    if (threadIdx.x < 8)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen offset:0 lds" ::"v"(v), "s"(m + 4096), "s"(r), "s"(so) : "memory", "m0");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += 64) out[i] = buf[i];
}
int main() {
    unsigned h[8192], *d, *o, res[2048];
    for (int i = 0; i < 8192; i++) h[i] = i;
    hipMalloc(&d, sizeof h); hipMalloc(&o, sizeof res);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
    hipMemcpy(res, o, sizeof res, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 2048; i++) {
        unsigned want = 0xDEADBEEFu;
        const int byte = i * 4;
        if (byte >= 512 + 1024 && byte < 512 + 1024 + 1024) want = (4096 + 1024 + (byte - 512 - 1024)) / 4;
        if (byte >= 512 + 4096 && byte < 512 + 4096 + 128) want = (4096 + (byte - 512 - 4096)) / 4;
        if (res[i] != want) { if (bad < 8) printf("dword %d: got %08x want %08x\n", i, res[i], want); bad++; }
    }
    printf("bufdma_check: %s (%d bad dwords)\n", bad ? "FAIL" : "ok", bad);
    return bad != 0;
}
