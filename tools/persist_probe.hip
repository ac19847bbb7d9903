// Persistent-decode probe (tools/, not part of the library).  One launch of G workgroups (one per
// CU) runs N dependent synthetic Q4_0 x Q8 matvec phases (K = 2048, M rows each, weights rotated
// through copies so they come cold from HBM).  Each workgroup owns M/G rows, issues the loads of
// its next phase's weights BEFORE waiting for the previous phase, then reads the activation the
// previous phase published.  Two hand-off forms:
//   ctr : sc1 payload stores + vmcnt(0) + workgroup barrier + one agent atomic add per workgroup
//         onto a per-XCD-class shard; consumers poll all 8 shards with sc1 loads (one wave),
//   gran: 8-byte {epoch, value} granules (one per output row), consumers sweep all of them.
// Every spin is bounded by s_memrealtime (give-up after ~50 ms sets a failure word).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/persist_probe tools/persist_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__global__ void k_flush(const int4 * p, size_t n, float * out) {
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i].x;
    if (acc == 0x12345678) out[0] = 1;
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_add(float v) {
    const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, false);
    return v + __builtin_bit_cast(float, o);
}
__device__ __forceinline__ float wave_sum63(float v) {
    v = dpp_add<0xB1, 0xF>(v);
    v = dpp_add<0x4E, 0xF>(v);
    v = dpp_add<0x141, 0xF>(v);
    v = dpp_add<0x140, 0xF>(v);
    v = dpp_add<0x142, 0xA>(v);
    v = dpp_add<0x143, 0xC>(v);
    return v;
}

__device__ __forceinline__ bool timed_out(unsigned long long t0) {
    return __builtin_amdgcn_s_memrealtime() - t0 > 5000000ull;  // 100 MHz -> 50 ms
}

// acts: [2][2048] int8 (+ d [2][64] f32) for ctr; granules [2][M] u64 for gran
struct Args {
    const char * pool;       // weight copies
    size_t per;              // bytes per copy (W then sc)
    int copies, M, N;
    int8_t * act;            // ctr: [2][2048]
    float * ad;              // ctr: [2][64]
    unsigned * ctr;          // ctr: [N][8] shards (zeroed per call)
    unsigned long long * gran;  // gran: [2][M] (zeroed per call)
    unsigned * fail;
    float * y;
};

template <int R, bool GRAN>
__global__ __launch_bounds__(256) void k_persist(Args a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int G = gridDim.x;
    const int rows_per_wg = a.M / G;           // host checks divisibility
    const int row0 = blockIdx.x * rows_per_wg + wave * R;
    const size_t wbytes = (size_t)a.M * 64 * 16;
    __shared__ int8_t s_act[2048];
    __shared__ float s_d[64];
    __shared__ int s_ok;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < a.N; p++) {
        const char * base = a.pool + (size_t)(p % a.copies) * a.per;
        const int4 * W = (const int4 *)base;
        const unsigned short * sc = (const unsigned short *)(base + wbytes);
        int4 w[R];
        unsigned short s[R];
        const bool active = wave * R < rows_per_wg;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int row = min(row0 + r, a.M - 1);
            { typedef int v4i __attribute__((ext_vector_type(4))); const v4i t = __builtin_nontemporal_load((const v4i *)&W[(size_t)row * 64 + lane]); w[r] = make_int4(t.x, t.y, t.z, t.w); }
            s[r] = sc[(size_t)row * 64 + lane];
        }
        if (p > 0) {
            if (!GRAN) {
                // wait for all G producers of phase p-1
                if (wave == 0) {
                    const unsigned need = G / 8;
                    for (;;) {
                        unsigned v = lane < 8 ? __hip_atomic_load((gu32 *)&a.ctr[(p - 1) * 8 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : need;
                        if (__all(v >= need)) break;
                        if (timed_out(t0)) { if (lane == 0) atomicOr(a.fail, 1u); break; }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                __syncthreads();
                // sc1 loads of the activation into LDS
                const int8_t * src = a.act + ((p - 1) & 1) * 2048;
                if (threadIdx.x < 128) {
                    const int4 v = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(
                        __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, 2048, 0x00027000), threadIdx.x * 16, 0, 16));
                    *(int4 *)&s_act[threadIdx.x * 16] = v;
                } else if (threadIdx.x < 192) {
                    const float * sd = a.ad + ((p - 1) & 1) * 64;
                    s_d[threadIdx.x - 128] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        __builtin_amdgcn_make_buffer_rsrc((void *)sd, 0, 256, 0x00027000), (threadIdx.x - 128) * 4, 0, 16));
                }
                __syncthreads();
            } else {
                // every wave sweeps the granules of phase p-1 for its own needs: wave w takes
                // 512 of the 2048 inputs (8 per lane) into LDS
                const unsigned epoch = p;  // phase p-1 stored epoch p
                const gu64 * g = (const gu64 *)(a.gran + ((p - 1) & 1) * (size_t)a.M);
                unsigned v[8];
                for (;;) {
                    bool ok = true;
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        const unsigned long long x = __hip_atomic_load(g + wave * 512 + k * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        v[k] = (unsigned)x;
                        ok &= (unsigned)(x >> 32) == epoch;
                    }
                    if (__all(ok)) break;
                    if (timed_out(t0)) { if (lane == 0) atomicOr(a.fail, 2u); break; }
                }
#pragma unroll
                for (int k = 0; k < 8; k++) s_act[wave * 512 + k * 64 + lane] = (int8_t)(v[k] & 0x7f);
                if (threadIdx.x < 64) s_d[threadIdx.x] = 0.001f;
                __syncthreads();
            }
        } else {
            if (threadIdx.x < 128) *(int4 *)&s_act[threadIdx.x * 16] = make_int4(0x01010101, 0x01010101, 0x01010101, 0x01010101);
            if (threadIdx.x < 64) s_d[threadIdx.x] = 0.001f;
            __syncthreads();
        }
        const int4 xl = *(const int4 *)&s_act[lane * 32];
        const int4 xh = *(const int4 *)&s_act[lane * 32 + 16];
        const float d = s_d[lane];
        __syncthreads();  // s_act reused next phase
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int q[4] = {w[r].x, w[r].y, w[r].z, w[r].w};
            const int xs[8] = {xl.x, xl.y, xl.z, xl.w, xh.x, xh.y, xh.z, xh.w};
            int acc = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                acc = __builtin_amdgcn_sdot4((q[j] & 0x0f0f0f0f) - 0x08080808, xs[j], acc, false);
                acc = __builtin_amdgcn_sdot4(((q[j] >> 4) & 0x0f0f0f0f) - 0x08080808, xs[4 + j], acc, false);
            }
            const float f = wave_sum63(__half2float(__ushort_as_half(s[r])) * d * (float)acc);
            const int row = row0 + r;
            if (lane == 63 && active && row < a.M) {
                a.y[row] = f;
                if (GRAN) {
                    const unsigned long long x = ((unsigned long long)(p + 1) << 32) | (unsigned)((int)f & 0x7f);
                    __hip_atomic_store((gu64 *)(a.gran + (p & 1) * (size_t)a.M + row), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else if (row < 2048) {
                    // sc1 byte store
                    __hip_atomic_store((gu32 *)(a.act + (p & 1) * 2048 + (row & ~3)), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        if (!GRAN) {
            if (blockIdx.x < 8 && threadIdx.x < 64) {
                __hip_atomic_store((gu32 *)(a.ad + (p & 1) * 64 + lane), __builtin_bit_cast(unsigned, 0.001f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_fetch_add((gu32 *)&a.ctr[p * 8 + (blockIdx.x & 7)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (*(volatile unsigned *)a.fail) return;
    }
}

__global__ void k_triv(float * p) { if (threadIdx.x == 1000) p[0] = 1; }

int main(int argc, char ** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 168;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    float * y;
    int8_t * act;
    float * ad;
    unsigned * ctr;
    unsigned long long * gran;
    unsigned * fail;
    CK(hipMalloc(&y, 1 << 20));
    CK(hipMalloc(&act, 4096));
    CK(hipMalloc(&ad, 512));
    CK(hipMalloc(&ctr, (size_t)N * 8 * 4));
    CK(hipMalloc(&gran, (size_t)2 * 8192 * 8));
    CK(hipMalloc(&fail, 16));
    CK(hipMemset(act, 1, 4096));
    CK(hipMemset(ad, 0, 512));
    CK(hipMemset(fail, 0, 16));
    int4 * flush;
    CK(hipMalloc(&flush, (size_t)512 << 20));
    CK(hipMemset(flush, 0, (size_t)512 << 20));
    const size_t total = (size_t)1 << 30;
    char * pool;
    CK(hipMalloc(&pool, total));
    CK(hipMemset(pool, 0x35, total));
    hipEvent_t ea, eb;
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    int dev;
    hipDeviceProp_t prop;
    CK(hipGetDevice(&dev));
    CK(hipGetDeviceProperties(&prop, dev));
    const int G = prop.multiProcessorCount;
    printf("CUs %d\n", G);
    auto run = [&](auto kern, int M, const char * name) {
        Args a;
        a.per = (size_t)M * 64 * 18;
        a.copies = (int)(total / a.per);
        a.pool = pool;
        a.M = M;
        a.N = N;
        a.act = act;
        a.ad = ad;
        a.ctr = ctr;
        a.gran = gran;
        a.fail = fail;
        a.y = y;
        if (M % G) { printf("M %% G\n"); return; }
        float tot = 0;
        const int reps = 6;
        for (int i = 0; i < reps + 1; i++) {
            hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, st, flush, (size_t)(512 << 20) / 16, y);
            CK(hipMemsetAsync(ctr, 0, (size_t)N * 8 * 4, st));
            CK(hipMemsetAsync(gran, 0, (size_t)2 * 8192 * 8, st));
            CK(hipEventRecord(ea, st));
            hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, st, a);
            CK(hipEventRecord(eb, st));
            CK(hipEventSynchronize(eb));
            float t;
            CK(hipEventElapsedTime(&t, ea, eb));
            if (i) tot += t;
        }
        unsigned f = 0;
        CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
        const double us = tot * 1e3 / reps / N;
        printf("%-40s M=%5d  %7.2f us/phase  %7.1f GB/s  fail=%u\n", name, M, us, (double)M * 64 * 18 / (us * 1e3), f);
        if (f) exit(2);
    };
    run(k_persist<2, false>, 2048, "persist ctr R2");
    run(k_persist<2, true>, 2048, "persist gran R2");
    run(k_persist<7, false>, 7168, "persist ctr R7");
    run(k_persist<7, true>, 7168, "persist gran R7");
    run(k_persist<2, false>, 512, "persist ctr (512 rows)");
    return 0;
}
