// mv_common.hpp -- the decode matvec (k_mv) and the device helpers it shares with the
// per-head attention kernels.  Included by kernels_decode.hip and by the per-weight-type
// instantiation units mv_*.hip (so the many launch shapes compile in parallel).
#pragma once
#include "device_common.hpp"
#include "kernels.hpp"

#include <limits.h>
#include <stdio.h>

namespace rwkvmi {

// group input kinds (compile-time in k_mv)
enum MVKind : int { MVK_ACT = 0, MVK_F32 = 1, MVK_LN = 2 };


// Phase timestamps for tools/mv_probe.hip (never defined in the library build).
#ifdef MV_PROBE
__device__ unsigned long long * g_probe;
#define PROBE(k)                                                                               \
    do {                                                                                       \
        if (threadIdx.x == 0 && g_probe) g_probe[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PROBE(k) \
    do {         \
    } while (0)
#endif

// LDS image of one activation row in the consumer's format.
__device__ __forceinline__ ActBuf lds_act(char * smem, int fmt, int K) {
    ActBuf a;
    a.fmt = fmt;
    a.K = K;
    a.q = nullptr;
    a.d = a.s = nullptr;
    a.qsum = nullptr;
    a.h = nullptr;
    a.f = nullptr;
    if (fmt == A_F32) {
        a.f = (float *)smem;
    } else if (fmt == A_F16) {
        a.h = (__half *)smem;
    } else {
        const int nb = K >> 5;
        a.q = (int8_t *)smem;
        a.d = (float *)(smem + ((K + 15) & ~15));
        a.s = a.d + ((nb + 3) & ~3);
        a.qsum = (int *)(a.s + ((nb + 3) & ~3));
    }
    return a;
}

__host__ __device__ inline int lds_bytes_for(int fmt, int K) {
    if (fmt == A_F32) return K * 4;
    if (fmt == A_F16) return K * 2;
    const int nb = K / 32;
    return ((K + 15) & ~15) + 3 * ((nb + 3) & ~3) * 4;
}

// --------------------------------------------------------------------------- decode matvec
// A lane owns 16-byte "units" of a row: quantized weights one 32-block (lane + 64u), F16 eight
// halves (k = 8*lane + 512u), F32 four floats (k = 4*lane + 256u) -- the same lane/unit
// assignment and accumulation order as the batched kernel k_mm, so decode and sequence
// results are bit-identical.  All R*U weight units of a wave are loaded before anything else
// waits (rows past M clamp to M-1, units past K clamp to the last unit and are skipped in the
// dot), so the whole row-block is one HBM round trip, overlapped with the prologue.

__host__ __device__ inline int mv_units(int type, int K) {
    if (type == W_F32) return (K + 255) / 256;
    if (type == W_F16) return (K + 511) / 512;
    return (K / 32 + 63) / 64;
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const i32x4_t lds_i32x4_t;
typedef __attribute__((address_space(3))) const float lds_float_t;
typedef __attribute__((address_space(3))) const int lds_int_t;

template <bool LDS>
__device__ __forceinline__ int4 load16(const void * p) {
    if constexpr (LDS) {
        const i32x4_t t = *(const lds_i32x4_t *)(uintptr_t)p;
        return make_int4(t.x, t.y, t.z, t.w);
    } else {
        return *(const int4 *)p;
    }
}
template <bool LDS>
__device__ __forceinline__ float loadf(const float * p) {
    if constexpr (LDS) return *(const lds_float_t *)(uintptr_t)p;
    else return *p;
}
template <bool LDS>
__device__ __forceinline__ int loadi(const int * p) {
    if constexpr (LDS) return *(const lds_int_t *)(uintptr_t)p;
    else return *p;
}

// NT (default): the row is streamed once per token by this wave -- non-temporal loads
template <int WF, bool NT = true>
__device__ __forceinline__ WBlk load_unit(const DMat & W, int row, int u, int lane) {
    const int K = W.K;
    if constexpr (WF == W_F32) {
        WBlk w;
        const int k = min(lane * 4 + u * 256, K - 4);
        w.q0 = ld16w<NT>((const float *)W.qs + (size_t)row * K + k);
        return w;
    } else if constexpr (WF == W_F16) {
        WBlk w;
        const int k = min(lane * 8 + u * 512, K - 8);
        w.q0 = ld16w<NT>((const __half *)W.qs + (size_t)row * K + k);
        return w;
    } else {
        const int nb = K >> 5;
        const int b = min(lane + u * 64, nb - 1);
        return load_wblk<WF, NT>(W, (size_t)row * nb + b);
    }
}

struct AUnit {
    int4 lo, hi;
    float d, s;
    int qs;
};

template <int WF, bool LDS>
__device__ __forceinline__ AUnit load_act_unit(const ActBuf & a, int u, int lane) {
    AUnit x;
    const int K = a.K;
    if constexpr (WF == W_F32) {
        x.lo = load16<LDS>(a.f + min(lane * 4 + u * 256, K - 4));
    } else if constexpr (WF == W_F16) {
        x.lo = load16<LDS>(a.h + min(lane * 8 + u * 512, K - 8));
    } else {
        const int b = min(lane + u * 64, (K >> 5) - 1);
        x.lo = load16<LDS>(a.q + (size_t)b * 32);
        x.hi = load16<LDS>(a.q + (size_t)b * 32 + 16);
        x.d = loadf<LDS>(a.d + b);
        x.qs = loadi<LDS>(a.qsum + b);
        x.s = (WF == W_Q4_1 || WF == W_Q5_1) ? loadf<LDS>(a.s + b) : 0.0f;
    }
    return x;
}

template <int WF>
__device__ __forceinline__ bool unit_valid(int K, int u, int lane) {
    if constexpr (WF == W_F32) return lane * 4 + u * 256 < K;
    else if constexpr (WF == W_F16) return lane * 8 + u * 512 < K;
    else return lane + u * 64 < (K >> 5);
}

template <int WF>
__device__ __forceinline__ void dot_unit(const WBlk & w, const AUnit & x, float & acc, float & acc2) {
    if constexpr (WF == W_F32) {
        float s = acc;
        s = fmaf(__int_as_float(w.q0.x), __int_as_float(x.lo.x), s);
        s = fmaf(__int_as_float(w.q0.y), __int_as_float(x.lo.y), s);
        s = fmaf(__int_as_float(w.q0.z), __int_as_float(x.lo.z), s);
        s = fmaf(__int_as_float(w.q0.w), __int_as_float(x.lo.w), s);
        acc = s;
    } else if constexpr (WF == W_F16) {
        acc = dot8_f16(w.q0, x.lo, acc);
    } else {
        float dw, mw;
        const int sumi = dot_wblk<WF>(w, x.lo, x.hi, x.qs, dw, mw);
        acc = fmaf(dw * x.d, (float)sumi, acc);
        if constexpr (WF == W_Q4_1 || WF == W_Q5_1) acc2 = fmaf(mw, x.s, acc2);  // m * s exact (fp16 x fp16): = acc2 + m * s
    }
}

// Per-thread register image of a K-vector: thread t owns k = i*NT + t (i < E).
template <int E, int NT = 256>
__device__ __forceinline__ void load_vec(float (&v)[E], const float * p, int K) {
#pragma unroll
    for (int i = 0; i < E; i++) {
        // unconditional (clamped) loads: no per-load branches, so the waitcnt pass keeps
        // them all in flight
        const int k = i * NT + (int)threadIdx.x;
        const float t = p[min(k, K - 1)];
        v[i] = (k < K) ? t : 0.0f;
    }
}

// Matvec prologue (SRC_F32 / SRC_LNMIX): the waves of a workgroup build the activation image
// in LDS chunk by chunk (512 elements per wave-chunk, 8 consecutive elements per lane, so a
// quantization block is one lane quad): token-shift mix of the LayerNorm output, then ggml's
// Q8 quantization with quad DPP reductions (F16: packed halves, F32: as is).  Loading a chunk
// (chunk_load) is separate from using it (chunk_store) so the first chunk's loads can be
// issued ahead of the weight stream.
struct ChunkIn {
    float x[8], w[8], b[8], c[8], m[8];
};

__device__ __forceinline__ void ld8(float (&v)[8], const float * p) {
    const float4 t0 = *(const float4 *)p, t1 = *(const float4 *)(p + 4);
    v[0] = t0.x, v[1] = t0.y, v[2] = t0.z, v[3] = t0.w, v[4] = t1.x, v[5] = t1.y, v[6] = t1.z, v[7] = t1.w;
}

template <int SRCK, int FORM>
__device__ __forceinline__ void chunk_load(const MVEntry & E, int kc, ChunkIn & ci) {
    if constexpr (SRCK == MVK_F32) {
        ld8(ci.x, E.f + kc);
    } else {
        ld8(ci.x, E.x + kc);
        ld8(ci.w, E.lnw + kc);
        ld8(ci.b, E.lnb + kc);
        if constexpr (FORM != 2) {
            ld8(ci.c, E.carry + kc);
            ld8(ci.m, E.mu + kc);
        }
    }
}

// chunk_load for a whole workgroup without a branch: every wave issues the same raw buffer
// loads, and the waves that do not build the image (on = false, wave-uniform) get descriptors
// with no records, so their loads return zeros without touching memory.  A branch around the
// loads would make the compiler copy the loaded registers at the join -- copies that wait for
// the loads to ARRIVE, ahead of the issue-order barrier that releases the weight stream.
__device__ __forceinline__ void ld8_buf(float (&v)[8], const float * p, int kc, bool on) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, on ? 0x7fffffff : 0, 0x00020000);
    typedef float v4f_t __attribute__((ext_vector_type(4)));
    const v4f_t t0 = __builtin_amdgcn_raw_buffer_load_b128(r, kc * 4, 0, 0);
    const v4f_t t1 = __builtin_amdgcn_raw_buffer_load_b128(r, kc * 4 + 16, 0, 0);
    v[0] = t0.x, v[1] = t0.y, v[2] = t0.z, v[3] = t0.w, v[4] = t1.x, v[5] = t1.y, v[6] = t1.z, v[7] = t1.w;
}

template <int SRCK, int FORM>
__device__ __forceinline__ void chunk_load_all(const MVEntry & E, int kc, ChunkIn & ci, bool on) {
    if constexpr (SRCK == MVK_F32) {
        ld8_buf(ci.x, E.f, kc, on);
    } else {
        ld8_buf(ci.x, E.x, kc, on);
        ld8_buf(ci.w, E.lnw, kc, on);
        ld8_buf(ci.b, E.lnb, kc, on);
        if constexpr (FORM != 2) {
            ld8_buf(ci.c, E.carry, kc, on);
            ld8_buf(ci.m, E.mu, kc, on);
        }
    }
}

template <int WF, int SRCK, int FORM>
__device__ __forceinline__ void chunk_store(const MVEntry & E, const ActBuf & a, const ChunkIn & ci, float mean,
                                            float scale, bool write_carry, int k0, bool valid, int lane) {
    float v[8], xa[8];
    if constexpr (SRCK == MVK_F32) {
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = ci.x[j];
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            xa[j] = ln_apply(ci.x[j], mean, scale, ci.w[j], ci.b[j]);
            if constexpr (FORM == 2) v[j] = xa[j];
            else if constexpr (FORM == 0) v[j] = xa[j] * ci.m[j] + (ci.c[j] - ci.c[j] * ci.m[j]);
            else v[j] = (ci.c[j] - xa[j]) * ci.m[j] + xa[j];
        }
    }
    // The carry (LayerNorm output) is stored last: vmcnt counts loads and stores in one order, so a
    // global store issued before the last use of the inputs makes the waits for those inputs also
    // wait for weight loads issued after them (measured: the carry-writing workgroup ended last).
    auto store_carry = [&]() {
        if constexpr (SRCK != MVK_F32) {
            if (write_carry && valid) {
                *(float4 *)(E.carry_out + k0) = make_float4(xa[0], xa[1], xa[2], xa[3]);
                *(float4 *)(E.carry_out + k0 + 4) = make_float4(xa[4], xa[5], xa[6], xa[7]);
            }
        }
    };
    if constexpr (WF == W_F32) {
        if (valid) {
            *(float4 *)(a.f + k0) = make_float4(v[0], v[1], v[2], v[3]);
            *(float4 *)(a.f + k0 + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
        store_carry();
    } else if constexpr (WF == W_F16) {
        int p[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            p[j] = __builtin_bit_cast(int, __halves2half2(to_half(v[2 * j]), to_half(v[2 * j + 1])));
        if (valid) *(int4 *)(a.h + k0) = make_int4(p[0], p[1], p[2], p[3]);
        store_carry();
    } else {
        // ggml quantize_row_q8_0 / q8_1 (x86): d = amax/127, q = rint(x*127/amax)
        float am = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) am = fmaxf(am, fabsf(v[j]));
        am = fmaxf(am, __int_as_float(dpp_mov<0xB1>(__float_as_int(am))));
        am = fmaxf(am, __int_as_float(dpp_mov<0x4E>(__float_as_int(am))));
        const float d = am / 127.f;
        const float id = (am != 0.0f) ? 127.f / am : 0.0f;
        int lo = 0, hi = 0, sum = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int q = (int)rintf(v[j] * id);
            sum += q;
            if (j < 4) lo |= (q & 0xff) << (8 * j);
            else hi |= (q & 0xff) << (8 * (j - 4));
        }
        sum += dpp_mov<0xB1>(sum);
        sum += dpp_mov<0x4E>(sum);
        if (valid) {
            *(int2 *)(a.q + k0) = make_int2(lo, hi);
            if ((lane & 3) == 0) {
                const int bi = k0 >> 5;
                a.d[bi] = f16_round(d);
                a.qsum[bi] = sum;
                if (a.fmt == A_Q8_1) a.s[bi] = f16_round(d * (float)sum);
            }
        }
        store_carry();
    }
}

// Hand-off of a C-vector inside a fused decode launch (the head / channel outputs y feeding the
// Wo rows): every element is a granule {tag (high word), value bits (low word)} written by ONE
// aligned 8-byte agent-scope store, so the data is its own flag.  The gathering waves of a
// workgroup (wave, wave + nwaves, ... over 512-element chunks; 8 consecutive granules per lane, so
// a quad holds one quantization block) re-read their chunk, sleeping between passes, until every
// tag reads `tag`, then write it into the LDS image in WF's activation format with the matvec
// prologue's SRC_F32 arithmetic (chunk_store): Wo's input bits equal a separate Wo launch's.  The
// poll IS the gather -- one round trip after the last value lands, not a flag poll and then a
// gather.  Bounded: after spin_max passes *err (a host-mapped word) is set at system scope.
typedef __attribute__((address_space(1))) unsigned long long gran_u64_t;
typedef __attribute__((address_space(1))) unsigned gran_u32_t;
template <int WF>
__device__ __forceinline__ void gran_gather_image(const unsigned long long * yg, unsigned tag, int C, const ActBuf & img,
                                                  int wave, int nwaves, unsigned * err, unsigned spin_max, int lane) {
    MVEntry none{};
    for (int ck = wave; ck * LN_CHUNK < C; ck += nwaves) {
        const int k0 = ck * LN_CHUNK + lane * 8;
        const bool valid = k0 < C;
        const unsigned long long * g = yg + max(min(k0, C - 8), 0);
        ChunkIn ci;
        for (unsigned it = 0;; it++) {
            unsigned long long x[8];
#pragma unroll
            for (int j = 0; j < 8; j++)
                x[j] = __hip_atomic_load((gran_u64_t *)(g + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool ok = true;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                ci.x[j] = __uint_as_float((unsigned)x[j]);
                ok = ok && (unsigned)(x[j] >> 32) == tag;
            }
            if (__all(ok || !valid)) break;
            if (it >= spin_max) {
                __hip_atomic_store((gran_u32_t *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        chunk_store<WF, MVK_F32, 0>(none, img, ci, 0.0f, 1.0f, false, k0, valid, lane);
    }
}

// Wait before a gather: ONE wave polls n granules (lane i: yg[off + i * stride], n <= 64) with a
// sleep between passes until every tag reads `tag` -- a few hundred bytes per pass instead of the
// gather's whole vector, so a waiting workgroup adds little traffic beside the producers' weight
// streams (the gather after it checks every tag again).  Bounded like the gather.  (Several passes
// in flight at once -- a rolling poll -- measured far slower: v6-1B6 750 vs 693 us/token.)
__device__ __forceinline__ void gran_prepoll(const unsigned long long * yg, int n, int stride, int off, unsigned tag,
                                             unsigned * err, unsigned spin_max, int lane) {
    for (unsigned it = 0;; it++) {
        const unsigned long long x = lane < n ? __hip_atomic_load((gran_u64_t *)(yg + off + (size_t)lane * stride),
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                              : ((unsigned long long)tag << 32);
        if (__all((unsigned)(x >> 32) == tag)) return;
        if (it >= spin_max) {
            __hip_atomic_store((gran_u32_t *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

// Q8 blocks published by pub_q8 (KG_STRIDE granules per 32-element block, nb blocks) -> the LDS
// activation image: thread tid of nthr reads granules tid + nthr i (i < GI), re-reading until every
// tag it holds reads `tag` (bounded like the gather above), then writes the q dwords, d and Q8_1's
// s.  The caller recomputes the qsums (q8_image_qsum) after a barrier.
template <int GI>
__device__ __forceinline__ void q8_gather_image(const unsigned long long * kg, int nb, unsigned tag, const ActBuf & img,
                                                int tid, int nthr, unsigned * err, unsigned spin_max) {
    const int ng = KG_STRIDE * nb;
    unsigned pay[GI];
    for (unsigned it = 0;; it++) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < GI; i++) {
            const int g = tid + nthr * i;
            unsigned long long x = (unsigned long long)tag << 32;
            if (g < ng) x = __hip_atomic_load((gran_u64_t *)(kg + g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pay[i] = (unsigned)x;
            ok = ok && (unsigned)(x >> 32) == tag;
        }
        if (__all(ok)) break;
        if (it >= spin_max) {
            __hip_atomic_store((gran_u32_t *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
#pragma unroll
    for (int i = 0; i < GI; i++) {
        const int g = tid + nthr * i;
        if (g < ng) {
            const int b = g / KG_STRIDE, j = g - b * KG_STRIDE;
            if (j < 8) *(unsigned *)(img.q + (size_t)b * 32 + 4 * j) = pay[i];
            else if (j == 8) img.d[b] = __uint_as_float(pay[i]);
            else if (img.fmt == A_Q8_1) img.s[b] = __uint_as_float(pay[i]);
        }
    }
}
// the exact integer block sums of a gathered Q8 image (store32's qsum)
__device__ __forceinline__ void q8_image_qsum(const ActBuf & img, int nb, int tid, int nthr) {
    for (int b = tid; b < nb; b += nthr) {
        const int4 lo = *(const int4 *)(img.q + (size_t)b * 32), hi = *(const int4 *)(img.q + (size_t)b * 32 + 16);
        const int ws[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        int s = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) s = __builtin_amdgcn_sdot4(ws[k], 0x01010101, s, false);
        img.qsum[b] = s;
    }
}

// Row sums r = 0..R-1 (valid in lane 63 after wave_sum63) gathered so that lane r holds row r's
// sum: the rows' epilogues (exp/tanh chains) then run side by side in R lanes instead of one
// after another in lane 63.  Pure data movement: results are bit-identical.
template <int R>
__device__ __forceinline__ float lane_row_sum(const float (&s)[R], int lane) {
    float mine = 0.0f;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const float v = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s[r]), 63));
        mine = lane == r ? v : mine;
    }
    return mine;
}

// R rows whose U units per lane are already in registers, dotted with an LDS activation image:
// k_mva's per-row arithmetic (lane/unit order, wave_sum63 tree; the unit count mv_units(WF, K)
// must be <= U).  Lane r < R returns row r's sum.
template <int WF, int R, int U>
__device__ __forceinline__ float rows_dot_img(const WBlk (&w)[R][U], const ActBuf & img, int K, int lane) {
    float acc[R], acc2[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const AUnit xu = load_act_unit<WF, true>(img, u, lane);
        const bool uv = unit_valid<WF>(K, u, lane);
#pragma unroll
        for (int r = 0; r < R; r++) {
            float t = acc[r], t2 = acc2[r];
            dot_unit<WF>(w[r][u], xu, t, t2);
            acc[r] = uv ? t : acc[r];
            acc2[r] = uv ? t2 : acc2[r];
        }
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    float s[R];
#pragma unroll
    for (int r = 0; r < R; r++) s[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
    return lane_row_sum<R>(s, lane);
}

// Epilogue operands of one output row, loaded at kernel start (not after the dots).
struct EpiIn {
    float y, aux, bias;
};
// Branch-free: absent operands read a zero word instead (uniform pointer select), so these
// loads never split the kernel into blocks that make the waitcnt pass drain the weight stream.
static __device__ const float g_mv_zero[4] = {0.0f, 0.0f, 0.0f, 0.0f};
__device__ __forceinline__ EpiIn epi_load(const MVEntry & E, int row) {
    EpiIn p;
    const float * py = E.y ? E.y + row : g_mv_zero;
    const float * pa = E.aux ? E.aux + row : g_mv_zero;
    const float * pb = E.bias ? E.bias + row : g_mv_zero;
    p.y = *py;
    p.aux = *pa;
    p.bias = *pb;
    return p;
}
__device__ __forceinline__ float epi_apply(int epi, float acc, const EpiIn & p) {
    switch (epi) {
        case EPI_SIGMOID: return sigmoidf_(acc);
        case EPI_TANH: return rk_tanhf(acc);
        case EPI_SILU: return siluf_(acc);
        case EPI_RELU_SQ: {
            const float r = acc > 0.0f ? acc : 0.0f;
            return r * r;
        }
        case EPI_ADD: return p.y + acc;
        case EPI_SIGMUL_ADD: return p.y + sigmoidf_(p.aux) * acc;
        case EPI_DECAY6: return rk_expf(-rk_expf(acc + p.bias));
        case EPI_DECAY7: return rk_expf(sigmoidf_(acc + p.bias) * -0.606531f);
        case EPI_SIGMOID_BIAS: return sigmoidf_(acc + p.bias);
        case EPI_VMIX7: return p.y + (p.aux - p.y) * sigmoidf_(acc + p.bias);
        default: return acc;
    }
}

// wave_sum63's fixed tree applied to partials held by one thread: p[l] is what lane l of the
// batched kernel (k_mm) accumulates for a row whose units fit in lanes 0..31 (one unit each).
__device__ __forceinline__ float tree16(const float * p) {
    const float q0 = (p[0] + p[1]) + (p[2] + p[3]);
    const float q1 = (p[4] + p[5]) + (p[6] + p[7]);
    const float q2 = (p[8] + p[9]) + (p[10] + p[11]);
    const float q3 = (p[12] + p[13]) + (p[14] + p[15]);
    return (q0 + q1) + (q2 + q3);
}
__device__ __forceinline__ float tree_wave32(const float (&p)[32]) {
    const float r0 = tree16(p), r1 = tree16(p + 16);
    return (0.0f + 0.0f) + (r1 + r0);
}

// One row of the v6 decay LoRA tail by one thread: lanes 0..nl-1 of k_mm's row (nl <= NL <= 32,
// one unit each); the first PF units were prefetched into wp[].  Partials of lanes >= NL are
// compile-time zeros, so the tree folds to the nonzero part.
template <int WF, int PF, int NL, bool NT = true>
__device__ __forceinline__ float decay_row_thread(const DMat & W, int row, const ActBuf & act, int nl,
                                                  const WBlk (&wp)[PF > 0 ? PF : 1]) {
    float p[32], p2[32];
#pragma unroll
    for (int l = 0; l < 32; l++) {
        p[l] = p2[l] = 0.0f;
        if (l < NL && l < nl) {
            const WBlk w = (l < PF) ? wp[l < PF ? l : 0] : load_unit<WF, NT>(W, row, 0, l);
            const AUnit x = load_act_unit<WF, true>(act, 0, l);
            dot_unit<WF>(w, x, p[l], p2[l]);
        }
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    return one ? tree_wave32(p) + tree_wave32(p2) : tree_wave32(p) + 0.0f;
}

// One workgroup = NW waves (SRC_ACT) or 2 NW waves (prologue sources); RW rows per row block.
// stride > 0: the workgroup walks row blocks wgi, wgi+stride, ... with one prologue.
// Prologue sources (SRC_F32 / SRC_LNMIX): waves NW..2NW-1 build the activation image in LDS
// (LayerNorm statistics, one 512-element chunk each, token shift, quantization); their input
// loads go out first (issue-order barrier) and the streaming waves' weight loads right behind
// them, then the streaming waves dot the block's rows once the image is ready.
template <int WF, int R, int U, int SRCK, int FORM, bool EMIT, int NW, int LNP>
__device__ __forceinline__ void mv_body(const MVEntry & Ent, int wgi, int b0, int stride, char * smem, float * red,
                                        int late, unsigned long long * stamp_mid = nullptr,
                                        unsigned long long * stamp_x = nullptr) {
    constexpr bool PRO = SRCK != MVK_ACT;
    // LayerNorm chunks per prologue wave held in registers: LNP 32 -> K <= 2048, 64 -> K <= 4096
    constexpr int LCW = LNP > 32 ? 2 : 1;
    // Prologue groups with K <= 2048 (one LayerNorm chunk per image wave; larger K: mv_body_split):
    // the rows of a block go over all 2 NW waves -- the image waves too, so the per-wave dot and
    // reduction chains are half as long.
    constexpr bool IMGR = PRO;
    constexpr int NWT = (PRO && IMGR) ? 2 * NW : NW;  // waves with rows
    constexpr int RR = (PRO && !IMGR) ? 2 * R : R;    // rows per wave with rows
    constexpr int RW = NWT * RR;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform branches
    const DMat & W = Ent.W;
    const int M = W.M, K = W.K;
    const int nblk = (M + RW - 1) / RW;
    const int units = mv_units(WF, K);
    PROBE(0);
    // every scalar the epilogue needs, in SGPRs before anything waits: a kernarg field first read
    // after the dots is a scalar-cache round trip on the kernel's critical path
    const int epi = Ent.epi;
    float * const ey = Ent.y;
    ActBuf ao = Ent.act_out;
    const bool emit_on = EMIT && Ent.emit && ao.fmt >= 0;
    asm volatile("" ::"s"(epi), "s"(ey));
    if constexpr (EMIT) pin_act(ao);
    ActBuf a;
    const bool pro_wave = PRO && wave >= NW;
    const int pw = wave - NW, nch = (K + LN_CHUNK - 1) / LN_CHUNK;
    const bool write_carry = PRO && Ent.carry_out && (int)blockIdx.x == b0;  // one writer per entry
    ChunkIn ci[LCW];
    int kc[LCW];
    float mean = 0.0f, scale = 0.0f;
    if constexpr (PRO) {
        a = lds_act(smem, act_fmt_for(WF), K);
        // the image waves' inputs: chunks pw, pw + NW (512 elements each, 8 per lane); issued
        // by every wave without a branch (chunk_load_all: the dot waves' loads are empty)
#pragma unroll
        for (int q = 0; q < LCW; q++) {
            kc[q] = (pw + q * NW) * LN_CHUNK + lane * 8;
            chunk_load_all<SRCK, FORM>(Ent, max(min(kc[q], K - 8), 0), ci[q], pro_wave);
        }
        // the weight pointers reach SGPRs before the issue-order barrier, so the stream starts
        // right after it (a kernarg scalar load behind the barrier is a round trip in the path)
        asm volatile("" ::"s"(W.qs), "s"(W.sc), "s"(W.qh));
        // issue order: the image inputs go out before any weight stream starts
        asm volatile("s_barrier" ::: "memory");
    }
    // ---- this wave's weight units (HBM), all in flight before anything waits
    const bool has_rows = !pro_wave || IMGR;
    int row0 = wgi * RW + wave * RR;
    int rows[RR];
#pragma unroll
    for (int r = 0; r < RR; r++) rows[r] = min(row0 + r, M - 1);
    WBlk w[RR][U];
    auto issue_w = [&]() {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < RR; r++) w[r][u] = load_unit<WF>(W, rows[r], u, lane);
    };
    if (has_rows) issue_w();
    if constexpr (PRO) {
        if (pro_wave) {
            if constexpr (SRCK == MVK_LN) {
                // LayerNorm statistics in the chunk association (device_common.hpp, one pass): each
                // image wave sums its chunks and their squares, the chunk sums meet in LDS (one
                // barrier every wave joins)
                __shared__ double ln_part[2][8];
#pragma unroll
                for (int q = 0; q < LCW; q++)
                    if (pw + q * NW < nch) {
                        double c1, c2;
                        ln_chunk_sums(ci[q].x, kc[q] < K, c1, c2);
                        if (lane == 0) {
                            ln_part[0][pw + q * NW] = c1;
                            ln_part[1][pw + q * NW] = c2;
                        }
                    }
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                double s1 = 0.0, s2 = 0.0;
                for (int c = 0; c < nch; c++) s1 += ln_part[0][c], s2 += ln_part[1][c];
                ln_finish(s1, s2, K, 1e-5f, mean, scale);
            }
#ifdef RWKV_STAMP
            if (pw == 0 && stamp_x && lane == 0) stamp_x[1] = __builtin_amdgcn_s_memrealtime() + (scale == 1.2345f);
#endif
#pragma unroll
            for (int q = 0; q < LCW; q++)
                if (pw + q * NW < nch) chunk_store<WF, SRCK, FORM>(Ent, a, ci[q], mean, scale, false, kc[q], kc[q] < K, lane);
            if constexpr (SRCK == MVK_F32) {
                // plain fp32 input: any K, further chunks streamed
                for (int c = pw + LCW * NW; c < nch; c += NW) {
                    const int kk = c * LN_CHUNK + lane * 8;
                    chunk_load<SRCK, FORM>(Ent, min(kk, K - 8), ci[0]);
                    chunk_store<WF, SRCK, FORM>(Ent, a, ci[0], mean, scale, write_carry, kk, kk < K, lane);
                }
            }
#ifdef RWKV_STAMP
            if (pw == 0 && stamp_x) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane == 0) stamp_x[2] = __builtin_amdgcn_s_memrealtime();
            }
#endif
        } else if constexpr (SRCK == MVK_LN) {
            asm volatile("s_barrier" ::: "memory");  // the image waves' statistics exchange
        }
    }
    // epilogue operands: !EMIT lane r < R runs row row0 + r's epilogue; EMIT thread tid < RW row tid
    EpiIn ep;
    if constexpr (!EMIT) ep = epi_load(Ent, min(row0 + min(lane, RR - 1), M - 1));
    else ep = epi_load(Ent, min(wgi * RW + (tid < RW ? tid : 0), M - 1));
    if constexpr (PRO) __syncthreads();  // activation image ready
    else a = Ent.act;
    PROBE(1);
#ifdef RWKV_STAMP
    if (stamp_mid && wgi == (int)blockIdx.x - b0) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        *stamp_mid = __builtin_amdgcn_s_memrealtime();
    }
#endif

    for (;;) {
        // dots (the waves with rows)
        constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
        float s[RR];
        if (has_rows) {
            float acc[RR], acc2[RR];
#pragma unroll
            for (int r = 0; r < RR; r++) acc[r] = acc2[r] = 0.0f;
            for (int u0 = 0; u0 < units; u0 += U) {
                if (u0 > 0) {
#pragma unroll
                    for (int u = 0; u < U; u++)
#pragma unroll
                        for (int r = 0; r < RR; r++) w[r][u] = load_unit<WF>(W, rows[r], u0 + u, lane);
                }
                AUnit x[U];
#pragma unroll
                for (int u = 0; u < U; u++) x[u] = load_act_unit<WF, PRO>(a, u0 + u, lane);
#pragma unroll
                for (int u = 0; u < U; u++) {
                    if (unit_valid<WF>(K, u0 + u, lane)) {
#pragma unroll
                        for (int r = 0; r < RR; r++) dot_unit<WF>(w[r][u], x[u], acc[r], acc2[r]);
                    }
                }
            }
            // reduce
#pragma unroll
            for (int r = 0; r < RR; r++) s[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
        } else {
#pragma unroll
            for (int r = 0; r < RR; r++) s[r] = 0.0f;
        }
        if constexpr (!EMIT) {
#ifdef MV_PROBE
            if (s[0] == 1.2345f) g_probe[0] = 0;  // orders the stamp after the dots
#endif
            PROBE(2);
            const float v = epi_apply(epi, lane_row_sum<RR>(s, lane), ep);
            if (has_rows && lane < RR && row0 + lane < M) ey[row0 + lane] = v;
        } else {
            // RW rows per block (a multiple of 32): apply the epilogue and emit each 32 rows as
            // one quantization block of the next matmul's input (ggml Q8 / fp16 / fp32)
#pragma unroll
            for (int r = 0; r < RR; r++)
                if (has_rows && lane == 63) red[wave * RR + r] = s[r];
#ifdef RWKV_STAMP
            if (wave == 0 && stamp_x && lane == 0) stamp_x[3] = __builtin_amdgcn_s_memrealtime() + (s[0] == 1.2345f);
#endif
            __syncthreads();
            PROBE(2);
            if (tid < RW) {
                const int row = wgi * RW + tid;
                float vv = 0.0f;
                if (row < M) {
                    vv = epi_apply(epi, red[tid], ep);
                    if (ey) ey[row] = vv;
                }
                if (emit_on) emit32(ao, 0, row, vv);
            }
        }
        PROBE(3);
        wgi += stride;
        if (stride <= 0 || wgi >= nblk) break;
        if constexpr (EMIT) __syncthreads();  // red[] reuse
        row0 = wgi * RW + wave * RR;
#pragma unroll
        for (int r = 0; r < RR; r++) rows[r] = min(row0 + r, M - 1);
        if (has_rows) issue_w();
        if constexpr (!EMIT) ep = epi_load(Ent, min(row0 + min(lane, RR - 1), M - 1));
        else ep = epi_load(Ent, min(wgi * RW + (tid < RW ? tid : 0), M - 1));
    }
    if constexpr (SRCK == MVK_LN) {
        // the carry (this LayerNorm output, the next token's shift input) after the rows: vmcnt
        // counts loads and stores in one order, so a store ahead of the dots would make waits
        // for earlier loads also wait for the weight stream behind it
        if (pro_wave && write_carry) {
#pragma unroll
            for (int q = 0; q < LCW; q++)
                if (pw + q * NW < nch && kc[q] < K) {
                    float xa[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) xa[j] = ln_apply(ci[q].x[j], mean, scale, ci[q].w[j], ci[q].b[j]);
                    *(float4 *)(Ent.carry_out + kc[q]) = make_float4(xa[0], xa[1], xa[2], xa[3]);
                    *(float4 *)(Ent.carry_out + kc[q] + 4) = make_float4(xa[4], xa[5], xa[6], xa[7]);
                }
        }
    }
    if constexpr (SRCK == MVK_LN && FORM != 2) {
        // the entry's first workgroup, after its rows: the same LayerNorm output mixed with mu2
        // into a global activation row (the channel-mix receptance input of k_mvsig).  (Spread
        // block-interleaved over all workgroups instead: 704 vs 695 us/token -- every workgroup's
        // image waves then pay the reload and quantization pass.)
        if (pro_wave && Ent.mu2 && (int)blockIdx.x == b0) {
            MVEntry E2 = Ent;
            E2.mu = Ent.mu2;
#pragma unroll
            for (int q = 0; q < LCW; q++)
                if (pw + q * NW < nch) {
                    ld8(ci[q].m, Ent.mu2 + min(kc[q], K - 8));
                    chunk_store<WF, SRCK, FORM>(E2, Ent.act2_out, ci[q], mean, scale, false, kc[q], kc[q] < K, lane);
                }
        }
    }
}

// Prologue groups with K > 2048: the image waves hold two LayerNorm chunks of inputs, so they stay
// rowless (the NW streaming waves take 2 R rows each), and the two roles run as separate straight
// paths that meet only at barriers.  With both roles in one path the compiler keeps the streaming
// waves' weight registers live through the image waves' statistics (it cannot tell the two wave
// conditions apart), the kernel needs 145-235 VGPRs -- one workgroup per CU -- and the multi-round
// LayerNorm groups of the 2.9B / 7B models ran 10-14 % slower.  Same arithmetic and association as
// mv_body (bit-identical); the barrier sequence of both paths matches one for one.
// Outputs of a producer group handed to consumers in the same launch (mv_ffnf.hpp): an emitting
// entry publishes each 32-row Q8 block as KG_STRIDE granules {tag, dword} -- the block's 32 int8 (4
// per granule), its fp16-rounded d and Q8_1's fp16-rounded d * sum (the qsum is an exact integer sum
// the consumer recomputes) -- and a plain entry its rows' values as granules: emit32's bits.
struct GranPub {
    unsigned long long * kg;  // KG_STRIDE granules per 32-row block of the emitting entry
    unsigned long long * rg;  // one granule per row of the other entry
    unsigned tag;
};
// lanes 0..31 (one half-wave, block-uniform): rows 32 b .. 32 b + 31 of the emitting entry
__device__ __forceinline__ void pub_q8(unsigned long long * kg, int b, float v, unsigned tag, int lane) {
    const Q32 q = quant32(v);
    unsigned p = ((unsigned)q.q & 0xffu) << (8 * (lane & 3));
    p |= (unsigned)__shfl_xor((int)p, 1);
    p |= (unsigned)__shfl_xor((int)p, 2);
    const unsigned long long t = (unsigned long long)tag << 32;
    unsigned long long * const g = kg + (size_t)b * KG_STRIDE;
    if ((lane & 3) == 0)
        __hip_atomic_store((gran_u64_t *)(g + ((lane & 31) >> 2)), t | p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((lane & 31) == 0) {
        __hip_atomic_store((gran_u64_t *)(g + 8), t | __float_as_uint(f16_round(q.d)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((gran_u64_t *)(g + 9), t | __float_as_uint(f16_round(q.d * (float)q.sum)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int WF, int R, int U, int SRCK, int FORM, bool EMIT, int NW, int LNP, bool PUB = false>
__device__ __forceinline__ void mv_body_split(const MVEntry & Ent, int wgi, int b0, int stride, char * smem,
                                              float * red, int late, const GranPub * pub = nullptr) {
    constexpr int LCW = LNP > 32 ? 2 : 1;
    constexpr int RR = 2 * R, RW = NW * RR;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const DMat & W = Ent.W;
    const int M = W.M, K = W.K;
    const int nblk = (M + RW - 1) / RW;
    const int units = mv_units(WF, K);
    const int nch = (K + LN_CHUNK - 1) / LN_CHUNK;
    const ActBuf a = lds_act(smem, act_fmt_for(WF), K);
    if (wave >= NW) {
        // ---- image waves: inputs, statistics, the image; then only the barriers of the rows
        const int pw = wave - NW;
        const bool write_carry = Ent.carry_out && (int)blockIdx.x == b0;
        ChunkIn ci[LCW];
        int kc[LCW];
#pragma unroll
        for (int q = 0; q < LCW; q++) {
            kc[q] = (pw + q * NW) * LN_CHUNK + lane * 8;
            chunk_load<SRCK, FORM>(Ent, min(kc[q], K - 8), ci[q]);
        }
        asm volatile("s_barrier" ::: "memory");  // issue order: the image inputs ahead of the weights
        float mean = 0.0f, scale = 0.0f;
        if constexpr (SRCK == MVK_LN) {
            __shared__ double ln_part[2][8];
#pragma unroll
            for (int q = 0; q < LCW; q++)
                if (pw + q * NW < nch) {
                    double c1, c2;
                    ln_chunk_sums(ci[q].x, kc[q] < K, c1, c2);
                    if (lane == 0) {
                        ln_part[0][pw + q * NW] = c1;
                        ln_part[1][pw + q * NW] = c2;
                    }
                }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            double s1 = 0.0, s2 = 0.0;
            for (int c = 0; c < nch; c++) s1 += ln_part[0][c], s2 += ln_part[1][c];
            ln_finish(s1, s2, K, 1e-5f, mean, scale);
        }
#pragma unroll
        for (int q = 0; q < LCW; q++)
            if (pw + q * NW < nch) chunk_store<WF, SRCK, FORM>(Ent, a, ci[q], mean, scale, false, kc[q], kc[q] < K, lane);
        if constexpr (SRCK == MVK_F32) {
            for (int c = pw + LCW * NW; c < nch; c += NW) {
                const int kk = c * LN_CHUNK + lane * 8;
                chunk_load<SRCK, FORM>(Ent, min(kk, K - 8), ci[0]);
                chunk_store<WF, SRCK, FORM>(Ent, a, ci[0], mean, scale, false, kk, kk < K, lane);
            }
        }
        __syncthreads();  // activation image ready
        for (;;) {
            if constexpr (EMIT) __syncthreads();  // the streaming waves' row sums in red[]
            wgi += stride;
            if (stride <= 0 || wgi >= nblk) break;
            if constexpr (EMIT) __syncthreads();  // red[] reuse
        }
        if constexpr (SRCK == MVK_LN) {
            if (write_carry) {  // after the rows (see mv_body)
#pragma unroll
                for (int q = 0; q < LCW; q++)
                    if (pw + q * NW < nch && kc[q] < K) {
                        float xa[8];
#pragma unroll
                        for (int j = 0; j < 8; j++) xa[j] = ln_apply(ci[q].x[j], mean, scale, ci[q].w[j], ci[q].b[j]);
                        *(float4 *)(Ent.carry_out + kc[q]) = make_float4(xa[0], xa[1], xa[2], xa[3]);
                        *(float4 *)(Ent.carry_out + kc[q] + 4) = make_float4(xa[4], xa[5], xa[6], xa[7]);
                    }
            }
        }
        if constexpr (SRCK == MVK_LN && FORM != 2) {
            if (Ent.mu2 && (int)blockIdx.x == b0) {
                MVEntry E2 = Ent;
                E2.mu = Ent.mu2;
#pragma unroll
                for (int q = 0; q < LCW; q++)
                    if (pw + q * NW < nch) {
                        ld8(ci[q].m, Ent.mu2 + min(kc[q], K - 8));
                        chunk_store<WF, SRCK, FORM>(E2, Ent.act2_out, ci[q], mean, scale, false, kc[q], kc[q] < K, lane);
                    }
            }
        }
    } else {
        // ---- streaming waves: weights at once, the rows after the image
        const int epi = Ent.epi;
        float * const ey = Ent.y;
        ActBuf ao = Ent.act_out;
        const bool emit_on = EMIT && Ent.emit && ao.fmt >= 0;
        asm volatile("" ::"s"(epi), "s"(ey));
        if constexpr (EMIT) pin_act(ao);
        asm volatile("" ::"s"(W.qs), "s"(W.sc), "s"(W.qh));
        asm volatile("s_barrier" ::: "memory");  // issue order
        int row0 = wgi * RW + wave * RR;
        int rows[RR];
#pragma unroll
        for (int r = 0; r < RR; r++) rows[r] = min(row0 + r, M - 1);
        WBlk w[RR][U];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < RR; r++) w[r][u] = load_unit<WF>(W, rows[r], u, lane);
        if constexpr (SRCK == MVK_LN) asm volatile("s_barrier" ::: "memory");  // the statistics exchange
        EpiIn ep;
        if constexpr (!EMIT) ep = epi_load(Ent, min(row0 + min(lane, RR - 1), M - 1));
        else ep = epi_load(Ent, min(wgi * RW + (tid < RW ? tid : 0), M - 1));
        __syncthreads();  // activation image ready
        for (;;) {
            constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
            float acc[RR], acc2[RR];
#pragma unroll
            for (int r = 0; r < RR; r++) acc[r] = acc2[r] = 0.0f;
            for (int u0 = 0; u0 < units; u0 += U) {
                if (u0 > 0) {
#pragma unroll
                    for (int u = 0; u < U; u++)
#pragma unroll
                        for (int r = 0; r < RR; r++) w[r][u] = load_unit<WF>(W, rows[r], u0 + u, lane);
                }
                AUnit x[U];
#pragma unroll
                for (int u = 0; u < U; u++) x[u] = load_act_unit<WF, true>(a, u0 + u, lane);
#pragma unroll
                for (int u = 0; u < U; u++) {
                    if (unit_valid<WF>(K, u0 + u, lane)) {
#pragma unroll
                        for (int r = 0; r < RR; r++) dot_unit<WF>(w[r][u], x[u], acc[r], acc2[r]);
                    }
                }
            }
            float s[RR];
#pragma unroll
            for (int r = 0; r < RR; r++) s[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
            if constexpr (!EMIT) {
                const float v = epi_apply(epi, lane_row_sum<RR>(s, lane), ep);
                if (lane < RR && row0 + lane < M) ey[row0 + lane] = v;
            } else {
#pragma unroll
                for (int r = 0; r < RR; r++)
                    if (lane == 63) red[wave * RR + r] = s[r];
                __syncthreads();
                if (tid < RW) {
                    const int row = wgi * RW + tid;
                    float vv = 0.0f;
                    if (row < M) {
                        vv = epi_apply(epi, red[tid], ep);
                        if constexpr (PUB) {
                            if (!emit_on)
                                __hip_atomic_store((gran_u64_t *)(pub->rg + row),
                                                   ((unsigned long long)pub->tag << 32) | __float_as_uint(vv),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        } else if (ey) {
                            ey[row] = vv;
                        }
                    }
                    if (emit_on) {
                        if constexpr (PUB) pub_q8(pub->kg, wgi, vv, pub->tag, tid);
                        else emit32(ao, 0, row, vv);
                    }
                }
            }
            wgi += stride;
            if (stride <= 0 || wgi >= nblk) break;
            if constexpr (EMIT) __syncthreads();  // red[] reuse
            row0 = wgi * RW + wave * RR;
#pragma unroll
            for (int r = 0; r < RR; r++) rows[r] = min(row0 + r, M - 1);
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int r = 0; r < RR; r++) w[r][u] = load_unit<WF>(W, rows[r], u, lane);
            if constexpr (!EMIT) ep = epi_load(Ent, min(row0 + min(lane, RR - 1), M - 1));
            else ep = epi_load(Ent, min(wgi * RW + (tid < RW ? tid : 0), M - 1));
        }
    }
}

// mv_body, or mv_body_split for the prologue groups with K > 2048
template <int WF, int R, int U, int SRCK, int FORM, bool EMIT, int NW, int LNP>
__device__ __forceinline__ void mv_run(const MVEntry & Ent, int wgi, int b0, int stride, char * smem, float * red,
                                       int late, unsigned long long * stamp_mid, unsigned long long * stamp_x) {
    // every prologue group in the split form (K <= 2048 too: v6-1B6 decode 686-692 vs 696-698 us per
    // token with the image waves carrying rows in mv_body, v4-169M 244 vs 251); MV_IMG_ROWS: mv_body
#ifdef MV_IMG_ROWS
    constexpr int LNS = 32;
#else
    constexpr int LNS = 0;
#endif
    if constexpr (SRCK != MVK_ACT && LNP > LNS) mv_body_split<WF, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, stride, smem, red, late);
    else mv_body<WF, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, stride, smem, red, late, stamp_mid, stamp_x);
}

// WFIX >= 0: every entry of the group has weight type WFIX (one body, fewer registers);
// WFIX < 0: per-entry switch.  SRCK / FORM: the group's input source and token-shift form
// (compile-time, so the prologue has no data-independent branches).
//
// The entry's first workgroups b1..b7 (b_i = e[i].block0, or INT_MAX past the last entry) are
// scalar arguments ahead of the group so the code object preloads them into SGPRs
// (-amdgpu-kernarg-preload-count): the entry index is SALU compares, and the entry's weight
// pointers are one scalar-load round trip away from the kernel's first instruction (a loop
// over g.e[].block0 would be one dependent kernarg load per entry).
template <int R, int U, int SRCK, int FORM, bool EMIT, int WFIX, int LNP>
__global__ __launch_bounds__(512) void k_mv(int b1, int b2, int b3, int b4, int b5, int b6, int b7, MVGroup g) {
    constexpr int NW = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float red[(SRCK == MVK_ACT ? NW : 2 * NW) * R];
    const int bx = (int)blockIdx.x;
    const int e = (bx >= b1) + (bx >= b2) + (bx >= b3) + (bx >= b4) + (bx >= b5) + (bx >= b6) + (bx >= b7);
    const int b0 = e == 0 ? 0 : e == 1 ? b1 : e == 2 ? b2 : e == 3 ? b3 : e == 4 ? b4 : e == 5 ? b5 : e == 6 ? b6 : b7;
    const MVEntry & Ent = g.e[e];
    const int wgi = bx - b0;
    STAMP_BEGIN();
#ifdef RWKV_STAMP
    unsigned long long * smid = &stamp_t1_;
    unsigned long long * sx = stamp_x_;
#else
    unsigned long long * smid = nullptr;
    unsigned long long * sx = nullptr;
#endif
    if constexpr (WFIX >= 0) {
        mv_run<WFIX, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, g.stride, smem, red, g.late, smid, sx);
    } else {
        switch (Ent.W.type) {
            case W_F32: mv_run<W_F32, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, g.stride, smem, red, g.late, nullptr, nullptr); break;
            case W_F16: mv_run<W_F16, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, g.stride, smem, red, g.late, nullptr, nullptr); break;
            case W_Q4_0: mv_run<W_Q4_0, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, g.stride, smem, red, g.late, nullptr, nullptr); break;
            case W_Q4_1: mv_run<W_Q4_1, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, g.stride, smem, red, g.late, nullptr, nullptr); break;
            case W_Q5_0: mv_run<W_Q5_0, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, g.stride, smem, red, g.late, nullptr, nullptr); break;
            case W_Q5_1: mv_run<W_Q5_1, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, g.stride, smem, red, g.late, nullptr, nullptr); break;
            case W_Q8_0: mv_run<W_Q8_0, R, U, SRCK, FORM, EMIT, NW, LNP>(Ent, wgi, b0, g.stride, smem, red, g.late, nullptr, nullptr); break;
            default: break;
        }
    }
    (void)smid;
    (void)sx;
    STAMP_END(2);
}

// Activation-input matvec (SRC_ACT, no emission, one weight type): the lean form of mv_body's
// dot-wave path.  Every scalar the launch needs (weights, activation, epilogue) is read from
// the group before any arithmetic, so they arrive in one scalar-load round trip and the weight
// stream is issued right after it; no persistent walk, no prologue waves.  Same lane/unit
// assignment and accumulation order as mv_body (bit-identical results).
template <int WF, int R, int U>
__global__ __launch_bounds__(256) void k_mva(int b1, int b2, int b3, int b4, int b5, int b6, int b7, MVGroup g) {
    const int bx = (int)blockIdx.x;
    const int e = (bx >= b1) + (bx >= b2) + (bx >= b3) + (bx >= b4) + (bx >= b5) + (bx >= b6) + (bx >= b7);
    const int b0 = e == 0 ? 0 : e == 1 ? b1 : e == 2 ? b2 : e == 3 ? b3 : e == 4 ? b4 : e == 5 ? b5 : e == 6 ? b6 : b7;
    const MVHot h = g.hot[e];
    DMat W;
    W.type = WF;
    W.M = h.M;
    W.K = h.K;
    W.qs = h.qs;
    W.qh = h.qh;
    W.sc = h.sc;
    ActBuf a;
    a.K = h.K;
    a.q = (int8_t *)h.aq;
    a.d = (float *)h.ad;
    a.s = (float *)h.as;
    a.qsum = (int *)h.aqsum;
    a.h = (__half *)h.ahf;
    a.f = (float *)h.ahf;
    const float * const aux = (h.steps & 1) ? h.aux : g_mv_zero;
    const float * const bias = (h.steps & 2) ? h.bias : g_mv_zero;
    const int astep = h.steps & 1, bstep = (h.steps >> 1) & 1;

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int M = h.M, K = h.K;
    STAMP_BEGIN();
    const int row0 = (bx - b0) * (4 * R) + wave * R;
    int rows[R];
#pragma unroll
    for (int r = 0; r < R; r++) rows[r] = min(row0 + r, M - 1);
    // all U units of every row in flight before anything waits (clamped loads, no branches)
    WBlk w[R][U];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < R; r++) w[r][u] = load_unit<WF>(W, rows[r], u, lane);
    AUnit x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = load_act_unit<WF, false>(a, u, lane);
    // epilogue operands of row row0 + lane (lanes 0..R-1 run the rows' epilogues)
    const int erow = min(row0 + min(lane, R - 1), M - 1);
    EpiIn ep;
    ep.y = h.y[erow];
    ep.aux = aux[erow * astep];
    ep.bias = bias[erow * bstep];
    // keep the machine scheduler from interleaving later rows' loads with earlier rows' dots
    __builtin_amdgcn_sched_barrier(0);
    STAMP_MID();
    float acc[R], acc2[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const bool valid = unit_valid<WF>(K, u, lane);
#pragma unroll
        for (int r = 0; r < R; r++) {
            float t = acc[r], t2 = acc2[r];
            dot_unit<WF>(w[r][u], x[u], t, t2);
            acc[r] = valid ? t : acc[r];
            acc2[r] = valid ? t2 : acc2[r];
        }
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    float sr[R];
#pragma unroll
    for (int r = 0; r < R; r++) sr[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
    // epilogue on lane r for row r, on every lane (the operand loads stay ahead of the dots
    // instead of being sunk into the store branch: a dependent round trip at the kernel's end)
    const float v = epi_apply(h.epi, lane_row_sum<R>(sr, lane), ep);
    if (lane < R && row0 + lane < M) h.y[row0 + lane] = v;
    STAMP_END(1);
}

// Channel mix value + receptance in one launch (decode v4/v5/v6, rwkv_graph.inc:484-531):
// y[row] += sigmoid(Wr[row] . xr) * (Wv[row] . k).  Wave w of the workgroup owns rows row0..row0+R-1 of
// BOTH matrices (Wv units U over the FFN width, Wr units U2 over n_embed), so the receptance of
// a row never leaves the wave; each product is k_mva's arithmetic (lane/unit order, wave_sum63
// tree), and the epilogue is EPI_SIGMUL_ADD with aux = the receptance row (EPI_STORE) -- the same
// bits as the Wr matvec + k_mva pair it replaces.  hv: Wv / k / y, hr: Wr / xr.
template <int WF, int R, int U, int U2>
__global__ __launch_bounds__(256) void k_mvsig(MVHot hv, MVHot hr) {
    DMat W, W2;
    W.type = W2.type = WF;
    W.M = W2.M = hv.M;
    W.K = hv.K;
    W2.K = hr.K;
    W.qs = hv.qs, W.qh = hv.qh, W.sc = hv.sc;
    W2.qs = hr.qs, W2.qh = hr.qh, W2.sc = hr.sc;
    ActBuf a, a2;
    a.K = hv.K, a.q = (int8_t *)hv.aq, a.d = (float *)hv.ad, a.s = (float *)hv.as, a.qsum = (int *)hv.aqsum;
    a2.K = hr.K, a2.q = (int8_t *)hr.aq, a2.d = (float *)hr.ad, a2.s = (float *)hr.as, a2.qsum = (int *)hr.aqsum;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int M = hv.M;
    STAMP_BEGIN();
    const int row0 = (int)blockIdx.x * (4 * R) + wave * R;
    int rows[R];
#pragma unroll
    for (int r = 0; r < R; r++) rows[r] = min(row0 + r, M - 1);
    WBlk w[R][U], w2[R][U2];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < R; r++) w[r][u] = load_unit<WF>(W, rows[r], u, lane);
#pragma unroll
    for (int u = 0; u < U2; u++)
#pragma unroll
        for (int r = 0; r < R; r++) w2[r][u] = load_unit<WF>(W2, rows[r], u, lane);
    AUnit x[U], x2[U2];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = load_act_unit<WF, false>(a, u, lane);
#pragma unroll
    for (int u = 0; u < U2; u++) x2[u] = load_act_unit<WF, false>(a2, u, lane);
    const float yv = hv.y[min(row0 + min(lane, R - 1), M - 1)];
    __builtin_amdgcn_sched_barrier(0);
    STAMP_MID();
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    float sv[R], sr[R];
    {
        float acc[R], acc2[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
#pragma unroll
        for (int u = 0; u < U2; u++) {
            const bool valid = unit_valid<WF>(W2.K, u, lane);
#pragma unroll
            for (int r = 0; r < R; r++) {
                float t = acc[r], t2 = acc2[r];
                dot_unit<WF>(w2[r][u], x2[u], t, t2);
                acc[r] = valid ? t : acc[r];
                acc2[r] = valid ? t2 : acc2[r];
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) sr[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
    }
    {
        float acc[R], acc2[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool valid = unit_valid<WF>(W.K, u, lane);
#pragma unroll
            for (int r = 0; r < R; r++) {
                float t = acc[r], t2 = acc2[r];
                dot_unit<WF>(w[r][u], x[u], t, t2);
                acc[r] = valid ? t : acc[r];
                acc2[r] = valid ? t2 : acc2[r];
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) sv[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
    }
    const float rr = lane_row_sum<R>(sr, lane), vv = lane_row_sum<R>(sv, lane);
    const float v = yv + sigmoidf_(rr) * vv;  // EPI_SIGMUL_ADD, aux = the receptance row
    if (lane < R && row0 + lane < M) hv.y[row0 + lane] = v;
    STAMP_END(7);
}

// One weight-type translation unit (mv_*.hip) instantiates every launch shape for WFIX.
// LayerNorm prologues hold the normalized vector in registers: LNP = 32 (K <= 2048) or 64
// (K <= 4096) elements per lane.
template <int WFIX>
bool launch_mv_shape(hipStream_t st, MVGroup & g, int U, int srck, int form, bool emit, dim3 grid) {
    static_assert(MM_MAX_ENTRIES == 8, "k_mv takes b1..b7");
    int b[MM_MAX_ENTRIES];
    for (int i = 1; i < MM_MAX_ENTRIES; i++) b[i] = i < g.n ? g.e[i].block0 : INT_MAX;
#define MV_L(Rv, Uv, S, F, E, P)                                                                              \
    RK_LAUNCH((k_mv<Rv, Uv, S, F, E, WFIX, P>), grid, dim3((S) == MVK_ACT ? 256 : 512), g.lds_bytes, st, \
                       b[1], b[2], b[3], b[4], b[5], b[6], b[7], g)
    const int K = g.e[0].W.K;
    if constexpr (WFIX >= 0) {
        if (srck == MVK_ACT && !emit && g.units_max <= U && U <= 4) {  // k_mva: <= 4 units per lane
#define MVA_R(Rv, Uv) \
    RK_LAUNCH((k_mva<WFIX, Rv, Uv>), grid, dim3(256), 0, st, b[1], b[2], b[3], b[4], b[5], b[6], b[7], g)
#define MVA_L(Uv)                          \
    do {                                   \
        if (g.rows == 2) MVA_R(2, Uv);     \
        else if (g.rows == 8) MVA_R(8, Uv); \
        else MVA_R(4, Uv);                 \
    } while (0)
            if (U == 1) MVA_L(1);
            else if (U == 2) MVA_L(2);
            else MVA_L(4);
#undef MVA_L
#undef MVA_R
            return true;
        }
    }
    if (srck == MVK_ACT) {
        if (U == 1) MV_L(2, 1, MVK_ACT, 0, false, 0);
        else if (U == 2) MV_L(2, 2, MVK_ACT, 0, false, 0);
        else if (U == 4) MV_L(2, 4, MVK_ACT, 0, false, 0);
        else MV_L(2, 8, MVK_ACT, 0, false, 0);
        return true;
    }
    if (srck == MVK_F32) {
        if (U == 1) MV_L(1, 1, MVK_F32, 0, false, 0);
        else MV_L(1, 4, MVK_F32, 0, false, 0);
        return true;
    }
    for (int i = 1; i < g.n; i++)
        if (g.e[i].W.K != K) {
            fprintf(stderr, "rwkv: LayerNorm matvec group needs one K\n");
            return false;
        }
    if (K > 64 * 64) {
        fprintf(stderr, "rwkv: LayerNorm matvec prologue needs K <= 4096 (K=%d)\n", K);
        return false;
    }
    // prologue groups: the rows of a block over all 8 waves (image waves included), so R here is
    // half of launch_mv_group's rows per wave (g.rows, which counts the 4 streaming waves)
#define MV_PR(Rv, S, F, E)                                    \
    do {                                                      \
        if (K <= 2048) {                                      \
            if (U == 1) MV_L(Rv, 1, S, F, E, 32);             \
            else if (U == 2) MV_L(Rv, 2, S, F, E, 32);        \
            else MV_L(Rv, 4, S, F, E, 32);                    \
        } else {                                              \
            if (U == 1) MV_L(Rv, 1, S, F, E, 64);             \
            else if (U == 2) MV_L(Rv, 2, S, F, E, 64);        \
            else MV_L(Rv, 4, S, F, E, 64);                    \
        }                                                     \
    } while (0)
    // not emitting: g.rows rows per streaming wave (2, or 4 for large LayerNorm groups, or 8 with
    // one unit per round trip: <= 128 VGPRs, two workgroups per CU); emitting: 8
#define MV_P(S, F, E)                                         \
    do {                                                      \
        if constexpr (WFIX == W_F16) {                        \
            if (U == 8 && K > 2048 && g.rows == 2) {          \
                MV_L(1, 8, S, F, false, 64);                  \
                break;                                        \
            }                                                 \
        }                                                     \
        if (g.rows == 8 && K > 2048 && U == 2) MV_L(4, 1, S, F, false, 64); \
        else if (g.rows == 4) MV_PR(2, S, F, false);          \
        else MV_PR(1, S, F, false);                           \
    } while (0)
    if (emit) {
        if (form == 0) MV_PR(4, MVK_LN, 0, true);
        else MV_PR(4, MVK_LN, 1, true);
    } else {
        if (form == 0) MV_P(MVK_LN, 0, false);
        else if (form == 1) MV_P(MVK_LN, 1, false);
        else MV_P(MVK_LN, 2, false);
    }
#undef MV_P
#undef MV_PR
#undef MV_L
    return true;
}

}  // namespace rwkvmi
