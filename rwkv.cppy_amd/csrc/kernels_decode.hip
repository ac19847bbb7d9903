// kernels_decode.hip -- single-token (decode) kernels for gfx950.
//
// Decode is a chain of dependent matvecs over HBM-resident weights.  To keep the chain short,
// every matvec workgroup builds its own input in LDS from fp32 vectors that sit in L2 (the
// previous kernel's output): LayerNorm statistics, token-shift mix and the ggml Q8
// activation quantization are recomputed per workgroup (a few KB of L2 reads) instead of
// costing a separate launch.  Per-head attention work (decay LoRA tail, wkv, GroupNorm) is
// one kernel with the head's state in registers.
#include "device_common.hpp"
#include "kernels.hpp"

#include <stdio.h>

namespace rwkvmi {

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

static int lds_bytes_for(int fmt, int K) {
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

template <int WF>
__device__ __forceinline__ WBlk load_unit(const DMat & W, int row, int u, int lane) {
    const int K = W.K;
    if constexpr (WF == W_F32) {
        WBlk w;
        const int k = min(lane * 4 + u * 256, K - 4);
        w.q0 = *(const int4 *)((const float *)W.qs + (size_t)row * K + k);
        return w;
    } else if constexpr (WF == W_F16) {
        WBlk w;
        const int k = min(lane * 8 + u * 512, K - 8);
        w.q0 = *(const int4 *)((const __half *)W.qs + (size_t)row * K + k);
        return w;
    } else {
        const int nb = K >> 5;
        const int b = min(lane + u * 64, nb - 1);
        return load_wblk<WF>(W, (size_t)row * nb + b);
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
        float s = acc;
        s = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, w.q0.x), __builtin_bit_cast(half2_t, x.lo.x), s, false);
        s = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, w.q0.y), __builtin_bit_cast(half2_t, x.lo.y), s, false);
        s = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, w.q0.z), __builtin_bit_cast(half2_t, x.lo.z), s, false);
        s = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, w.q0.w), __builtin_bit_cast(half2_t, x.lo.w), s, false);
        acc = s;
    } else {
        float dw, mw;
        const int sumi = dot_wblk<WF>(w, x.lo, x.hi, x.qs, dw, mw);
        acc = fmaf(dw * x.d, (float)sumi, acc);
        if constexpr (WF == W_Q4_1 || WF == W_Q5_1) acc2 += mw * x.s;
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
// Q8 quantization with quad DPP reductions (F16: packed halves, F32: as is).
template <int WF>
__device__ __forceinline__ void prologue_chunks(const MVEntry & E, const ActBuf & a, float mean, float scale,
                                                bool write_carry, int wave, int nw, int lane) {
    const int K = E.W.K;
    for (int c = wave; c * 512 < K; c += nw) {
        const int k0 = c * 512 + lane * 8;
        const bool valid = k0 < K;  // quad-uniform (K % 32 == 0)
        const int kc = min(k0, K - 8);
        float v[8];
        if (E.src == SRC_F32) {
            const float4 t0 = *(const float4 *)(E.f + kc), t1 = *(const float4 *)(E.f + kc + 4);
            v[0] = t0.x, v[1] = t0.y, v[2] = t0.z, v[3] = t0.w, v[4] = t1.x, v[5] = t1.y, v[6] = t1.z, v[7] = t1.w;
        } else {
            float xs[8], ws[8], bs[8], cs[8], ms[8];
#pragma unroll
            for (int h = 0; h < 8; h += 4) {
                const float4 px = *(const float4 *)(E.x + kc + h);
                const float4 pw = *(const float4 *)(E.lnw + kc + h);
                const float4 pb = *(const float4 *)(E.lnb + kc + h);
                xs[h] = px.x, xs[h + 1] = px.y, xs[h + 2] = px.z, xs[h + 3] = px.w;
                ws[h] = pw.x, ws[h + 1] = pw.y, ws[h + 2] = pw.z, ws[h + 3] = pw.w;
                bs[h] = pb.x, bs[h + 1] = pb.y, bs[h + 2] = pb.z, bs[h + 3] = pb.w;
                if (E.form != 2) {
                    const float4 pc = *(const float4 *)(E.carry + kc + h);
                    const float4 pm = *(const float4 *)(E.mu + kc + h);
                    cs[h] = pc.x, cs[h + 1] = pc.y, cs[h + 2] = pc.z, cs[h + 3] = pc.w;
                    ms[h] = pm.x, ms[h + 1] = pm.y, ms[h + 2] = pm.z, ms[h + 3] = pm.w;
                }
            }
            float xa[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                xa[j] = ln_apply(xs[j], mean, scale, ws[j], bs[j]);
                if (E.form == 2) v[j] = xa[j];
                else if (E.form == 0) v[j] = xa[j] * ms[j] + (cs[j] - cs[j] * ms[j]);
                else v[j] = (cs[j] - xa[j]) * ms[j] + xa[j];
            }
            if (write_carry && valid) {
                *(float4 *)(E.carry_out + k0) = make_float4(xa[0], xa[1], xa[2], xa[3]);
                *(float4 *)(E.carry_out + k0 + 4) = make_float4(xa[4], xa[5], xa[6], xa[7]);
            }
        }
        if constexpr (WF == W_F32) {
            if (valid) {
                *(float4 *)(a.f + k0) = make_float4(v[0], v[1], v[2], v[3]);
                *(float4 *)(a.f + k0 + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
        } else if constexpr (WF == W_F16) {
            int p[4];
#pragma unroll
            for (int j = 0; j < 4; j++)
                p[j] = __builtin_bit_cast(int, __halves2half2(__float2half(v[2 * j]), __float2half(v[2 * j + 1])));
            if (valid) *(int4 *)(a.h + k0) = make_int4(p[0], p[1], p[2], p[3]);
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
        }
    }
}

// Epilogue operands of one output row, loaded at kernel start (not after the dots).
struct EpiIn {
    float y, aux, bias;
};
__device__ __forceinline__ EpiIn epi_load(const MVEntry & E, int row) {
    EpiIn p;
    const bool yin = E.epi == EPI_ADD || E.epi == EPI_SIGMUL_ADD || E.epi == EPI_VMIX7;
    const bool ain = E.epi == EPI_SIGMUL_ADD || E.epi == EPI_VMIX7;
    const bool bin = E.epi == EPI_DECAY6 || E.epi == EPI_DECAY7 || E.epi == EPI_SIGMOID_BIAS || E.epi == EPI_VMIX7;
    p.y = yin ? E.y[row] : 0.0f;
    p.aux = ain ? E.aux[row] : 0.0f;
    p.bias = bin ? E.bias[row] : 0.0f;
    return p;
}
__device__ __forceinline__ float epi_apply(int epi, float acc, const EpiIn & p) {
    switch (epi) {
        case EPI_SIGMOID: return sigmoidf_(acc);
        case EPI_TANH: return tanhf(acc);
        case EPI_SILU: return siluf_(acc);
        case EPI_RELU_SQ: {
            const float r = acc > 0.0f ? acc : 0.0f;
            return r * r;
        }
        case EPI_ADD: return p.y + acc;
        case EPI_SIGMUL_ADD: return p.y + sigmoidf_(p.aux) * acc;
        case EPI_DECAY6: return expf(-expf(acc + p.bias));
        case EPI_DECAY7: return expf(sigmoidf_(acc + p.bias) * -0.606531f);
        case EPI_SIGMOID_BIAS: return sigmoidf_(acc + p.bias);
        case EPI_VMIX7: return p.y + (p.aux - p.y) * sigmoidf_(acc + p.bias);
        default: return acc;
    }
}

// One workgroup = NW waves x R rows (RW = NW*R rows per row block).  E == 0: the input is an
// activation buffer in global memory (SRC_ACT, NW = 4); E > 0: the prologue builds it in LDS
// (SRC_F32 / SRC_LNMIX, K <= 64*NW*E; NW = 16 so the per-wave prologue work is short).
// stride > 0: the workgroup walks row blocks wgi, wgi+stride, ... with one prologue.
template <int WF, int R, int U, bool PRO, bool EMIT, int NW>
__device__ __forceinline__ void mv_body(const MVEntry & Ent, int wgi, int stride, char * smem, float * red) {
    constexpr int RW = NW * R;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const DMat & W = Ent.W;
    const int M = W.M, K = W.K;
    const int nblk = (M + RW - 1) / RW;
    const int units = mv_units(WF, K);
    PROBE(0);

    // (1) this wave's weight units (HBM) and the epilogue operands, in flight during the
    // prologue
    int row0 = wgi * RW + wave * R;
    int rows[R];
#pragma unroll
    for (int r = 0; r < R; r++) rows[r] = min(row0 + r, M - 1);
    WBlk w[R][U];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < R; r++) w[r][u] = load_unit<WF>(W, rows[r], u, lane);
    EpiIn ep[R];
    if constexpr (!EMIT) {
#pragma unroll
        for (int r = 0; r < R; r++) ep[r] = epi_load(Ent, rows[r]);
    } else {
        ep[0] = epi_load(Ent, min(wgi * RW + (tid < RW ? tid : 0), M - 1));
    }
    // (2) prologue: LayerNorm statistics (every wave for itself), then the activation image
    ActBuf a;
    if constexpr (PRO) {
        a = lds_act(smem, act_fmt_for(WF), K);
        float mean = 0.0f, scale = 0.0f;
        if (Ent.src == SRC_LNMIX) ln_stats_any(Ent.x, K, 1e-5f, mean, scale);
#ifdef MV_PROBE
        if (mean == 1.2345f) g_probe[1] = 0;
#endif
        PROBE(4);
        const bool write_carry = Ent.carry_out && wgi == (int)blockIdx.x - Ent.block0;
        prologue_chunks<WF>(Ent, a, mean, scale, write_carry, wave, NW, lane);
        PROBE(6);
        __syncthreads();
    } else {
        a = Ent.act;
    }
    PROBE(1);

    for (;;) {
        // (4) dots
        float acc[R], acc2[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
        for (int u0 = 0; u0 < units; u0 += U) {
            if (u0 > 0) {
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int r = 0; r < R; r++) w[r][u] = load_unit<WF>(W, rows[r], u0 + u, lane);
            }
            AUnit x[U];
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = load_act_unit<WF, PRO>(a, u0 + u, lane);
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (unit_valid<WF>(K, u0 + u, lane)) {
#pragma unroll
                    for (int r = 0; r < R; r++) dot_unit<WF>(w[r][u], x[u], acc[r], acc2[r]);
                }
            }
        }

        // (5) reduce + epilogue
        constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
        float s[R];
#pragma unroll
        for (int r = 0; r < R; r++) s[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
        if constexpr (!EMIT) {
#ifdef MV_PROBE
            if (s[0] == 1.2345f) g_probe[0] = 0;  // orders the stamp after the dots
#endif
            PROBE(2);
#pragma unroll
            for (int r = 0; r < R; r++) {
                const int row = row0 + r;
                if (lane == 63 && row < M) Ent.y[row] = epi_apply(Ent.epi, s[r], ep[r]);
            }
        } else {
            // RW rows per block (a multiple of 32): apply the epilogue and emit each 32 rows as
            // one quantization block of the next matmul's input (ggml Q8 / fp16 / fp32)
#pragma unroll
            for (int r = 0; r < R; r++)
                if (lane == 63) red[wave * R + r] = s[r];
            __syncthreads();
            PROBE(2);
            if (tid < RW) {
                const int row = wgi * RW + tid;
                float vv = 0.0f;
                if (row < M) {
                    vv = epi_apply(Ent.epi, red[tid], ep[0]);
                    if (Ent.y) Ent.y[row] = vv;
                }
                if (Ent.act_out.fmt >= 0 && Ent.emit) emit32(Ent.act_out, 0, row, vv);
            }
        }
        PROBE(3);
        wgi += stride;
        if (stride <= 0 || wgi >= nblk) break;
        if constexpr (EMIT) __syncthreads();  // red[] reuse
        row0 = wgi * RW + wave * R;
#pragma unroll
        for (int r = 0; r < R; r++) rows[r] = min(row0 + r, M - 1);
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < R; r++) w[r][u] = load_unit<WF>(W, rows[r], u, lane);
        if constexpr (!EMIT) {
#pragma unroll
            for (int r = 0; r < R; r++) ep[r] = epi_load(Ent, rows[r]);
        } else {
            ep[0] = epi_load(Ent, min(wgi * RW + (tid < RW ? tid : 0), M - 1));
        }
    }
}

// WFIX >= 0: every entry of the group has weight type WFIX (one body, fewer registers);
// WFIX < 0: per-entry switch.
template <int R, int U, bool PRO, bool EMIT, int WFIX>
__global__ __launch_bounds__(256) void k_mv(MVGroup g) {
    constexpr int NW = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float red[NW * R];
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MVEntry & Ent = g.e[e];
    const int wgi = (int)blockIdx.x - Ent.block0;
    if constexpr (WFIX >= 0) {
        mv_body<WFIX, R, U, PRO, EMIT, NW>(Ent, wgi, g.stride, smem, red);
    } else {
        switch (Ent.W.type) {
            case W_F32: mv_body<W_F32, R, U, PRO, EMIT, NW>(Ent, wgi, g.stride, smem, red); break;
            case W_F16: mv_body<W_F16, R, U, PRO, EMIT, NW>(Ent, wgi, g.stride, smem, red); break;
            case W_Q4_0: mv_body<W_Q4_0, R, U, PRO, EMIT, NW>(Ent, wgi, g.stride, smem, red); break;
            case W_Q4_1: mv_body<W_Q4_1, R, U, PRO, EMIT, NW>(Ent, wgi, g.stride, smem, red); break;
            case W_Q5_0: mv_body<W_Q5_0, R, U, PRO, EMIT, NW>(Ent, wgi, g.stride, smem, red); break;
            case W_Q5_1: mv_body<W_Q5_1, R, U, PRO, EMIT, NW>(Ent, wgi, g.stride, smem, red); break;
            case W_Q8_0: mv_body<W_Q8_0, R, U, PRO, EMIT, NW>(Ent, wgi, g.stride, smem, red); break;
            default: break;
        }
    }
}

static int g_mv_cus = 256;
void set_mv_device_cus(int n) { g_mv_cus = n > 0 ? n : 256; }

template <int U, int WFIX>
static void launch_mv_w(hipStream_t st, MVGroup & g, bool pro, bool emit, dim3 grid) {
    if (emit) hipLaunchKernelGGL((k_mv<8, U, true, true, WFIX>), grid, dim3(256), g.lds_bytes, st, g);
    else if (pro) hipLaunchKernelGGL((k_mv<2, U, true, false, WFIX>), grid, dim3(256), g.lds_bytes, st, g);
    else hipLaunchKernelGGL((k_mv<2, U, false, false, WFIX>), grid, dim3(256), 0, st, g);
}

template <int U>
static void launch_mv_u(hipStream_t st, MVGroup & g, bool pro, bool emit, int wfix, dim3 grid) {
    switch (wfix) {
        case W_F16: launch_mv_w<U, W_F16>(st, g, pro, emit, grid); break;
        case W_Q4_0: launch_mv_w<U, W_Q4_0>(st, g, pro, emit, grid); break;
        case W_Q4_1: launch_mv_w<U, W_Q4_1>(st, g, pro, emit, grid); break;
        case W_Q5_0: launch_mv_w<U, W_Q5_0>(st, g, pro, emit, grid); break;
        case W_Q5_1: launch_mv_w<U, W_Q5_1>(st, g, pro, emit, grid); break;
        case W_Q8_0: launch_mv_w<U, W_Q8_0>(st, g, pro, emit, grid); break;
        default: launch_mv_w<U, -1>(st, g, pro, emit, grid); break;
    }
}

bool launch_mv_group(hipStream_t st, MVGroup & g) {
    bool emit = false, prologue = false, plain = false;
    for (int i = 0; i < g.n; i++) {
        emit |= g.e[i].emit != 0;
        (g.e[i].src == SRC_ACT ? plain : prologue) = true;
    }
    if (prologue && plain) {
        fprintf(stderr, "rwkv: matvec group mixes activation and prologue sources\n");
        return false;
    }
    if (emit && !prologue) {
        fprintf(stderr, "rwkv: emitting matvec needs a prologue source\n");
        return false;
    }
    const int R = emit ? 8 : 2, RW = 4 * R;
    int blocks = 0, umax = 1, lds = 0;
    for (int i = 0; i < g.n; i++) {
        MVEntry & e = g.e[i];
        if (e.W.K % 32) {
            fprintf(stderr, "rwkv: matvec needs K %% 32 == 0 (K=%d)\n", e.W.K);
            return false;
        }
        if (e.src == SRC_LNMIX && (e.W.K % 64 || e.W.K > 64 * 128)) {
            fprintf(stderr, "rwkv: LayerNorm prologue needs K %% 64 == 0 and K <= 8192 (K=%d)\n", e.W.K);
            return false;
        }
        if (e.emit && e.W.M % 32) {
            fprintf(stderr, "rwkv: emitting matvec needs M %% 32 == 0 (M=%d)\n", e.W.M);
            return false;
        }
        if (e.src == SRC_ACT && (e.act.K != e.W.K || e.act.fmt != act_fmt_for(e.W.type))) {
            fprintf(stderr, "rwkv: matvec input format/size mismatch (K=%d vs %d)\n", e.act.K, e.W.K);
            return false;
        }
        e.block0 = blocks;
        blocks += (e.W.M + RW - 1) / RW;
        umax = std::max(umax, mv_units(e.W.type, e.W.K));
        if (e.src != SRC_ACT) lds = std::max(lds, lds_bytes_for(act_fmt_for(e.W.type), e.W.K));
    }
    g.lds_bytes = lds;
    if (!blocks) return true;
    // a single large prologue entry (the head): persistent walk over its row blocks, one
    // LayerNorm per workgroup
    g.stride = 0;
    int grid = blocks;
    if (prologue && g.n == 1 && !emit && blocks > 8 * g_mv_cus) {
        grid = 2 * g_mv_cus;
        g.stride = grid;
    }
    const int U = umax <= 1 ? 1 : umax <= 2 ? 2 : 4;
    int wfix = g.e[0].W.type;
    for (int i = 1; i < g.n; i++)
        if (g.e[i].W.type != wfix) wfix = -1;
    switch (U) {
        case 1: launch_mv_u<1>(st, g, prologue, emit, wfix, dim3(grid)); break;
        case 2: launch_mv_u<2>(st, g, prologue, emit, wfix, dim3(grid)); break;
        default: launch_mv_u<4>(st, g, prologue, emit, wfix, dim3(grid)); break;
    }
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v6 mix5 (decode)
struct Mix5Dec {
    int C, D;
    const float * xa, * carry, * lora, * w2t;
    const float * maa[5];
    ActBuf out[5];
};

// grid (C/256, 5): block (cx, n) computes mixed vector n for 256 channels from xa = LN(x),
// which the preceding W1 matvec already wrote as the new att_xx carry.  w2t [5][D][C] makes
// the per-channel D-long dots coalesced across lanes; accumulation order matches the oracle
// (sequential over i, fp64).
__global__ __launch_bounds__(256) void k_v6_mix5_dec(Mix5Dec a) {
    const int n = blockIdx.y, C = a.C, D = a.D;
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if ((int)(blockIdx.x * blockDim.x + (threadIdx.x & ~31)) >= C) return;  // half-wave uniform
    float w2v[64];
    const float * w2 = a.w2t + (size_t)n * D * C + c;
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const float t = w2[(size_t)min(i, D - 1) * C];
        w2v[i] = (i < D) ? t : 0.0f;
    }
    const float xa = a.xa[c], cc = a.carry[c], mu = a.maa[n][c];
    const float sx = cc - xa;
    const float * lv = a.lora + n * D;
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 64; i++)
        if (i < D) acc += (double)(w2v[i] * lv[i]);
    const float m = (float)acc;
    emit32(a.out[n], 0, c, (m + mu) * sx + xa);
}

bool launch_v6_mix5_dec(hipStream_t st, int C, int D, const float * xa, const float * carry, const float * lora,
                        const float * w2t, const float * const * maa, const ActBuf * outs) {
    Mix5Dec a;
    a.C = C;
    a.D = D;
    a.xa = xa;
    a.carry = carry;
    a.lora = lora;
    a.w2t = w2t;
    for (int n = 0; n < 5; n++) {
        a.maa[n] = maa[n];
        a.out[n] = outs[n];
    }
    if (D > 64 || C % 32) {
        fprintf(stderr, "rwkv: v6 maa LoRA width %d / n_embed %d unsupported\n", D, C);
        return false;
    }
    dim3 grid((C + 255) / 256, 5);
    hipLaunchKernelGGL(k_v6_mix5_dec, grid, dim3(256), 0, st, a);
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v5/v6 attention (decode)
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

// One row of the v6 decay LoRA tail by one thread (units <= 32, one per lane of k_mm);
// PF units were prefetched into wp[].
template <int WF, int PF>
__device__ __forceinline__ float decay_row_thread(const DMat & W, int row, const ActBuf & act, int nl,
                                                  const WBlk (&wp)[PF > 0 ? PF : 1]) {
    float p[32], p2[32];
#pragma unroll
    for (int l = 0; l < 32; l++) {
        p[l] = p2[l] = 0.0f;
        if (l < nl) {
            const WBlk w = (l < PF) ? wp[l < PF ? l : 0] : load_unit<WF>(W, row, 0, l);
            const AUnit x = load_act_unit<WF, true>(act, 0, l);
            dot_unit<WF>(w, x, p[l], p2[l]);
        }
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    return one ? tree_wave32(p) + tree_wave32(p2) : tree_wave32(p) + 0.0f;
}

// One row by one wave, exactly k_mm's loop (any K).
template <int WF>
__device__ __forceinline__ float decay_row_wave(const DMat & W, int row, const ActBuf & act, int lane) {
    float acc = 0.0f, acc2 = 0.0f;
    const int units = mv_units(WF, W.K);
    for (int u = 0; u < units; u++) {
        const WBlk w = load_unit<WF>(W, row, u, lane);
        const AUnit x = load_act_unit<WF, true>(act, u, lane);
        if (unit_valid<WF>(W.K, u, lane)) dot_unit<WF>(w, x, acc, acc2);
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    return one ? wave_sum63(acc) + wave_sum63(acc2) : wave_sum63(acc) + 0.0f;
}

// lanes of k_mm that hold a unit of a K-long row, when each holds at most one; else 0
__host__ __device__ inline int one_unit_lanes(int type, int K) {
    const int per = type == W_F32 ? 4 : type == W_F16 ? 8 : 32;
    const int n = K / per;
    return n <= 64 ? n : 0;
}

template <int WF>
__device__ __forceinline__ void decay_rows(const Att6Dec & a, const ActBuf & act, float * sw, int c0, int S) {
    const int tid = threadIdx.x;
    const int nl = one_unit_lanes(WF, a.wd2.K);
    if (nl > 0 && nl <= 32) {
        const WBlk none[1] = {};
        if (tid < S) {
            const float s = decay_row_thread<WF, 0>(a.wd2, c0 + tid, act, nl, none);
            sw[tid] = expf(-expf(s + a.decay[c0 + tid]));
        }
    } else {
        const int lane = tid & 63, nw = blockDim.x >> 6;
        for (int j = tid >> 6; j < S; j += nw) {
            const float s = decay_row_wave<WF>(a.wd2, c0 + j, act, lane);
            if (lane == 63) sw[j] = expf(-expf(s + a.decay[c0 + j]));
        }
    }
}

// One workgroup per head, S*G threads (G = min(256/S, S), as the sequence kernel k_wkv6):
// thread (j = tid % S, g = tid / S) owns state column j for keys i in [g*IPG, (g+1)*IPG) --
// each state load/store instruction covers S consecutive floats.  The per-thread partial y
// sums meet in LDS and are folded with group_sum's butterfly tree, so decode and sequence
// agree bit for bit.  PF > 0: quantized decay LoRA with <= PF units per row, prefetched.
template <int WF, int PF>
__global__ __launch_bounds__(256) void k_att6_dec(Att6Dec a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float sr[64], sk[64], sv[64], sw[64], su[64];
    __shared__ float part[16][64];
    const int h = blockIdx.x, S = a.S, G = min(256 / S, S), IPG = S / G;
    const int tid = threadIdx.x, j = tid % S, g = min(tid / S, G - 1), c0 = h * S;
    const bool active = tid < S * G;
    const size_t hb = (size_t)h * S * S;
    float st[16];
#pragma unroll
    for (int ii = 0; ii < 16; ii++)
        st[ii] = ii < IPG && active ? a.sin[hb + (size_t)(g * IPG + ii) * S + j] : 0.0f;
    WBlk wp[PF > 0 ? PF : 1];
    if constexpr (PF > 0) {
        const int nb = a.wd2.K >> 5;
        const int row = c0 + min(tid, S - 1);
#pragma unroll
        for (int l = 0; l < PF; l++) wp[l] = load_wblk<WF>(a.wd2, (size_t)row * nb + min(l, nb - 1));
    }
    if (tid < S) {
        sr[tid] = a.r[c0 + tid];
        sk[tid] = a.k[c0 + tid];
        sv[tid] = a.v[c0 + tid];
        su[tid] = a.u[c0 + tid];
        if (a.w) sw[tid] = a.w[c0 + tid];
    }
    ActBuf act;
    if (!a.w) {
        // v6 decay LoRA tail: w = exp(-exp(Wd2 . dl + decay)), rwkv_graph.inc:357-367
        const int D = a.wd2.K;
        act = lds_act(smem, act_fmt_for(a.wd2.type), D);
        for (int k0 = 0; k0 < D; k0 += blockDim.x) {
            if (k0 + (tid & ~31) >= D) continue;
            emit32(act, 0, k0 + tid, a.dl[k0 + tid]);
        }
    }
    __syncthreads();
    if (!a.w) {
        if constexpr (PF > 0) {
            if (tid < S) {
                const float s = decay_row_thread<WF, PF>(a.wd2, c0 + tid, act, a.wd2.K >> 5, wp);
                sw[tid] = expf(-expf(s + a.decay[c0 + tid]));
            }
        } else {
            switch (a.wd2.type) {
                case W_F32: decay_rows<W_F32>(a, act, sw, c0, S); break;
                case W_F16: decay_rows<W_F16>(a, act, sw, c0, S); break;
                case W_Q4_0: decay_rows<W_Q4_0>(a, act, sw, c0, S); break;
                case W_Q4_1: decay_rows<W_Q4_1>(a, act, sw, c0, S); break;
                case W_Q5_0: decay_rows<W_Q5_0>(a, act, sw, c0, S); break;
                case W_Q5_1: decay_rows<W_Q5_1>(a, act, sw, c0, S); break;
                case W_Q8_0: decay_rows<W_Q8_0>(a, act, sw, c0, S); break;
                default: break;
            }
        }
        __syncthreads();
    }
    // wkv6 for one token (ggml_rwkv_wkv6 semantics, same arithmetic as k_wkv6)
    if (active) {
        const float vj = sv[j];
        float acc = 0.0f;
#pragma unroll
        for (int ii = 0; ii < 16; ii++) {
            if (ii < IPG) {
                const int i = g * IPG + ii;
                const float prev = st[ii];
                const float kv = vj * sk[i];
                const float temp = kv * su[i] + prev;
                acc += temp * sr[i];
                a.sout[hb + (size_t)i * S + j] = prev * sw[i] + kv;
            }
        }
        part[g][j] = acc;
    }
    __syncthreads();
    // GroupNorm over the head (ggml_norm, fp64 sums) * ln_x (+ b) (* g)
    if (tid < S) {
        float p[16];
#pragma unroll
        for (int q = 0; q < 16; q++) p[q] = q < G ? part[q][tid] : 0.0f;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1)
            if (o < G)
#pragma unroll
                for (int q = 0; q < o; q++) p[q] = p[q] + p[q + o];
        const float x = p[0];
        const double s = group_sum((double)x, S);
        const float mean = (float)(s / (double)S);
        const float d = x - mean;
        const double s2 = group_sum((double)(d * d), S);
        const float var = (float)(s2 / (double)S);
        const float scale = 1.0f / sqrtf(var + a.eps);
        float o = d * scale;
        o = o * a.lnx_w[c0 + tid];
        o = o + a.lnx_b[c0 + tid];
        if (a.g) o = o * a.g[c0 + tid];
        if (a.yq.fmt >= 0) emit32(a.yq, 0, c0 + tid, o);  // S >= 32: whole half-wave blocks
        else a.y[c0 + tid] = o;
    }
}

bool launch_att6_dec(hipStream_t st, const Att6Dec & a) {
    if (a.S > 64 || (a.S & (a.S - 1))) {
        fprintf(stderr, "rwkv: head size %d unsupported\n", a.S);
        return false;
    }
    int G = 256 / a.S;
    if (G > a.S) G = a.S;
    const int threads = a.S * G;
    int lds = 0;
    if (!a.w) {
        const int D = a.wd2.K;
        if (D % 32) {
            fprintf(stderr, "rwkv: v6 decay LoRA width %d unsupported\n", D);
            return false;
        }
        lds = lds_bytes_for(act_fmt_for(a.wd2.type), D);
    }
    if (a.yq.fmt >= 0 && a.S < 32) {
        fprintf(stderr, "rwkv: quantized attention output needs head size >= 32\n");
        return false;
    }
    dim3 grid(a.H), block(std::max(threads, 64));
    const bool pf = !a.w && a.wd2.type >= W_Q4_0 && (a.wd2.K >> 5) <= 4;
    if (!pf) {
        hipLaunchKernelGGL((k_att6_dec<-1, 0>), grid, block, lds, st, a);
    } else {
        switch (a.wd2.type) {
            case W_Q4_0: hipLaunchKernelGGL((k_att6_dec<W_Q4_0, 4>), grid, block, lds, st, a); break;
            case W_Q4_1: hipLaunchKernelGGL((k_att6_dec<W_Q4_1, 4>), grid, block, lds, st, a); break;
            case W_Q5_0: hipLaunchKernelGGL((k_att6_dec<W_Q5_0, 4>), grid, block, lds, st, a); break;
            case W_Q5_1: hipLaunchKernelGGL((k_att6_dec<W_Q5_1, 4>), grid, block, lds, st, a); break;
            default: hipLaunchKernelGGL((k_att6_dec<W_Q8_0, 4>), grid, block, lds, st, a); break;
        }
    }
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v7 attention (decode)
template <int JPG>
__global__ __launch_bounds__(256) void k_att7_dec(Att7Dec a) {
    __shared__ float sr[64], sw[64], sk[64], sv[64], snb[64], sbb[64], sy[64];
    __shared__ float sbonus;
    const int h = blockIdx.x, S = a.S, G = S / JPG;
    const int tid = threadIdx.x, c0 = h * S;
    if (tid < S) {
        // prep (rwkv_graph.inc:432-437 + rwkv_operators.inc:40-82)
        const int c = c0 + tid;
        const float kv = a.k[c];
        const float kkr = kv * a.k_k[c];
        const float sum = group_sum(kkr * kkr, S);
        const float scale = 1.0f / fmaxf(sqrtf(sum), 1e-12f);
        const float kk = kkr * scale;
        const float av = a.a[c];
        const float ka = kv * a.k_a[c];
        const float kadj = kv + (av * ka - ka);
        const float rv = a.r[c];
        sr[tid] = rv;
        sw[tid] = a.w[c];
        sk[tid] = kadj;
        sv[tid] = a.v[c];
        snb[tid] = -kk;
        sbb[tid] = kk * av;
        const float bs = group_sum((kadj * rv) * a.r_k[c], S);
        if (tid == 0) sbonus = bs;
    }
    __syncthreads();
    if (tid < S * G) {
        // wkv7 (rwkv_operators_wkv_v7.inc:37-107): state [h][i(value)][j(key)], g splits j
        const int i = tid / G, g = tid % G;
        const size_t base = (size_t)h * S * S + (size_t)i * S + g * JPG;
        float st[JPG];
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) st[jj] = a.sin[base + jj];
        float sa = 0.0f;
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) sa += snb[g * JPG + jj] * st[jj];
        sa = group_sum(sa, G);
        const float vi = sv[i];
        float acc = 0.0f;
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) {
            const int j = g * JPG + jj;
            const float kv = vi * sk[j];
            const float ns = st[jj] * sw[j] + kv + sa * sbb[j];
            a.sout[base + jj] = ns;
            acc += ns * sr[j];
        }
        acc = group_sum(acc, G);
        if (g == 0) sy[i] = acc;
    }
    __syncthreads();
    if (tid < S) {
        const int c = c0 + tid;
        const float x = sy[tid];
        const double s = group_sum((double)x, S);
        const float mean = (float)(s / (double)S);
        const float d = x - mean;
        const double s2 = group_sum((double)(d * d), S);
        const float var = (float)(s2 / (double)S);
        const float scale = 1.0f / sqrtf(var + 64e-5f);
        float o = d * scale;
        o = o * a.lnx_w[c];
        o = o + a.lnx_b[c];
        o = o + sv[tid] * sbonus;
        o = o * a.g[c];
        if (a.yq.fmt >= 0) emit32(a.yq, 0, c, o);  // S >= 32: whole half-wave blocks
        else a.y[c] = o;
    }
}

bool launch_att7_dec(hipStream_t st, const Att7Dec & a) {
    if (a.S > 64 || (a.S & (a.S - 1))) {
        fprintf(stderr, "rwkv: head size %d unsupported\n", a.S);
        return false;
    }
    int G = 256 / a.S;
    if (G > a.S) G = a.S;
    const int JPG = a.S / G;
    const int threads = std::max(64, a.S * G);
    if (a.yq.fmt >= 0 && a.S < 32) {
        fprintf(stderr, "rwkv: quantized attention output needs head size >= 32\n");
        return false;
    }
    dim3 grid(a.H), block(threads);
    switch (JPG) {
        case 1: hipLaunchKernelGGL(k_att7_dec<1>, grid, block, 0, st, a); break;
        case 2: hipLaunchKernelGGL(k_att7_dec<2>, grid, block, 0, st, a); break;
        case 4: hipLaunchKernelGGL(k_att7_dec<4>, grid, block, 0, st, a); break;
        case 8: hipLaunchKernelGGL(k_att7_dec<8>, grid, block, 0, st, a); break;
        case 16: hipLaunchKernelGGL(k_att7_dec<16>, grid, block, 0, st, a); break;
        default: return false;
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
