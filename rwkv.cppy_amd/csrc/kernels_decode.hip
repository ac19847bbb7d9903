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

__device__ __forceinline__ float apply_epi_mv(const MVEntry & E, int row, float acc) {
    switch (E.epi) {
        case EPI_SIGMOID: return sigmoidf_(acc);
        case EPI_TANH: return tanhf(acc);
        case EPI_SILU: return siluf_(acc);
        case EPI_RELU_SQ: {
            const float r = acc > 0.0f ? acc : 0.0f;
            return r * r;
        }
        case EPI_ADD: return E.y[row] + acc;
        case EPI_SIGMUL_ADD: return E.y[row] + sigmoidf_(E.aux[row]) * acc;
        case EPI_DECAY6: return expf(-expf(acc + E.bias[row]));
        case EPI_DECAY7: return expf(sigmoidf_(acc + E.bias[row]) * -0.606531f);
        case EPI_SIGMOID_BIAS: return sigmoidf_(acc + E.bias[row]);
        case EPI_VMIX7: {
            const float v = E.y[row];
            return v + (E.aux[row] - v) * sigmoidf_(acc + E.bias[row]);
        }
        default: return acc;
    }
}

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

// One row-block of a matvec for a lane: the weight blocks of all R rows (and the activation
// block) are loaded unconditionally first -- rows past M are clamped to M-1 and discarded --
// so R 16-byte HBM loads are in flight together; then the int8 dots.  LDS=true reads the
// activation through a __shared__ pointer (ds_read), LDS=false from global memory.
template <int WF, int R, bool LDS>
__device__ __forceinline__ void mv_accumulate(const DMat & W, const ActBuf & a, int row0, int lane, float (&acc)[R],
                                              float (&acc2)[R]) {
    const int K = W.K, M = W.M;
    int rows[R];
#pragma unroll
    for (int r = 0; r < R; r++) rows[r] = min(row0 + r, M - 1);
    if constexpr (WF == W_F32) {
        for (int k = lane * 4; k < K; k += 256) {
            float4 w[R];
#pragma unroll
            for (int r = 0; r < R; r++) w[r] = *(const float4 *)((const float *)W.qs + (size_t)rows[r] * K + k);
            const float4 x = *(const float4 *)(a.f + k);
#pragma unroll
            for (int r = 0; r < R; r++) {
                float s = acc[r];
                s = fmaf(w[r].x, x.x, s);
                s = fmaf(w[r].y, x.y, s);
                s = fmaf(w[r].z, x.z, s);
                s = fmaf(w[r].w, x.w, s);
                acc[r] = s;
            }
        }
    } else if constexpr (WF == W_F16) {
        for (int k = lane * 8; k < K; k += 512) {
            int4 w[R];
#pragma unroll
            for (int r = 0; r < R; r++) w[r] = *(const int4 *)((const __half *)W.qs + (size_t)rows[r] * K + k);
            const int4 x = *(const int4 *)(a.h + k);
#pragma unroll
            for (int r = 0; r < R; r++) {
                float s = acc[r];
                s = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, w[r].x), __builtin_bit_cast(half2_t, x.x), s, false);
                s = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, w[r].y), __builtin_bit_cast(half2_t, x.y), s, false);
                s = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, w[r].z), __builtin_bit_cast(half2_t, x.z), s, false);
                s = __builtin_amdgcn_fdot2(__builtin_bit_cast(half2_t, w[r].w), __builtin_bit_cast(half2_t, x.w), s, false);
                acc[r] = s;
            }
        }
    } else {
        const int nb = K >> 5;
        for (int b = lane; b < nb; b += 64) {
            WBlk w[R];
#pragma unroll
            for (int r = 0; r < R; r++) w[r] = load_wblk<WF>(W, (size_t)rows[r] * nb + b);
            int4 alo, ahi;
            float dx, sx;
            int qs;
            if constexpr (LDS) {
                typedef int i32x4 __attribute__((ext_vector_type(4)));
                typedef __attribute__((address_space(3))) const i32x4 lds_i32x4;
                typedef __attribute__((address_space(3))) const float lds_float;
                typedef __attribute__((address_space(3))) const int lds_int;
                const lds_i32x4 * ap = (const lds_i32x4 *)(uintptr_t)(a.q + (size_t)b * 32);
                const i32x4 t0 = ap[0], t1 = ap[1];
                alo = make_int4(t0.x, t0.y, t0.z, t0.w);
                ahi = make_int4(t1.x, t1.y, t1.z, t1.w);
                dx = *(const lds_float *)(uintptr_t)(a.d + b);
                qs = *(const lds_int *)(uintptr_t)(a.qsum + b);
                sx = (WF == W_Q4_1 || WF == W_Q5_1) ? *(const lds_float *)(uintptr_t)(a.s + b) : 0.0f;
            } else {
                const int4 * ap = (const int4 *)(a.q + (size_t)b * 32);
                alo = ap[0];
                ahi = ap[1];
                dx = a.d[b];
                qs = a.qsum[b];
                sx = (WF == W_Q4_1 || WF == W_Q5_1) ? a.s[b] : 0.0f;
            }
#pragma unroll
            for (int r = 0; r < R; r++) {
                float dw, mw;
                const int sumi = dot_wblk<WF>(w[r], alo, ahi, qs, dw, mw);
                acc[r] = fmaf(dw * dx, (float)sumi, acc[r]);
                if constexpr (WF == W_Q4_1 || WF == W_Q5_1) acc2[r] += mw * sx;
            }
        }
    }
}

template <int R, bool LDS>
__device__ __forceinline__ void mv_dispatch(const DMat & W, const ActBuf & a, int row0, int lane, float (&acc)[R],
                                            float (&acc2)[R]) {
    switch (W.type) {
        case W_F32: mv_accumulate<W_F32, R, LDS>(W, a, row0, lane, acc, acc2); break;
        case W_F16: mv_accumulate<W_F16, R, LDS>(W, a, row0, lane, acc, acc2); break;
        case W_Q4_0: mv_accumulate<W_Q4_0, R, LDS>(W, a, row0, lane, acc, acc2); break;
        case W_Q4_1: mv_accumulate<W_Q4_1, R, LDS>(W, a, row0, lane, acc, acc2); break;
        case W_Q5_0: mv_accumulate<W_Q5_0, R, LDS>(W, a, row0, lane, acc, acc2); break;
        case W_Q5_1: mv_accumulate<W_Q5_1, R, LDS>(W, a, row0, lane, acc, acc2); break;
        case W_Q8_0: mv_accumulate<W_Q8_0, R, LDS>(W, a, row0, lane, acc, acc2); break;
        default: break;
    }
}

// Per-thread register image of a K-vector: thread t owns k = i*256 + t (i < E).  All loads of
// a phase are issued before any is used (one dependent L2 round trip per phase).
template <int E>
__device__ __forceinline__ void load_vec(float (&v)[E], const float * p, int K) {
#pragma unroll
    for (int i = 0; i < E; i++) {
        const int k = i * 256 + (int)threadIdx.x;
        v[i] = (k < K) ? p[k] : 0.0f;
    }
}

// LayerNorm statistics of the register image (ggml_norm: fp64 sums, two passes).
template <int E>
__device__ __forceinline__ void ln_stats_reg(const float (&xv)[E], int K, float & mean, float & scale, double * sh) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < E; i++)
        if (i * 256 + (int)threadIdx.x < K) s += (double)xv[i];
    s = block_sum_d(s, sh);
    mean = (float)(s / (double)K);
    double s2 = 0.0;
#pragma unroll
    for (int i = 0; i < E; i++)
        if (i * 256 + (int)threadIdx.x < K) {
            const float d = xv[i] - mean;
            s2 += (double)(d * d);
        }
    s2 = block_sum_d(s2, sh);
    scale = 1.0f / sqrtf((float)(s2 / (double)K) + 1e-5f);
}

template <int R, int E, bool EMIT>
__global__ __launch_bounds__(256) void k_mv(MVGroup g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ double sh[8];
    __shared__ float red[4 * R];
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MVEntry & Ent = g.e[e];
    const int K = Ent.W.K, fmt = act_fmt_for(Ent.W.type);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    ActBuf a;
    if (Ent.src == SRC_ACT) {
        a = Ent.act;
    } else {
        a = lds_act(smem, fmt, K);
        float v[E];
        if (Ent.src == SRC_F32) {
            load_vec<E>(v, Ent.f, K);
        } else {
            float xv[E], lw[E], lb[E];
            load_vec<E>(xv, Ent.x, K);
            load_vec<E>(lw, Ent.lnw, K);
            load_vec<E>(lb, Ent.lnb, K);
            float cv[E], mv[E];
            if (Ent.form != 2) {
                load_vec<E>(cv, Ent.carry, K);
                load_vec<E>(mv, Ent.mu, K);
            }
            float mean, scale;
            ln_stats_reg<E>(xv, K, mean, scale, sh);
            const bool write_carry = Ent.carry_out && (int)blockIdx.x == Ent.block0;
#pragma unroll
            for (int i = 0; i < E; i++) {
                const float xa = ln_apply(xv[i], mean, scale, lw[i], lb[i]);
                const int k = i * 256 + tid;
                if (write_carry && k < K) Ent.carry_out[k] = xa;
                if (Ent.form == 2) v[i] = xa;
                else if (Ent.form == 0) v[i] = xa * mv[i] + (cv[i] - cv[i] * mv[i]);
                else v[i] = (cv[i] - xa) * mv[i] + xa;
            }
        }
#pragma unroll
        for (int i = 0; i < E; i++) {
            const int k0 = i * 256;
            if (k0 + (tid & ~31) < K) emit32(a, 0, k0 + tid, v[i]);  // half-wave uniform
        }
        __syncthreads();
    }
    const int rowwg = ((int)blockIdx.x - Ent.block0) * 4 * R;
    const int row0 = rowwg + wave * R;
    float acc[R], acc2[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
    if (Ent.src == SRC_ACT) mv_dispatch<R, false>(Ent.W, a, row0, lane, acc, acc2);
    else mv_dispatch<R, true>(Ent.W, a, row0, lane, acc, acc2);
    const bool one = Ent.W.type == W_Q4_1 || Ent.W.type == W_Q5_1;
    if constexpr (!EMIT) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const float s = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
            const int row = row0 + r;
            if (lane == 63 && row < Ent.W.M) Ent.y[row] = apply_epi_mv(Ent, row, s);
        }
    } else {
        // 4*R == 32 rows per workgroup: apply the epilogue and emit the 32 values as one
        // quantization block of the next matmul's input (ggml Q8 / fp16 / fp32)
#pragma unroll
        for (int r = 0; r < R; r++) {
            const float s = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
            if (lane == 63) red[wave * R + r] = s;
        }
        __syncthreads();
        if (tid < 32) {
            const int row = rowwg + tid;
            float vv = 0.0f;
            if (row < Ent.W.M) {
                vv = apply_epi_mv(Ent, row, red[tid]);
                if (Ent.y) Ent.y[row] = vv;
            }
            if (Ent.act_out.fmt >= 0 && Ent.emit) emit32(Ent.act_out, 0, row, vv);
        }
    }
}

template <int R, bool EMIT>
static void launch_mv_e(hipStream_t st, MVGroup & g, int E, int blocks) {
    dim3 grid(blocks), block(256);
    switch (E) {
        case 4: hipLaunchKernelGGL((k_mv<R, 4, EMIT>), grid, block, g.lds_bytes, st, g); break;
        case 16: hipLaunchKernelGGL((k_mv<R, 16, EMIT>), grid, block, g.lds_bytes, st, g); break;
        default: hipLaunchKernelGGL((k_mv<R, 32, EMIT>), grid, block, g.lds_bytes, st, g); break;
    }
}

bool launch_mv_group(hipStream_t st, MVGroup & g) {
    bool emit = false;
    for (int i = 0; i < g.n; i++) emit |= g.e[i].emit != 0;
    const int R = emit ? 8 : 2, RW = 4 * R;
    int blocks = 0, lds = 0, kmax = 0;
    for (int i = 0; i < g.n; i++) {
        MVEntry & e = g.e[i];
        if (e.W.K % 32) {
            fprintf(stderr, "rwkv: matvec needs K %% 32 == 0 (K=%d)\n", e.W.K);
            return false;
        }
        if (e.emit && e.W.M % 32) {
            fprintf(stderr, "rwkv: emitting matvec needs M %% 32 == 0 (M=%d)\n", e.W.M);
            return false;
        }
        e.block0 = blocks;
        blocks += (e.W.M + RW - 1) / RW;
        if (e.src != SRC_ACT) {
            lds = std::max(lds, lds_bytes_for(act_fmt_for(e.W.type), e.W.K));
            kmax = std::max(kmax, e.W.K);
        }
    }
    if (kmax > 32 * 256) {
        fprintf(stderr, "rwkv: matvec prologue K=%d > 8192 unsupported\n", kmax);
        return false;
    }
    g.lds_bytes = lds;
    if (!blocks) return true;
    const int E = kmax <= 1024 ? 4 : kmax <= 4096 ? 16 : 32;
    if (emit) launch_mv_e<8, true>(st, g, E, blocks);
    else launch_mv_e<2, false>(st, g, E, blocks);
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v6 mix5 (decode)
struct Mix5Dec {
    int C, D;
    const float * x, * carry, * lnw, * lnb, * lora, * w2t;
    const float * maa[5];
    ActBuf out[5];
};

// grid (C/256, 5): block (cx, n) computes mixed vector n for 256 channels.  w2t [5][D][C]
// makes the per-channel D-long dots coalesced across lanes; accumulation order matches the
// oracle (sequential over i, fp64).
template <int E>
__global__ __launch_bounds__(256) void k_v6_mix5_dec(Mix5Dec a) {
    __shared__ double sh[8];
    const int n = blockIdx.y, C = a.C, D = a.D;
    float xv[E];
    load_vec<E>(xv, a.x, C);
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = (int)(blockIdx.x * blockDim.x + (threadIdx.x & ~63)) < C;  // wave-uniform
    float w2v[64];
    const float * w2 = a.w2t + (size_t)n * D * C + (active ? c : 0);
#pragma unroll
    for (int i = 0; i < 64; i++) w2v[i] = (i < D) ? w2[(size_t)i * C] : 0.0f;
    const float xc = active ? a.x[c] : 0.0f, cc = active ? a.carry[c] : 0.0f;
    const float lw = active ? a.lnw[c] : 0.0f, lb = active ? a.lnb[c] : 0.0f, mu = active ? a.maa[n][c] : 0.0f;
    float mean, scale;
    ln_stats_reg<E>(xv, C, mean, scale, sh);
    if (!active) return;
    const float xa = ln_apply(xc, mean, scale, lw, lb);
    const float sx = cc - xa;
    const float * lv = a.lora + n * D;
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 64; i++)
        if (i < D) acc += (double)(w2v[i] * lv[i]);
    const float m = (float)acc;
    emit32(a.out[n], 0, c, (m + mu) * sx + xa);
}

bool launch_v6_mix5_dec(hipStream_t st, int C, int D, const float * x, const float * carry, const float * lnw,
                        const float * lnb, const float * lora, const float * w2t, const float * const * maa,
                        const ActBuf * outs) {
    Mix5Dec a;
    a.C = C;
    a.D = D;
    a.x = x;
    a.carry = carry;
    a.lnw = lnw;
    a.lnb = lnb;
    a.lora = lora;
    a.w2t = w2t;
    for (int n = 0; n < 5; n++) {
        a.maa[n] = maa[n];
        a.out[n] = outs[n];
    }
    if (D > 64 || C > 32 * 256) {
        fprintf(stderr, "rwkv: v6 maa LoRA width %d / n_embed %d unsupported\n", D, C);
        return false;
    }
    dim3 grid((C + 255) / 256, 5);
    if (C <= 1024) hipLaunchKernelGGL(k_v6_mix5_dec<4>, grid, dim3(256), 0, st, a);
    else if (C <= 4096) hipLaunchKernelGGL(k_v6_mix5_dec<16>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_v6_mix5_dec<32>, grid, dim3(256), 0, st, a);
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v5/v6 attention (decode)
template <int IPG>
__global__ __launch_bounds__(256) void k_att6_dec(Att6Dec a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float sr[64], sk[64], sv[64], sw[64], su[64], sy[64];
    const int h = blockIdx.x, S = a.S, G = S / IPG, C = a.H * S;
    const int tid = threadIdx.x;
    const int c0 = h * S;
    if (tid < S) {
        sr[tid] = a.r[c0 + tid];
        sk[tid] = a.k[c0 + tid];
        sv[tid] = a.v[c0 + tid];
        su[tid] = a.u[c0 + tid];
        if (a.w) sw[tid] = a.w[c0 + tid];
    }
    if (!a.w) {
        // v6 decay LoRA tail: w = exp(-exp(Wd2 . dl + decay)), rwkv_graph.inc:357-367
        const int D = a.wd2.K;
        ActBuf act = lds_act(smem, act_fmt_for(a.wd2.type), D);
        for (int k0 = 0; k0 < D; k0 += blockDim.x) {
            const int k = k0 + tid;
            if (k0 + (tid & ~31) >= D) continue;
            emit32(act, 0, k, a.dl[k]);
        }
        __syncthreads();
        // rows of Wd2 for this head, one wave per group of rows, lanes over the K blocks with
        // all rows' weight blocks loaded first; reduced with wave_sum63 exactly like the
        // batched matmul kernel (k_mm, T > 1) so serial and sequence stay bit-identical.
        const int nbk = a.wd2.type <= W_F16 ? 0 : D / 32;
        if (nbk > 0 && nbk <= 64) {
            const int lane = tid & 63, nw = blockDim.x >> 6;
            const int rpw = (S + nw - 1) / nw;  // rows per wave (<= 64)
            const int jbase = (tid >> 6) * rpw;
            for (int jj = 0; jj < rpw; jj += 16) {
                float p[16], p2[16];
#pragma unroll
                for (int q = 0; q < 16; q++) p[q] = p2[q] = 0.0f;
                if (lane < nbk) {
                    const int4 * ap = (const int4 *)(act.q + (size_t)lane * 32);
                    const int4 alo = ap[0], ahi = ap[1];
                    const float dx = act.d[lane];
                    const int qs = act.qsum[lane];
                    const float sx = act.fmt == A_Q8_1 ? act.s[lane] : 0.0f;
#pragma unroll
                    for (int q = 0; q < 16; q++) {
                        const int j = min(jbase + jj + q, S - 1);
                        float dw = 0.0f, mw = 0.0f;
                        int sumi = 0;
                        const int row = c0 + j;
                        switch (a.wd2.type) {
                            case W_Q4_0: sumi = block_dot<W_Q4_0>(a.wd2, row, lane, nbk, alo, ahi, qs, dw, mw); break;
                            case W_Q4_1: sumi = block_dot<W_Q4_1>(a.wd2, row, lane, nbk, alo, ahi, qs, dw, mw); break;
                            case W_Q5_0: sumi = block_dot<W_Q5_0>(a.wd2, row, lane, nbk, alo, ahi, qs, dw, mw); break;
                            case W_Q5_1: sumi = block_dot<W_Q5_1>(a.wd2, row, lane, nbk, alo, ahi, qs, dw, mw); break;
                            case W_Q8_0: sumi = block_dot<W_Q8_0>(a.wd2, row, lane, nbk, alo, ahi, qs, dw, mw); break;
                            default: break;
                        }
                        p[q] = fmaf(dw * dx, (float)sumi, 0.0f);
                        p2[q] = 0.0f + mw * sx;
                    }
                }
                const bool one = act.fmt == A_Q8_1;
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    const float sum = one ? wave_sum63(p[q]) + wave_sum63(p2[q]) : wave_sum63(p[q]) + 0.0f;
                    const int j = jbase + jj + q;
                    if (lane == 63 && j < S && jj + q < rpw) sw[j] = expf(-expf(sum + a.decay[c0 + j]));
                }
            }
        } else {
            // F32 / F16 decay LoRA (FP16 checkpoints keep time_decay_w2 in FP32): one wave per row
            const int lane = tid & 63, nw = blockDim.x >> 6;
            for (int j = tid >> 6; j < S; j += nw) {
                float acc[1] = {0.0f}, acc2[1] = {0.0f};
                const int row = c0 + j;
                if (a.wd2.type == W_F32) mv_accumulate<W_F32, 1, false>(a.wd2, act, row, lane, acc, acc2);
                else mv_accumulate<W_F16, 1, false>(a.wd2, act, row, lane, acc, acc2);
                const float sum = wave_sum63(acc[0]) + 0.0f;
                if (lane == 63) sw[j] = expf(-expf(sum + a.decay[row]));
            }
        }
    }
    __syncthreads();
    // wkv6 for one token (ggml_rwkv_wkv6 semantics): lane group (j, g), g splits the keys i
    if (tid < S * G) {
        const int j = tid / G, g = tid % G;
        const size_t hb = (size_t)h * S * S;
        const float vj = sv[j];
        float acc = 0.0f;
#pragma unroll
        for (int ii = 0; ii < IPG; ii++) {
            const int i = g * IPG + ii;
            const float prev = a.sin[hb + (size_t)i * S + j];
            const float kv = vj * sk[i];
            const float temp = kv * su[i] + prev;
            acc += temp * sr[i];
            a.sout[hb + (size_t)i * S + j] = prev * sw[i] + kv;
        }
        acc = group_sum(acc, G);
        if (g == 0) sy[j] = acc;
    }
    __syncthreads();
    // GroupNorm over the head (ggml_norm, fp64 sums) * ln_x (+ b) (* g)
    if (tid < S) {
        const float x = sy[tid];
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
        a.y[c0 + tid] = o;
    }
    (void)C;
}

bool launch_att6_dec(hipStream_t st, const Att6Dec & a) {
    if (a.S > 64 || (a.S & (a.S - 1))) {
        fprintf(stderr, "rwkv: head size %d unsupported\n", a.S);
        return false;
    }
    int G = 256 / a.S;
    if (G > a.S) G = a.S;
    const int IPG = a.S / G;
    int threads = a.S * G;
    int lds = 0;
    if (!a.w) {
        const int D = a.wd2.K;
        threads = std::max(threads, (D + 63) / 64 * 64);
        lds = lds_bytes_for(act_fmt_for(a.wd2.type), D);
    }
    threads = std::min(std::max(threads, 64), 256);
    dim3 grid(a.H), block(threads);
    switch (IPG) {
        case 1: hipLaunchKernelGGL(k_att6_dec<1>, grid, block, lds, st, a); break;
        case 2: hipLaunchKernelGGL(k_att6_dec<2>, grid, block, lds, st, a); break;
        case 4: hipLaunchKernelGGL(k_att6_dec<4>, grid, block, lds, st, a); break;
        case 8: hipLaunchKernelGGL(k_att6_dec<8>, grid, block, lds, st, a); break;
        case 16: hipLaunchKernelGGL(k_att6_dec<16>, grid, block, lds, st, a); break;
        default: return false;
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
        a.y[c] = o;
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
