// device_common.hpp -- device helpers shared by the kernel translation units.
#pragma once

#include "common.hpp"
#include "stamp.hpp"

namespace rwkvmi {

// --------------------------------------------------------------------------- helpers

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Full-wave float sum with DPP (no LDS traffic): quad butterflies, row half-mirror and mirror
// give every lane its 16-lane row sum, then row_bcast15 / row_bcast31 fold the rows upward.
// The total is valid in lane 63 only.  Every matmul kernel (decode and sequence) reduces with
// this one function, so both paths round identically.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_add(float v) {
    const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xF, false);
    return v + __builtin_bit_cast(float, o);
}

__device__ __forceinline__ float wave_sum63(float v) {
    v = dpp_add<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v = dpp_add<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v = dpp_add<0x141, 0xF>(v);  // row_half_mirror
    v = dpp_add<0x140, 0xF>(v);  // row_mirror
    v = dpp_add<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_add<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
    return v;
}

// sum over groups of `width` adjacent lanes (width power of two <= 64); all lanes get the sum
template <typename T>
__device__ __forceinline__ T group_sum(T v, int width) {
    for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_add_d(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, ROW_MASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xF, false);
    const long long o = ((long long)hi << 32) | (long long)(unsigned)lo;
    return v + __builtin_bit_cast(double, o);
}

// wave_sum63 for doubles (same tree); valid in lane 63
__device__ __forceinline__ double wave_sum63_d(double v) {
    v = dpp_add_d<0xB1, 0xF>(v);
    v = dpp_add_d<0x4E, 0xF>(v);
    v = dpp_add_d<0x141, 0xF>(v);
    v = dpp_add_d<0x140, 0xF>(v);
    v = dpp_add_d<0x142, 0xA>(v);
    v = dpp_add_d<0x143, 0xC>(v);
    return v;
}

// deterministic block sum (fixed tree): every thread returns the total.  Every LayerNorm on
// the device (decode prologues and the sequence kernels) reduces through this one function.
__device__ inline double block_sum_d(double v, double * sh) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum63_d(v);
    if (lane == 63) sh[wave] = v;
    __syncthreads();
    double r = 0.0;
    for (int w = 0; w < nw; w++) r += sh[w];
    __syncthreads();
    return r;
}

// exp / tanh as fixed sequences of IEEE-exact operations (fma, mul, add, correctly rounded
// division, rint, ldexp), so a CPU restatement reproduces every result bit for bit (the oracle's
// GPU-association variant, oracle.c gpu_expf / gpu_tanhf).  The device libm (ocml) routes exp
// through v_exp_f32, whose rounding is not specified.  Accuracy: <= 1 ulp over the float range.
//   exp: x = n ln2 + r (Cody-Waite, |r| <= ln2/2), e^r = 1 + r + r^2 Q(r), degree-4 Q (fitted).
//   tanh: |x| < 0.625: x + x^3 P(x^2), degree-4 P (fitted); else 1 - 2 / (e^{2|x|} + 1).
__device__ __forceinline__ float rk_expf(float x) {
    if (x != x) return x;
    if (x > 0x1.62e43p+6f) return __int_as_float(0x7f800000);
    if (x < -0x1.9fe36ap+6f) return 0.0f;
    const float n = rintf(x * 0x1.715476p+0f);
    float r = fmaf(n, -0x1.62e43p-1f, x);
    r = fmaf(n, 0x1.05c61p-29f, r);
    float q = 0x1.687c22p-10f;
    q = fmaf(q, r, 0x1.123b8ep-7f);
    q = fmaf(q, r, 0x1.555b58p-5f);
    q = fmaf(q, r, 0x1.55548ep-3f);
    q = fmaf(q, r, 0x1.fffff8p-2f);
    const float r2 = r * r;
    const float p = fmaf(r2, q, r) + 1.0f;
    return ldexpf(p, (int)n);
}
__device__ __forceinline__ float rk_tanhf(float x) {
    const float ax = fabsf(x);
    if (ax < 0.625f) {
        const float x2 = x * x;
        float p = -0x1.7507acp-8f;
        p = fmaf(p, x2, 0x1.51f0f0p-6f);
        p = fmaf(p, x2, -0x1.b83322p-5f);
        p = fmaf(p, x2, 0x1.1106d6p-3f);
        p = fmaf(p, x2, -0x1.555532p-2f);
        return fmaf(x * x2, p, x);
    }
    const float t = ax > 9.0f ? 1.0f : 1.0f - 2.0f / (rk_expf(ax + ax) + 1.0f);
    return copysignf(t, x);
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + rk_expf(-x)); }
__device__ __forceinline__ float siluf_(float x) { return x / (1.0f + rk_expf(-x)); }

__device__ __forceinline__ float h2f(uint16_t b) { return __half2float(__ushort_as_half(b)); }
// f32 -> f16 of a value that was first rounded to f32 (ggml's GGML_FP32_TO_FP16(d * sum): two
// roundings).  The empty asm pins f as an f32 register value: without it the backend folds
// fptrunc(fmul(a, b)) into v_fma_mixlo_f16 a, b, 0 -- ONE rounding of the exact product, which
// differs from the two-step result whenever the f32 product lands on an f16 midpoint
// (tools/debug_stage.py found it in the Q8_1 s = d * sum of the activation quantizer).
__device__ __forceinline__ __half to_half(float f) {
    asm volatile("" : "+v"(f));
    return __float2half(f);
}
__device__ __forceinline__ float f16_round(float f) { return __half2float(to_half(f)); }

// Reductions across each 32-lane half-wave (all lanes get the result): DPP inside the 16-lane
// rows, then v_permlane16_swap between the two rows of the half.  Max and integer sums are
// order-independent, so these are exact.
template <int CTRL>
__device__ __forceinline__ int dpp_mov(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ float half_max(float v) {
    v = fmaxf(v, __int_as_float(dpp_mov<0xB1>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_mov<0x4E>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_mov<0x141>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_mov<0x140>(__float_as_int(v))));
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    return fmaxf(__int_as_float(p[0]), __int_as_float(p[1]));
}
__device__ __forceinline__ int half_sum_i(int v) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return p[0] + p[1];
}

// ggml quantize_row_q8_0 / q8_1 (x86) of one 32-block held one element per lane of a
// half-wave: d = amax/127 (fp16), q = rint(x * 127/amax), sum = sum q.  Pure (no stores), so
// several blocks can be quantized in flight before any is written.
struct Q32 {
    int q;
    float d;
    int sum;
};
__device__ __forceinline__ Q32 quant32(float v) {
    const float am = half_max(fabsf(v));
    const float id = (am != 0.0f) ? 127.f / am : 0.0f;
    Q32 r;
    r.q = (int)rintf(v * id);
    r.d = am / 127.f;
    r.sum = half_sum_i(r.q);
    return r;
}

// Store element k of row t (and, from the block's first lane, its scales).
__device__ __forceinline__ void store32(const ActBuf & a, int t, int k, const Q32 & r) {
    if (a.tiled) {  // sequence-GEMM token-tile record (common.hpp qg_*)
        const bool one = a.fmt == A_Q8_1;
        uint8_t * rec = a.tq + ((size_t)(t / QG_TOK) * (a.K >> 5) + (k >> 5)) * qg_a_bytes(one);
        const int tl = t % QG_TOK;
        rec[((k >> 4) & 1) * QG_TOK * 16 + tl * 16 + (k & 15)] = (uint8_t)(int8_t)r.q;
        if ((k & 31) == 0) {
            ((float *)(rec + QG_A_D))[tl] = f16_round(r.d);
            if (one) ((float *)(rec + QG_A_S))[tl] = f16_round(r.d * (float)r.sum);
        }
        return;
    }
    const size_t idx = (size_t)t * a.K + k;
    a.q[idx] = (int8_t)r.q;
    if ((k & 31) == 0) {
        const size_t bi = (size_t)t * (a.K >> 5) + (k >> 5);
        a.d[bi] = f16_round(r.d);
        a.qsum[bi] = r.sum;
        if (a.fmt == A_Q8_1) a.s[bi] = f16_round(r.d * (float)r.sum);
    }
}

// An activation record's fields forced into registers at this point (the kernarg loads issued and
// waited here, at the kernel's start, instead of on the critical path where they are first used).
__device__ __forceinline__ void pin_act(const ActBuf & a) {
    asm volatile("" ::"s"(a.q), "s"(a.d));
    asm volatile("" ::"s"(a.s), "s"(a.qsum));
    asm volatile("" ::"s"(a.h), "s"(a.f));
    asm volatile("" ::"s"(a.tq), "s"(a.fmt), "s"(a.K), "s"(a.tiled));
}

// Emit one element per lane into an activation buffer.  The 32 lanes of each half-wave must
// hold the 32 consecutive elements of one block (k & 31 == lane & 31) of the same row t, and
// all 32 must call (block-uniform control flow).
__device__ __forceinline__ void emit32(const ActBuf & a, int t, int k, float v) {
    const size_t idx = (size_t)t * a.K + k;
    if (a.fmt == A_F32) {
        a.f[idx] = v;
        return;
    }
    if (a.fmt == A_F16) {
        a.h[idx] = to_half(v);
        return;
    }
    store32(a, t, k, quant32(v));
}

// --------------------------------------------------------------------------- matmul
// One workgroup = 4 waves; each wave owns RPW consecutive rows; lanes stride over the K
// blocks of a row (lane l reads block l, l+64, ...: one 16-byte dwordx4 of nibbles per lane,
// 1 KiB per wave-instruction, fully coalesced).  Per 32-block: integer v_dot4 of the weight
// ints with the Q8 activation ints, then acc = fma(d_w * d_x, sumi, acc) (ggml x86 order);
// the m*s terms of the _1 formats go to a second accumulator added at the end.

__device__ __forceinline__ uint32_t spread4(uint32_t x) {
    // bit k of x (k<4) -> bit 4 of byte k
    return ((x & 1u) << 4) | ((x & 2u) << 11) | ((x & 4u) << 18) | ((x & 8u) << 25);
}

// One quantized weight block, loaded (phase 1) separately from its use (phase 2) so a lane can
// keep several 16-byte HBM loads in flight.
struct WBlk {
    int4 q0, q1;     // nibbles (Q4/Q5: q0 only) or int8 (Q8_0: q0, q1)
    uint32_t qh;     // Q5 high bits
    uint32_t sc;     // fp16 d (low half) | fp16 m << 16 (_1 formats)
};

// Weight loads.  NT: non-temporal (`nt`) loads for bytes that ONE workgroup reads once per
// token (the decode matvec stream, 1 GB per v6-1B6 token, far larger than L2 + MALL): they do
// not displace the activations and state the chain re-reads (MI355X_MICROARCH.md nt-weights).
typedef int wld_i32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ int4 ld16w(const void * p) {
    if constexpr (NT) {
        const wld_i32x4 t = __builtin_nontemporal_load((const wld_i32x4 *)p);
        return make_int4(t.x, t.y, t.z, t.w);
    } else {
        return *(const int4 *)p;
    }
}
template <bool NT, typename T>
__device__ __forceinline__ T ldw(const T * p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// Offsets in 32 bits (a weight tensor is far below 4 GiB): base (SGPR) + 32-bit offset is the
// saddr load form, whose offset register is not the destination -- with 64-bit per-lane addresses
// the compiler reuses an address register as a later load's destination and must wait for the
// earlier load to return before issuing the next (waits inside the weight stream's issue).
template <int WF, bool NT = false>
__device__ __forceinline__ WBlk load_wblk(const DMat & W, size_t bi_) {
    WBlk w;
    const uint32_t bi = (uint32_t)bi_;
    if constexpr (WF == W_Q8_0) {
        const int4 * p = (const int4 *)(W.qs + bi * 32u);
        w.q0 = ld16w<NT>(p);
        w.q1 = ld16w<NT>((const int4 *)(W.qs + (bi * 32u + 16u)));
    } else {
        w.q0 = ld16w<NT>(W.qs + bi * 16u);
        w.q1 = make_int4(0, 0, 0, 0);
    }
    w.qh = (WF == W_Q5_0 || WF == W_Q5_1) ? ldw<NT>((const uint32_t *)((const char *)W.qh + bi * 4u)) : 0u;
    if constexpr (WF == W_Q4_1 || WF == W_Q5_1) w.sc = ldw<NT>((const uint32_t *)((const char *)W.sc + bi * 4u));
    else w.sc = ldw<NT>((const uint16_t *)((const char *)W.sc + bi * 2u));
    return w;
}

template <int WF>
__device__ __forceinline__ int dot_wblk(const WBlk & w, const int4 & alo, const int4 & ahi, int qsum, float & dw,
                                        float & mw) {
    int sumi = 0;
    if constexpr (WF == W_Q8_0) {
        sumi = __builtin_amdgcn_sdot4(w.q0.x, alo.x, sumi, false);
        sumi = __builtin_amdgcn_sdot4(w.q0.y, alo.y, sumi, false);
        sumi = __builtin_amdgcn_sdot4(w.q0.z, alo.z, sumi, false);
        sumi = __builtin_amdgcn_sdot4(w.q0.w, alo.w, sumi, false);
        sumi = __builtin_amdgcn_sdot4(w.q1.x, ahi.x, sumi, false);
        sumi = __builtin_amdgcn_sdot4(w.q1.y, ahi.y, sumi, false);
        sumi = __builtin_amdgcn_sdot4(w.q1.z, ahi.z, sumi, false);
        sumi = __builtin_amdgcn_sdot4(w.q1.w, ahi.w, sumi, false);
        dw = h2f((uint16_t)(w.sc & 0xFFFF));
        mw = 0.0f;
        (void)qsum;
        return sumi;
    } else {
        uint32_t lo0 = (uint32_t)w.q0.x & 0x0F0F0F0Fu, lo1 = (uint32_t)w.q0.y & 0x0F0F0F0Fu;
        uint32_t lo2 = (uint32_t)w.q0.z & 0x0F0F0F0Fu, lo3 = (uint32_t)w.q0.w & 0x0F0F0F0Fu;
        uint32_t hi0 = ((uint32_t)w.q0.x >> 4) & 0x0F0F0F0Fu, hi1 = ((uint32_t)w.q0.y >> 4) & 0x0F0F0F0Fu;
        uint32_t hi2 = ((uint32_t)w.q0.z >> 4) & 0x0F0F0F0Fu, hi3 = ((uint32_t)w.q0.w >> 4) & 0x0F0F0F0Fu;
        if constexpr (WF == W_Q5_0 || WF == W_Q5_1) {
            const uint32_t qh = w.qh;
            lo0 |= spread4(qh & 0xF);
            lo1 |= spread4((qh >> 4) & 0xF);
            lo2 |= spread4((qh >> 8) & 0xF);
            lo3 |= spread4((qh >> 12) & 0xF);
            hi0 |= spread4((qh >> 16) & 0xF);
            hi1 |= spread4((qh >> 20) & 0xF);
            hi2 |= spread4((qh >> 24) & 0xF);
            hi3 |= spread4((qh >> 28) & 0xF);
        }
        sumi = __builtin_amdgcn_sdot4((int)lo0, alo.x, sumi, false);
        sumi = __builtin_amdgcn_sdot4((int)lo1, alo.y, sumi, false);
        sumi = __builtin_amdgcn_sdot4((int)lo2, alo.z, sumi, false);
        sumi = __builtin_amdgcn_sdot4((int)lo3, alo.w, sumi, false);
        sumi = __builtin_amdgcn_sdot4((int)hi0, ahi.x, sumi, false);
        sumi = __builtin_amdgcn_sdot4((int)hi1, ahi.y, sumi, false);
        sumi = __builtin_amdgcn_sdot4((int)hi2, ahi.z, sumi, false);
        sumi = __builtin_amdgcn_sdot4((int)hi3, ahi.w, sumi, false);
        if constexpr (WF == W_Q4_0) {
            sumi -= 8 * qsum;
        } else if constexpr (WF == W_Q5_0) {
            sumi -= 16 * qsum;
        }
        dw = h2f((uint16_t)(w.sc & 0xFFFF));
        mw = (WF == W_Q4_1 || WF == W_Q5_1) ? h2f((uint16_t)(w.sc >> 16)) : 0.0f;
        return sumi;
    }
}

template <int WF>
__device__ __forceinline__ int block_dot(const DMat & W, int row, int b, int nb, const int4 & alo,
                                         const int4 & ahi, int qsum, float & dw, float & mw) {
    const WBlk w = load_wblk<WF>(W, (size_t)row * nb + b);
    return dot_wblk<WF>(w, alo, ahi, qsum, dw, mw);
}

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

// F16 dot of one 16-byte unit (8 halves of w and x): acc = fma(w[k], x[k], acc) for k = 0..7 in
// order, the halves widened exactly to f32.  (v_dot2_f32_f16 is not used: its internal rounding
// is unspecified -- tools/arith_probe.hip measured 11% of results off a single-rounding model --
// so no CPU restatement could reproduce it.)
__device__ __forceinline__ float dot8_f16(const int4 & w, const int4 & x, float acc) {
    const int wv[4] = {w.x, w.y, w.z, w.w}, xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const half2_t a = __builtin_bit_cast(half2_t, wv[i]), b = __builtin_bit_cast(half2_t, xv[i]);
        acc = fmaf((float)a.x, (float)b.x, acc);
        acc = fmaf((float)a.y, (float)b.y, acc);
    }
    return acc;
}

// apply_epi with y[t][row] (yv) and aux[t][row] (av) already loaded (only read by the epilogues
// that use them: ADD / SIGMUL_ADD / VMIX7)
__device__ __forceinline__ float apply_epi_v(const MMEntry & E, int row, float acc, float yv, float av) {
    switch (E.epi) {
        case EPI_SIGMOID: return sigmoidf_(acc);
        case EPI_TANH: return rk_tanhf(acc);
        case EPI_SILU: return siluf_(acc);
        case EPI_RELU_SQ: {
            const float r = acc > 0.0f ? acc : 0.0f;
            return r * r;
        }
        case EPI_ADD: return yv + acc;
        case EPI_SIGMUL_ADD: return yv + sigmoidf_(av) * acc;
        case EPI_DECAY6: return rk_expf(-rk_expf(acc + E.bias[row]));
        case EPI_DECAY7: return rk_expf(sigmoidf_(acc + E.bias[row]) * -0.606531f);
        case EPI_SIGMOID_BIAS: return sigmoidf_(acc + E.bias[row]);
        case EPI_VMIX7: return yv + (av - yv) * sigmoidf_(acc + E.bias[row]);
        default: return acc;
    }
}
__device__ __forceinline__ bool epi_reads_y(int epi) { return epi == EPI_ADD || epi == EPI_SIGMUL_ADD || epi == EPI_VMIX7; }
__device__ __forceinline__ bool epi_reads_aux(int epi) { return epi == EPI_SIGMUL_ADD || epi == EPI_VMIX7; }

__device__ __forceinline__ float apply_epi(const MMEntry & E, int t, int row, float acc) {
    const size_t yi = (size_t)t * E.ldy + row;
    switch (E.epi) {
        case EPI_SIGMOID: return sigmoidf_(acc);
        case EPI_TANH: return rk_tanhf(acc);
        case EPI_SILU: return siluf_(acc);
        case EPI_RELU_SQ: {
            const float r = acc > 0.0f ? acc : 0.0f;
            return r * r;
        }
        case EPI_ADD: return E.y[yi] + acc;
        case EPI_SIGMUL_ADD: return E.y[yi] + sigmoidf_(E.aux[yi]) * acc;
        case EPI_DECAY6: return rk_expf(-rk_expf(acc + E.bias[row]));
        case EPI_DECAY7: return rk_expf(sigmoidf_(acc + E.bias[row]) * -0.606531f);
        case EPI_SIGMOID_BIAS: return sigmoidf_(acc + E.bias[row]);
        case EPI_VMIX7: {
            const float v = E.y[yi];
            return v + (E.aux[yi] - v) * sigmoidf_(acc + E.bias[row]);
        }
        default: return acc;
    }
}


// ggml_norm statistics with double accumulation (mean, 1/sqrt(var + eps))
// Sum across the wave, result broadcast to every lane.
__device__ __forceinline__ double wave_allsum_d(double v) {
    v = wave_sum63_d(v);
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// s / n for the statistics' means: a power-of-two n divides by scaling (v_ldexp, exact and
// bit-identical to the correctly rounded division), other n take the fp64 division.
__device__ __forceinline__ double div_count(double s, int n) {
    return (n & (n - 1)) == 0 ? ldexp(s, -__builtin_ctz((unsigned)n)) : s / (double)n;
}

// Per-head fp64 sum (GroupNorm statistics) in wave_sum63's association -- adjacent lanes
// paired first -- with the result on every lane of the group.  Width 64: the DPP tree plus a
// lane-63 broadcast (no LDS round trips); narrower groups: the xor butterfly with the stride
// doubling (1, 2, 4, ...), which folds in the same order.
__device__ __forceinline__ double group_tree_sum_d(double v, int width) {
    if (width == 64) return wave_allsum_d(v);
    for (int o = 1; o < width; o <<= 1) v += __shfl_xor(v, o);
    return v;
}

// LayerNorm statistics (ggml_norm: fp64 accumulation, population variance) in ONE pass, in the
// CHUNK association that every LayerNorm on the device and the oracle's GPU variant share:
// x is cut into 512-element chunks; lane l of a chunk owns its 8 consecutive elements 8l..8l+7
// (two 16-byte loads), whose values and exact squares ((double)x * (double)x: 48 significant
// bits) are summed as fp64 pairwise trees; a chunk's 64 lane sums fold by wave_sum63's tree;
// chunk sums are added in ascending chunk order.  Elements past K count as zeros (K % 8 == 0).
// mean = S1 / K, var = max(S2 / K - mean_d^2, 0) in fp64, rounded to f32 once (ln_finish).
// ggml's second pass sums fp32-rounded (x - mean_f32)^2; this one-pass form is the same
// quantity without those roundings (every statistic needs one exchange instead of two).  The
// decode prologues spread the chunks over several waves and exchange the chunk sums through
// LDS; the sequence kernels walk the chunks in one wave -- same bits.
constexpr int LN_CHUNK = 512;

__device__ __forceinline__ double ln_tree8(const float (&v)[8]) {
    const double a = ((double)v[0] + (double)v[1]) + ((double)v[2] + (double)v[3]);
    const double b = ((double)v[4] + (double)v[5]) + ((double)v[6] + (double)v[7]);
    return a + b;
}
__device__ __forceinline__ double ln_tree8_sq(const float (&v)[8]) {
    double q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = (double)v[j] * (double)v[j];
    const double a = (q[0] + q[1]) + (q[2] + q[3]);
    const double b = (q[4] + q[5]) + (q[6] + q[7]);
    return a + b;
}
// sums of one chunk's elements and squares (every lane gets them); x = this lane's 8 elements
__device__ __forceinline__ void ln_chunk_sums(const float (&x)[8], bool valid, double & s1, double & s2) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = valid ? x[j] : 0.0f;
    const double a = ln_tree8(v), b = ln_tree8_sq(v);  // two independent DPP chains
    s1 = wave_allsum_d(a);
    s2 = wave_allsum_d(b);
}
__device__ __forceinline__ void ln_finish(double s1, double s2, int K, float eps, float & mean, float & scale) {
    const double md = div_count(s1, K);
    double vd = div_count(s2, K) - md * md;
    vd = vd > 0.0 ? vd : 0.0;
    mean = (float)md;
    scale = 1.0f / sqrtf((float)vd + eps);
}


__device__ __forceinline__ void ln_load8(float (&v)[8], const float * x, int k, int K) {
    const float * p = x + min(k, K - 8);
    const float4 a = *(const float4 *)p, b = *(const float4 *)(p + 4);
    v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
}

// One wave, the chunks already in registers (nc <= NC): x[c] = this lane's 8 elements of chunk c.
// The chunk sums are independent DPP chains, so their latencies overlap.
template <int NC>
__device__ __forceinline__ void ln_stats_regs(const float (&x)[NC][8], int nc, int K, float eps, float & mean,
                                              float & scale) {
    const int lane = threadIdx.x & 63;
    double c1[NC], c2[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) {
        c1[c] = c2[c] = 0.0;
        if (c < nc) ln_chunk_sums(x[c], c * LN_CHUNK + lane * 8 < K, c1[c], c2[c]);
    }
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int c = 0; c < NC; c++)
        if (c < nc) s1 += c1[c], s2 += c2[c];
    ln_finish(s1, s2, K, eps, mean, scale);
}

// One wave, any K (x 16-byte aligned): the chunks in ascending order, 4 in flight at a time.
__device__ inline void ln_stats_wave(const float * x, int K, float eps, float & mean, float & scale) {
    const int lane = threadIdx.x & 63, nc = (K + LN_CHUNK - 1) / LN_CHUNK;
    double s1 = 0.0, s2 = 0.0;
    for (int c0 = 0; c0 < nc; c0 += 4) {
        float v[4][8];
#pragma unroll
        for (int c = 0; c < 4; c++) ln_load8(v[c], x, min(c0 + c, nc - 1) * LN_CHUNK + lane * 8, K);
        double c1[4], c2[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            c1[c] = c2[c] = 0.0;
            if (c0 + c < nc) ln_chunk_sums(v[c], (c0 + c) * LN_CHUNK + lane * 8 < K, c1[c], c2[c]);
        }
#pragma unroll
        for (int c = 0; c < 4; c++)
            if (c0 + c < nc) s1 += c1[c], s2 += c2[c];
    }
    ln_finish(s1, s2, K, eps, mean, scale);
}

__device__ __forceinline__ void ln_stats_any(const float * x, int K, float eps, float & mean, float & scale) {
    ln_stats_wave(x, K, eps, mean, scale);
}

// Block-level entry point kept for the sequence kernels: every wave computes the same
// statistics itself (sh unused).
__device__ inline void ln_stats(const float * x, int C, float eps, float & mean, float & scale, double * sh) {
    (void)sh;
    ln_stats_any(x, C, eps, mean, scale);
}

__device__ __forceinline__ float ln_apply(float x, float mean, float scale, float w, float b) {
    float y = (x - mean) * scale;
    y = y * w;
    return y + b;
}


}  // namespace rwkvmi
