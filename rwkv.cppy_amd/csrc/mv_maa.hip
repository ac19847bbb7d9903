// mv_maa.hip -- v6 decode: the maa LoRA in one launch (rwkv_graph.inc:306-346).
//
// Before: W1 matvec with the LN prologue (lora = tanh(W1 . xxx), one launch) then the W2 mix
// (k_v6_mix5_dec, a second launch that waits for the whole lora vector).  The mixed vector n
// only needs lora_n = rows [n*D, (n+1)*D) of W1, so workgroup (cx, n) computes those D rows
// itself -- LayerNorm + token shift + Q8 quantization of xxx in LDS (exactly the k_mv prologue),
// D rows dotted by the dot waves (exactly k_mv's lane/unit order and wave_sum63 tree, so the
// lora values are bit-identical) -- and then mixes its 256 channels (exactly k_v6_mix5_dec).
// The five row chunks are each recomputed by C/256 workgroups (W1 is 5*D x C: 37 KB per chunk
// for v6-1B6 Q4_0, read from L2), which replaces one dependent launch per layer.
#include "mv_maa.hpp"

#include <stdlib.h>
#include <string.h>

namespace rwkvmi {


// 512 threads.  Waves 4..7 build the activation image (LayerNorm + token shift + quantization,
// one 512-element chunk per wave per pass) and the fp32 xa image; then every wave dots R rows of
// W1 (D <= 8R: the image waves issue their weight loads right behind their input loads, so the
// rows stream while the LayerNorm runs), and waves 0..3 mix one channel per thread (its W2 column
// prefetched).  Each wave keeps well under 63 loads in flight, so none stalls on the vmcnt limit.
template <int WF, int R, int U, int LNP, int DM, int CPW>
__global__ __launch_bounds__(512) void k_v6_maa_dec(MaaDec a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float s_lora[64];
    const int n = blockIdx.y, C = a.C, D = a.D, K = C;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform branches
    const bool pro = wave >= 4;
    const int pw = wave - 4;
    const ActBuf act = lds_act(smem, act_fmt_for(WF), K);
    float * s_xa = (float *)(smem + a.xa_off);
    STAMP_BEGIN();
    // the emission target's fields in SGPRs now, not a scalar round trip after the mix
    const ActBuf ao = a.out[n];
    pin_act(ao);
    const DMat & W = a.w1;
    MVEntry E;
    E.x = a.x;
    E.carry = a.carry;
    E.lnw = a.lnw;
    E.lnb = a.lnb;
    E.mu = a.maa_x;
    E.carry_out = a.carry_out;
    E.f = nullptr;
    constexpr int LCW = LNP > 32 ? 2 : 1;
    const int nch = (K + LN_CHUNK - 1) / LN_CHUNK;
    ChunkIn ci[LCW];
    int kc[LCW];
    // chunks pw, pw + 4 of the LayerNorm input (512 elements each, 8 per lane); issued by every
    // wave without a branch (chunk_load_all: the mix waves' loads are empty)
#pragma unroll
    for (int q = 0; q < LCW; q++) {
        kc[q] = (pw + 4 * q) * LN_CHUNK + lane * 8;
        chunk_load_all<MVK_LN, 1>(E, max(min(kc[q], K - 8), 0), ci[q], pro);
    }
    asm volatile("" ::"s"(a.w1.qs), "s"(a.w1.sc), "s"(a.w1.qh));  // pointers before the barrier
    asm volatile("s_barrier" ::: "memory");  // image inputs issued ahead of the weight stream
    // ---- rows n*D + wave*R + r of W1 (all waves)
    const int units = mv_units(WF, K);
    const int row0 = n * D + wave * R, rlast = n * D + D - 1;
    int rows[R];
#pragma unroll
    for (int r = 0; r < R; r++) rows[r] = min(row0 + r, rlast);
    WBlk w[R][U];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < R; r++) w[r][u] = load_unit<WF, false>(W, rows[r], u, lane);
    if (pw == 0) STAMP_XN(0);  // weights issued
    // this thread's mix channel (waves 0..3): W2 column, carry, maa.  Issued by every wave without
    // a branch, the image waves' descriptors empty (as chunk_load_all): loads on one side of a
    // branch make the compiler's wait counts at the join conservative -- the image waves would
    // wait for their whole weight stream before the LayerNorm statistics.  Rows i >= D of the
    // column repeat row D - 1; the mix chain skips them.
    const int c = blockIdx.x * CPW + tid;
    const bool cval = tid < CPW && (int)(blockIdx.x * CPW + (tid & ~31)) < C;  // half-wave uniform
    const int cc = min(c, C - 1);
    float w2v[DM];
    float carry_c, mu_c;
    {
        const int on = pro ? 0 : 0x7fffffff;
        const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc((void *)(a.w2t + (size_t)n * D * C), 0, on, 0x00020000);
#pragma unroll
        for (int i = 0; i < DM; i++)
            w2v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2, (min(i, D - 1) * C + cc) * 4, 0, 0));
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void *)a.carry, 0, on, 0x00020000);
        const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc((void *)a.maa[n], 0, on, 0x00020000);
        carry_c = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, cc * 4, 0, 0));
        mu_c = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rm, cc * 4, 0, 0));
    }
    if (pro) {
        // LayerNorm statistics, chunk association, one pass (device_common.hpp); every wave joins
        // the exchange barrier
        __shared__ double ln_part[2][8];
#pragma unroll
        for (int q = 0; q < LCW; q++)
            if (pw + 4 * q < nch) {
                double c1, c2;
                ln_chunk_sums(ci[q].x, kc[q] < K, c1, c2);
                if (lane == 0) {
                    ln_part[0][pw + 4 * q] = c1;
                    ln_part[1][pw + 4 * q] = c2;
                }
            }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        double s1 = 0.0, s2 = 0.0;
        for (int q = 0; q < nch; q++) s1 += ln_part[0][q], s2 += ln_part[1][q];
        float mean, scale;
        ln_finish(s1, s2, K, 1e-5f, mean, scale);
#ifdef RWKV_STAMP
        if (pw == 0 && lane == 0) stamp_x_[1] = __builtin_amdgcn_s_memrealtime() + (scale == 1.2345f);
#endif
        const bool write_carry = blockIdx.x == 0 && n == 0;
#pragma unroll
        for (int q = 0; q < LCW; q++) {
            if (pw + 4 * q >= nch) continue;
            if (kc[q] < K) {
#pragma unroll
                for (int j = 0; j < 8; j++) s_xa[kc[q] + j] = ln_apply(ci[q].x[j], mean, scale, ci[q].w[j], ci[q].b[j]);
            }
            chunk_store<WF, MVK_LN, 1>(E, act, ci[q], mean, scale, write_carry, kc[q], kc[q] < K, lane);
        }
        if (pw == 0) STAMP_XN(2);
    } else {
        asm volatile("s_barrier" ::: "memory");  // the image waves' statistics exchange
    }
    __syncthreads();  // (1) activation image ready
    if (wave == 0) STAMP_MID();
    float acc[R], acc2[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
    for (int u0 = 0; u0 < units; u0 += U) {
        if (u0 > 0) {
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int r = 0; r < R; r++) w[r][u] = load_unit<WF, false>(W, rows[r], u0 + u, lane);
        }
        AUnit xu[U];
#pragma unroll
        for (int u = 0; u < U; u++) xu[u] = load_act_unit<WF, true>(act, u0 + u, lane);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (unit_valid<WF>(K, u0 + u, lane)) {
#pragma unroll
                for (int r = 0; r < R; r++) dot_unit<WF>(w[r][u], xu[u], acc[r], acc2[r]);
            }
        }
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    float sr[R];
#pragma unroll
    for (int r = 0; r < R; r++) sr[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
    const float t = rk_tanhf(lane_row_sum<R>(sr, lane));  // EPI_TANH, lane r for row r
    if (lane < R && wave * R + lane < D) s_lora[wave * R + lane] = t;
    __syncthreads();  // (2) lora_n ready
    if (wave == 0) STAMP_X(3);
    if (!pro) {
        // k_v6_mix5_dec's arithmetic: m = fma chain over i in order
        const float xa = s_xa[cc];
        const float sx = carry_c - xa;
        float m = 0.0f;
#pragma unroll
        for (int i = 0; i < DM; i++)
            if (i < D) m = fmaf(w2v[i], s_lora[i], m);
        if (cval) emit32(ao, 0, c, (m + mu_c) * sx + xa);
    }
    STAMP_END_NS(4 + 16 * blockIdx.y);
}

// D <= 32: mv_maa.hpp's workgroup (the image waves have no rows), x read from the residual stream.
// Same arithmetic and association as k_v6_maa_dec (bit-identical).
template <int WF, int U, int LNP, int CPW, bool EMB = false>
__global__ __launch_bounds__(512) void k_v6_maa_dec4(MaaDec a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float s_lora[64];
    __shared__ double ln_part[16];
    STAMP_BEGIN();
    maa_dec4_body<WF, U, LNP, CPW, false, EMB>(a, (int)blockIdx.x, (int)blockIdx.y, smem, s_lora, ln_part, nullptr,
                                               0u, nullptr, 0u);
    STAMP_END_NS(4 + 16 * blockIdx.y);
}

// Channels mixed per workgroup (CPW): the workgroups of one mix each recompute its D rows of W1
// (37 KB of L2 reads for v6-1B6) and stream CPW columns of W2 from HBM; 64 gives 32 x 5 = 160
// workgroups for C = 2048 (256: 40), so the W2 stream is spread over more CUs.
static int maa_cpw() { return 64; }

template <int WF>
static bool launch_maa_t(hipStream_t st, const MaaDec & a, int lds, int units) {
    const int cpw = maa_cpw();
    const dim3 grid((a.C + cpw - 1) / cpw, 5);
#define MAA_L(Rv, Uv, P)                                                                                           \
    do {                                                                                                           \
        if (cpw == 64) RK_LAUNCH((k_v6_maa_dec<WF, Rv, Uv, P, (Rv) * 8, 64>), grid, dim3(512), lds, st, a); \
        else if (cpw == 128) RK_LAUNCH((k_v6_maa_dec<WF, Rv, Uv, P, (Rv) * 8, 128>), grid, dim3(512), lds, st, a); \
        else RK_LAUNCH((k_v6_maa_dec<WF, Rv, Uv, P, (Rv) * 8, 256>), grid, dim3(512), lds, st, a);      \
    } while (0)
#define MAA_P(Rv, Uv) \
    do { if (a.C <= 2048) MAA_L(Rv, Uv, 32); else MAA_L(Rv, Uv, 64); } while (0)
    const bool u1 = units <= 1;
    if (a.D <= 32) {
        // rows on the 4 mix waves only (k_v6_maa_dec4)
#define MAA4_L(Uv, P)                                                                                   \
    do {                                                                                                \
        if (cpw == 64) RK_LAUNCH((k_v6_maa_dec4<WF, Uv, P, 64>), grid, dim3(512), lds, st, a);          \
        else if (cpw == 128) RK_LAUNCH((k_v6_maa_dec4<WF, Uv, P, 128>), grid, dim3(512), lds, st, a);   \
        else RK_LAUNCH((k_v6_maa_dec4<WF, Uv, P, 256>), grid, dim3(512), lds, st, a);                   \
    } while (0)
        if (a.C <= 2048) {
            if (u1) MAA4_L(1, 32); else MAA4_L(2, 32);
        } else {
            if (u1) MAA4_L(1, 64); else MAA4_L(2, 64);
        }
#undef MAA4_L
    } else {
        // rows per wave over all 8 waves (D <= 8R)
        if (u1) MAA_P(8, 1); else MAA_P(8, 2);
    }
#undef MAA_P
#undef MAA_L
    HIP_OK(hipGetLastError());
    return true;
}

bool v6_maa_dec_supported(int C, int D, int w1_type) {
    return D >= 1 && D <= 64 && C % 64 == 0 && C <= 4096 && w1_type >= 0;
}

void v6_maa_dec_args(MaaDec & a, int C, int D, const DMat & w1, const float * x, const float * carry, float * carry_out,
                     const float * lnw, const float * lnb, const float * maa_x, const float * w2t,
                     const float * const * maa, const ActBuf * outs) {
    memset(&a, 0, sizeof(a));
    a.C = C;
    a.D = D;
    a.w1 = w1;
    a.x = x;
    a.carry = carry;
    a.carry_out = carry_out;
    a.lnw = lnw;
    a.lnb = lnb;
    a.maa_x = maa_x;
    a.w2t = w2t;
    for (int i = 0; i < 5; i++) {
        a.maa[i] = maa[i];
        a.out[i] = outs[i];
    }
    a.xa_off = (lds_bytes_for(act_fmt_for(w1.type), C) + 15) & ~15;
}

// layer 0 with the embedding LayerNorm inside (MaaDec::tok): the k_v6_maa_dec4 shapes, an F16 / F32
// embedding of row length C
bool v6_maa_emb_supported(const MaaDec & a) {
    return a.tok && a.xout && a.ln0w && a.ln0b && (a.emb.type == W_F16 || a.emb.type == W_F32) &&
           (int)a.emb.K == a.C && a.D <= 32 && v6_maa_dec_supported(a.C, a.D, a.w1.type) &&
           wtype_quantized(a.w1.type) && (int)a.w1.M == 5 * a.D && (int)a.w1.K == a.C;
}

template <int WF>
static void launch_maa_emb_t(hipStream_t st, const MaaDec & a, int lds, bool u1) {
    const dim3 grid(a.C / 64, 5);
    if (a.C <= 2048) {
        if (u1) RK_LAUNCH((k_v6_maa_dec4<WF, 1, 32, 64, true>), grid, dim3(512), lds, st, a);
        else RK_LAUNCH((k_v6_maa_dec4<WF, 2, 32, 64, true>), grid, dim3(512), lds, st, a);
    } else {
        if (u1) RK_LAUNCH((k_v6_maa_dec4<WF, 1, 64, 64, true>), grid, dim3(512), lds, st, a);
        else RK_LAUNCH((k_v6_maa_dec4<WF, 2, 64, 64, true>), grid, dim3(512), lds, st, a);
    }
}

bool launch_v6_maa_dec_emb(hipStream_t st, const MaaDec & a) {
    if (!v6_maa_emb_supported(a) || maa_cpw() != 64) {
        fprintf(stderr, "rwkv: v6 maa decode with the embedding: unsupported shape\n");
        return false;
    }
    const int lds = a.xa_off + a.C * 4;
    const bool u1 = mv_units(a.w1.type, a.C) <= 1;
    switch (a.w1.type) {
        case W_Q4_0: launch_maa_emb_t<W_Q4_0>(st, a, lds, u1); break;
        case W_Q4_1: launch_maa_emb_t<W_Q4_1>(st, a, lds, u1); break;
        case W_Q5_0: launch_maa_emb_t<W_Q5_0>(st, a, lds, u1); break;
        case W_Q5_1: launch_maa_emb_t<W_Q5_1>(st, a, lds, u1); break;
        default: launch_maa_emb_t<W_Q8_0>(st, a, lds, u1); break;
    }
    HIP_OK(hipGetLastError());
    return true;
}

bool launch_v6_maa_dec(hipStream_t st, int C, int D, const DMat & w1, const float * x, const float * carry,
                       float * carry_out, const float * lnw, const float * lnb, const float * maa_x,
                       const float * w2t, const float * const * maa, const ActBuf * outs) {
    if (!v6_maa_dec_supported(C, D, w1.type) || (int)w1.M != 5 * D || (int)w1.K != C) {
        fprintf(stderr, "rwkv: fused v6 maa decode: unsupported shape (C %d, D %d, W1 %dx%d)\n", C, D,
                (int)w1.M, (int)w1.K);
        return false;
    }
    MaaDec a;
    v6_maa_dec_args(a, C, D, w1, x, carry, carry_out, lnw, lnb, maa_x, w2t, maa, outs);
    const int lds = a.xa_off + C * 4;
    const int units = mv_units(w1.type, C);
    switch (w1.type) {
        case W_F32: return launch_maa_t<W_F32>(st, a, lds, units);
        case W_F16: return launch_maa_t<W_F16>(st, a, lds, units);
        case W_Q4_0: return launch_maa_t<W_Q4_0>(st, a, lds, units);
        case W_Q4_1: return launch_maa_t<W_Q4_1>(st, a, lds, units);
        case W_Q5_0: return launch_maa_t<W_Q5_0>(st, a, lds, units);
        case W_Q5_1: return launch_maa_t<W_Q5_1>(st, a, lds, units);
        case W_Q8_0: return launch_maa_t<W_Q8_0>(st, a, lds, units);
        default: break;
    }
    fprintf(stderr, "rwkv: fused v6 maa decode: weight type %d\n", (int)w1.type);
    return false;
}

}  // namespace rwkvmi
