// mv_att4f.hip -- v4 decode: LayerNorm + token shift, the r, k, v matvecs and the WKV-4
// recurrence (rwkv_graph.inc:253-304) in ONE launch.
//
// Before: one k_mv launch over the 3 C rows of r, k, v (LN prologue), then k_wkv4 (a second
// launch that waits at the kernel boundary for every row although channel c only needs r[c],
// k[c], v[c]).  WKV-4 is per channel, so workgroup b takes channels [32 b, 32 b + 32): it builds
// the three token-shifted LayerNorm images itself (the k_mv prologue, once per workgroup), dots
// its 32 rows of each matrix (8 waves x 4 rows x 3 matrices, exactly k_mv's lane/unit order,
// wave_sum63 tree and epilogues, so r, k, v are bit-identical), runs k_wkv4's per-channel
// arithmetic and emits the 32 outputs -- one quantization block of Wo's input -- with no
// hand-off between workgroups at all.  Small models are launch-bound (v4-169M: 12 layers at
// C = 768), so this removes one dependent launch per layer.
//
// Fused Wo (WO): the channel outputs y are published as tagged granules and Wo's rows run in the
// same launch, on workgroups placed AFTER every producer in the grid ([0, C/8) produce, [C/8,
// C/8 + C/16) gather y and run 16 Wo rows each).  Producers never wait, so a waiting workgroup
// only ever waits on lower-index workgroups, which are dispatched first: the launch drains however
// few of its workgroups are resident (several contexts decoding on one GPU at once).
#include "mv_common.hpp"

#include <stdlib.h>
#include <string.h>

namespace rwkvmi {

struct Att4Fused {
    int C;
    DMat W[3];                  // r, k, v (M = K = C)
    const float * x;            // residual stream [C]
    const float * carry;        // previous att_xx [C]
    float * carry_out;          // new att_xx [C] (= LN(x)), written by workgroup 0
    const float * lnw, * lnb;
    const float * mix[3];       // time_mix_r, _k, _v [C]
    const float * first, * decay;
    const float * sin;          // layer state in: [aa | bb | pp] at 2C, 3C, 4C
    float * sout;               // layer state out (same layout)
    ActBuf out;                 // Wo's input (CPW = 32: emitted as Q8 blocks)
    float * y;                  // Wo's input as fp32 (CPW < 32: Wo quantizes it in its prologue)
    int img;                    // LDS bytes per activation image (16-aligned)
    // Wo fused (WO): the producers publish their channels' outputs as tagged granules; the Wo
    // workgroups after them gather all C, quantize them (the Wo prologue's arithmetic) and run
    // A4_WOR Wo rows per wave
    DMat wo;
    float * xres;
    unsigned long long * ygran;
    unsigned ytag;
    unsigned * err;
    unsigned spin_max;
    // EMB (layer 0, Wo fused): x = LN0(emb[*tok]) -- the producers' image waves normalise the
    // embedding row (k_embed_ln's loads, chunk sums in chunk order, ln_apply: the same bits) through
    // one more barrier, and each Wo wave computes its rows' x itself; the Wo rows store x + Wo . y
    const uint32_t * tok;
    DMat emb;
    const float * ln0w, * ln0b;
};

typedef __attribute__((address_space(1))) unsigned long long a4_gu64_t;

// 8 consecutive embedding elements k .. k + 7 (clamped to the row) as fp32
__device__ __forceinline__ void a4_emb8(float (&v)[8], const DMat & emb, size_t tok, int k, int C) {
    k = min(k, C - 8);
    if (emb.type == W_F16) {
        const int4 raw = *(const int4 *)((const __half *)emb.qs + tok * C + k);
        const __half * h = (const __half *)&raw;
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = __half2float(h[j]);
    } else {
        ln_load8(v, (const float *)emb.qs + tok * C, k, C);
    }
}
typedef __attribute__((address_space(1))) unsigned a4_gu32_t;

// 512 threads = 8 waves, CPW channels per workgroup.  Waves 4..7 build the three images (LayerNorm
// statistics in the chunk association, one 512-element chunk per wave, token shift per mix,
// quantization); every wave dots rows R w .. R w + R - 1 (R = CPW / 8) of each matrix within the
// workgroup's channels; wave 0 (CPW lanes) runs the recurrence.  CPW = 32 emits Wo's input as one
// Q8 block; smaller CPW (more workgroups streaming the rows) write it as fp32.
constexpr int A4_WOR = 2;  // Wo rows per wave of a Wo workgroup (8 waves: 16 rows)
template <int WF, int U, int CPW, bool WO = false, bool EMB = false>
__global__ __launch_bounds__(512) void k_v4_att_fused(Att4Fused a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float sr[CPW], sk[CPW], sv[CPW];
    constexpr int R = CPW / 8, LCW = 1;
    const int C = a.C, K = C, c0 = blockIdx.x * CPW;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    const int units = mv_units(WF, K);
    if constexpr (WO) {
        if ((int)blockIdx.x >= C / CPW) {
            // ---- a Wo workgroup (rwkv_graph.inc:171-175, x += Wo . y): A4_WOR rows per wave,
            // their first U units loaded now; every wave gathers y once the producers publish it
            STAMP_BEGIN();
            const int row0 = (((int)blockIdx.x - C / CPW) * 8 + wave) * A4_WOR;
            WBlk wo[A4_WOR][U];
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int r = 0; r < A4_WOR; r++) wo[r][u] = load_unit<WF>(a.wo, min(row0 + r, C - 1), u, lane);
            float xr;
            if constexpr (EMB) {
                // this layer's input x = LN0(emb[token]): the row's statistics in this wave's registers
                const size_t tk = *a.tok;
                const int nc = (C + LN_CHUNK - 1) / LN_CHUNK;
                float ev[4][8];
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    if (c < nc) a4_emb8(ev[c], a.emb, tk, c * LN_CHUNK + lane * 8, C);
                    else
#pragma unroll
                        for (int j = 0; j < 8; j++) ev[c][j] = 0.0f;
                }
                float m0, sc0;
                ln_stats_regs<4>(ev, nc, C, 1e-5f, m0, sc0);
                const int rr = min(row0 + min(lane, A4_WOR - 1), C - 1);
                const float e = a.emb.type == W_F16 ? __half2float(((const __half *)a.emb.qs)[tk * C + rr])
                                                    : ((const float *)a.emb.qs)[tk * C + rr];
                xr = ln_apply(e, m0, sc0, a.ln0w[rr], a.ln0b[rr]);
            } else {
                xr = a.xres[min(row0 + min(lane, A4_WOR - 1), C - 1)];
            }
            const ActBuf xq = lds_act(smem, act_fmt_for(WF), K);
            gran_gather_image<WF>(a.ygran, a.ytag, C, xq, wave, 8, a.err, a.spin_max, lane);
            __syncthreads();
            float acc[A4_WOR], acc2[A4_WOR];
#pragma unroll
            for (int r = 0; r < A4_WOR; r++) acc[r] = acc2[r] = 0.0f;
            for (int u0 = 0; u0 < units; u0 += U) {
                if (u0 > 0) {
#pragma unroll
                    for (int u = 0; u < U; u++)
#pragma unroll
                        for (int r = 0; r < A4_WOR; r++) wo[r][u] = load_unit<WF>(a.wo, min(row0 + r, C - 1), u0 + u, lane);
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const AUnit xu = load_act_unit<WF, true>(xq, u0 + u, lane);
                    if (unit_valid<WF>(K, u0 + u, lane)) {
#pragma unroll
                        for (int r = 0; r < A4_WOR; r++) dot_unit<WF>(wo[r][u], xu, acc[r], acc2[r]);
                    }
                }
            }
            float s[A4_WOR];
#pragma unroll
            for (int r = 0; r < A4_WOR; r++) s[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
            const float v = lane_row_sum<A4_WOR>(s, lane);
            if (lane < A4_WOR && row0 + lane < C) a.xres[row0 + lane] = xr + v;  // EPI_ADD
            STAMP_END_NS(8);
            return;
        }
    }
    const bool pro = wave >= 4;
    const int pw = wave - 4, nch = (K + LN_CHUNK - 1) / LN_CHUNK;
    STAMP_BEGIN();
    const ActBuf ao = a.out;
    pin_act(ao);
    MVEntry E;
    E.x = a.x;
    E.carry = a.carry;
    E.lnw = a.lnw;
    E.lnb = a.lnb;
    E.mu = a.mix[0];
    E.carry_out = a.carry_out;
    E.f = nullptr;
    // image inputs (chunk pw of x, carry, LN weights, mix r) and mixes k, v: every wave issues
    // the loads without a branch (chunk_load_all), the dot waves' are empty
    ChunkIn ci[LCW];
    float mk[8], mv[8];
    const int kc = max(min(pw * LN_CHUNK + lane * 8, K - 8), 0);
    const bool kval = pro && pw * LN_CHUNK + lane * 8 < K;
    chunk_load_all<MVK_LN, 0>(E, kc, ci[0], pro);
    ld8_buf(mk, a.mix[1], kc, pro);
    ld8_buf(mv, a.mix[2], kc, pro);
    asm volatile("" ::"s"(a.W[0].qs), "s"(a.W[1].qs), "s"(a.W[2].qs));
    asm volatile("s_barrier" ::: "memory");  // image inputs issued ahead of the weight stream
    // ---- rows c0 + 4 wave + r of r, k, v (all waves)
    WBlk w[3][R][U];
#pragma unroll
    for (int m = 0; m < 3; m++)
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < R; r++) w[m][r][u] = load_unit<WF>(a.W[m], min(c0 + R * wave + r, C - 1), u, lane);
    // the recurrence's operands (wave 0, lane = channel)
    float aa = 0.0f, bb = 0.0f, pp = 0.0f, fi = 0.0f, de = 0.0f;
    if (wave == 0 && lane < CPW) {
        const int c = min(c0 + lane, C - 1);
        aa = a.sin[2 * C + c];
        bb = a.sin[3 * C + c];
        pp = a.sin[4 * C + c];
        fi = a.first[c];
        de = a.decay[c];
    }
    ActBuf img[3];
#pragma unroll
    for (int m = 0; m < 3; m++) img[m] = lds_act(smem + m * a.img, act_fmt_for(WF), K);
    if (pro) {
        if constexpr (EMB) {
            // x = LN0(emb[token]) for this wave's chunk (k_embed_ln's arithmetic)
            __shared__ double e_part[2][8];
            const size_t tk = *a.tok;
            float w0[8], b0[8];
            ln_load8(w0, a.ln0w, kc, K);
            ln_load8(b0, a.ln0b, kc, K);
            a4_emb8(ci[0].x, a.emb, tk, kc, K);
            if (pw < nch) {
                double c1, c2;
                ln_chunk_sums(ci[0].x, kval, c1, c2);
                if (lane == 0) {
                    e_part[0][pw] = c1;
                    e_part[1][pw] = c2;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // (E) LN0 statistics
            double s1 = 0.0, s2 = 0.0;
            for (int q = 0; q < nch; q++) s1 += e_part[0][q], s2 += e_part[1][q];
            float m0, sc0;
            ln_finish(s1, s2, K, 1e-5f, m0, sc0);
#pragma unroll
            for (int j = 0; j < 8; j++) ci[0].x[j] = ln_apply(ci[0].x[j], m0, sc0, w0[j], b0[j]);
        }
        // LayerNorm statistics (chunk association, one pass); the chunk sums meet in LDS
        __shared__ double ln_part[2][8];
        if (pw < nch) {
            double c1, c2;
            ln_chunk_sums(ci[0].x, kval, c1, c2);
            if (lane == 0) {
                ln_part[0][pw] = c1;
                ln_part[1][pw] = c2;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        double s1 = 0.0, s2 = 0.0;
        for (int q = 0; q < nch; q++) s1 += ln_part[0][q], s2 += ln_part[1][q];
        float mean, scale;
        ln_finish(s1, s2, K, 1e-5f, mean, scale);
        if (pw < nch) {
            const bool wc = blockIdx.x == 0;
            chunk_store<WF, MVK_LN, 0>(E, img[0], ci[0], mean, scale, wc, kc, kval, lane);
#pragma unroll
            for (int j = 0; j < 8; j++) ci[0].m[j] = mk[j];
            chunk_store<WF, MVK_LN, 0>(E, img[1], ci[0], mean, scale, false, kc, kval, lane);
#pragma unroll
            for (int j = 0; j < 8; j++) ci[0].m[j] = mv[j];
            chunk_store<WF, MVK_LN, 0>(E, img[2], ci[0], mean, scale, false, kc, kval, lane);
        }
    } else {
        if constexpr (EMB) asm volatile("s_barrier" ::: "memory");  // (E)
        asm volatile("s_barrier" ::: "memory");  // the image waves' statistics exchange
    }
    __syncthreads();  // (1) images ready
    if (wave == 0) STAMP_MID();
#pragma unroll
    for (int m = 0; m < 3; m++) {
        float acc[R], acc2[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
        for (int u0 = 0; u0 < units; u0 += U) {
            if (u0 > 0) {
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int r = 0; r < R; r++) w[m][r][u] = load_unit<WF>(a.W[m], min(c0 + R * wave + r, C - 1), u0 + u, lane);
            }
            AUnit xu[U];
#pragma unroll
            for (int u = 0; u < U; u++) xu[u] = load_act_unit<WF, true>(img[m], u0 + u, lane);
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (unit_valid<WF>(K, u0 + u, lane)) {
#pragma unroll
                    for (int r = 0; r < R; r++) dot_unit<WF>(w[m][r][u], xu[u], acc[r], acc2[r]);
                }
            }
        }
        float s[R];
#pragma unroll
        for (int r = 0; r < R; r++) s[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
        const float v = lane_row_sum<R>(s, lane);  // lane r: row R wave + r
        float * dst = m == 0 ? sr : m == 1 ? sk : sv;
        if (lane < R) dst[R * wave + lane] = m == 0 ? sigmoidf_(v) : v;  // r: EPI_SIGMOID
    }
    __syncthreads();  // (2) r, k, v of the workgroup's channels ready
    if (wave == 0) {
        STAMP_X(0);
        if (lane < CPW) {
            // k_wkv4's arithmetic, in its order
            const int c = c0 + lane;
            const float kt = sk[lane], vt = sv[lane];
            float ww = fi + kt;
            float qq = fmaxf(pp, ww);
            float e1 = rk_expf(pp - qq), e2 = rk_expf(ww - qq);
            const float an = e1 * aa + e2 * vt;
            const float bn = e1 * bb + e2;
            ww = pp + de;
            qq = fmaxf(ww, kt);
            e1 = rk_expf(ww - qq);
            e2 = rk_expf(kt - qq);
            aa = e1 * aa + e2 * vt;
            bb = e1 * bb + e2;
            pp = qq;
            const float y = sr[lane] * (an / bn);
            if constexpr (WO)
                __hip_atomic_store((a4_gu64_t *)(a.ygran + c), ((unsigned long long)a.ytag << 32) | __float_as_uint(y),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if constexpr (CPW == 32) emit32(ao, 0, c, y);  // lanes 0..31: one quantization block
            else a.y[c] = y;
            if (c < C) {
                a.sout[2 * C + c] = aa;
                a.sout[3 * C + c] = bb;
                a.sout[4 * C + c] = pp;
            }
        }
    }
    STAMP_END(8);
}

// 8 channels per workgroup (96 workgroups for C = 768: 16 / 32 channels, fewer and longer-streaming
// workgroups, measured 269.6 / 285.1 against 256.6 us per v4-169M token)
bool v4_att_fused_supported(int C, const DMat & Wr, const DMat & Wk, const DMat & Wv, const ActBuf & out) {
    (void)out;
    if (C % 32 || C > 2048) return false;
    const int t = Wr.type;
    if (t < 0 || Wk.type != t || Wv.type != t || mv_units(t, C) > 2) return false;
    for (const DMat * W : {&Wr, &Wk, &Wv})
        if ((int)W->M != C || (int)W->K != C) return false;
    return true;
}

template <int WF>
static void launch_att4_t(hipStream_t st, const Att4Fused & a, int units) {
    const int lds = 3 * a.img;
    if (a.wo.qs) {
        // the producers, then the Wo workgroups (16 rows each)
        const dim3 grid(a.C / 8 + (a.C + 8 * A4_WOR - 1) / (8 * A4_WOR));
        if (a.tok) {
            if (units <= 1) RK_LAUNCH((k_v4_att_fused<WF, 1, 8, true, true>), grid, dim3(512), lds, st, a);
            else RK_LAUNCH((k_v4_att_fused<WF, 2, 8, true, true>), grid, dim3(512), lds, st, a);
            return;
        }
        if (units <= 1) RK_LAUNCH((k_v4_att_fused<WF, 1, 8, true>), grid, dim3(512), lds, st, a);
        else RK_LAUNCH((k_v4_att_fused<WF, 2, 8, true>), grid, dim3(512), lds, st, a);
        return;
    }
    if (units <= 1) RK_LAUNCH((k_v4_att_fused<WF, 1, 8>), dim3(a.C / 8), dim3(512), lds, st, a);
    else RK_LAUNCH((k_v4_att_fused<WF, 2, 8>), dim3(a.C / 8), dim3(512), lds, st, a);
}

bool launch_v4_att_fused(hipStream_t st, int C, const DMat & Wr, const DMat & Wk, const DMat & Wv, const float * x,
                         const float * carry, float * carry_out, const float * lnw, const float * lnb,
                         const float * mix_r, const float * mix_k, const float * mix_v, const float * first,
                         const float * decay, const float * sin, float * sout, const ActBuf & out, float * y,
                         const V4WoFused * wf) {
    if (wf && (wf->wo.type != Wr.type || wf->wo.M != C || wf->wo.K != C || C % 8)) {
        fprintf(stderr, "rwkv: fused v4 attention + Wo decode: unsupported shape (C %d)\n", C);
        return false;
    }
    if (!v4_att_fused_supported(C, Wr, Wk, Wv, out)) {
        fprintf(stderr, "rwkv: fused v4 attention decode: unsupported shape (C %d)\n", C);
        return false;
    }
    Att4Fused a;
    memset(&a, 0, sizeof(a));
    a.C = C;
    a.W[0] = Wr;
    a.W[1] = Wk;
    a.W[2] = Wv;
    a.x = x;
    a.carry = carry;
    a.carry_out = carry_out;
    a.lnw = lnw;
    a.lnb = lnb;
    a.mix[0] = mix_r;
    a.mix[1] = mix_k;
    a.mix[2] = mix_v;
    a.first = first;
    a.decay = decay;
    a.sin = sin;
    a.sout = sout;
    a.out = out;
    a.y = y;
    if (wf) {
        a.wo = wf->wo;
        a.xres = wf->xres;
        a.ygran = wf->ygran;
        a.ytag = wf->ytag;
        a.err = wf->err;
        a.spin_max = wf->spin_max;
        if (wf->tok) {
            if ((wf->emb.type != W_F16 && wf->emb.type != W_F32) || (int)wf->emb.K != C || !wf->ln0w || !wf->ln0b) {
                fprintf(stderr, "rwkv: fused v4 attention with the embedding: unsupported embedding\n");
                return false;
            }
            a.tok = wf->tok;
            a.emb = wf->emb;
            a.ln0w = wf->ln0w;
            a.ln0b = wf->ln0b;
        }
    }
    a.img = (lds_bytes_for(act_fmt_for(Wr.type), C) + 15) & ~15;
    const int units = mv_units(Wr.type, C);
    switch (Wr.type) {
        case W_F32: launch_att4_t<W_F32>(st, a, units); break;
        case W_F16: launch_att4_t<W_F16>(st, a, units); break;
        case W_Q4_0: launch_att4_t<W_Q4_0>(st, a, units); break;
        case W_Q4_1: launch_att4_t<W_Q4_1>(st, a, units); break;
        case W_Q5_0: launch_att4_t<W_Q5_0>(st, a, units); break;
        case W_Q5_1: launch_att4_t<W_Q5_1>(st, a, units); break;
        case W_Q8_0: launch_att4_t<W_Q8_0>(st, a, units); break;
        default: return false;
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
