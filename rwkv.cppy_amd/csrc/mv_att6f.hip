// mv_att6f.hip -- v6 decode: the r, k, v, g and decay-LoRA-first-stage matvecs and the per-head
// attention core (rwkv_graph.inc:349-384) in ONE launch.
//
// Before: k_mva over the 4*C + D rows (one launch), then k_att6_dec (one workgroup per head, a
// second launch that waits at the kernel boundary for every row although head h reads only its
// own 64 channels of r, k, v, g -- plus the D decay-LoRA values every head shares).  Here the
// grid is 8 workgroups per head: workgroup (h, s) computes 32 of head h's 256 r/k/v/g rows (4
// waves x 8 rows, exactly k_mva's lane/unit order, wave_sum63 tree and epilogues, so the values
// are bit-identical) and, on a fifth wave, the decay-LoRA rows of its slot.  Every row is
// published as a granule (value + tag in one 8-byte write-through store, below); a decay-LoRA
// value once per head, so each head owns its copy.  The head's reducer -- which loads the head's
// state, decay-tail weights and per-channel operands at kernel start -- sweeps its head's granules
// and runs k_att6_dec's arithmetic (decay tail, wkv6, GroupNorm, gate, Q8 emission of Wo's
// input).  Each granule has exactly one reader, which clears it right after reading: no
// counters, no atomics, and a replayed graph needs no memset node.
//
// Progress without co-residency.  The grid is ordered so that every waiting workgroup waits only
// on workgroups of LOWER index: [0, 8H) the producers -- workgroup b is (h = b % H, s = b / H) and
// owns decay-LoRA slots b, b + 8H, ... --, [8H, 9H) the reducers (no rows of their own: a reducer
// dispatched last must not hold back its head's rows), [9H, 9H + C / (4 WOR)) the Wo workgroups
// (fused Wo: each gathers every head's outputs and runs 4 WOR rows of Wo).  Producers
// never wait, so however few workgroups are resident (several contexts decoding on one GPU at
// once), the lowest-index waiting workgroup's producers have all been dispatched: the launch
// drains.  Every spin is also bounded: a timeout sets *err (a host-mapped word) and the engine
// fails the evaluation that synchronises next, then clears every granule (a late producer may
// have left one tagged) -- never a hang, never a silently wrong result.
//
// The state update uses 16-byte accesses: wave g owns keys 16g..16g+15, lane (kk, jq) keys
// 16g + 4kk + q (q < 4) of value columns 4jq..4jq+3.  Each output column's sum keeps
// k_att6_dec's association: ((t0 + t1) + t2) + t3 per 4-key run (from +0), (p0 + p1) + (p2 + p3)
// per 16-key group, (s0 + s2) + (s1 + s3) over the groups.
#include "mv_att6.hpp"

#include <stdlib.h>

#include <algorithm>

namespace rwkvmi {

// WOR: Wo rows per wave of a Wo workgroup (4 waves: 4 WOR rows); 0 = no Wo in this launch
template <int WF, int U, int WD, int WOR>
__global__ __launch_bounds__(320) void k_v6_att_fused(Att6Fused a) {
    constexpr bool WO = WOR > 0;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // Q8 image of dl (decay tail input)
    __shared__ __attribute__((aligned(16))) float sr[64], sk[64], sv[64], sg[64], sw[64], su[64];
    __shared__ __attribute__((aligned(16))) float part[16][64];
    constexpr int S = 64;
    const int wg = (int)blockIdx.x, H = a.H, C = a.C, D = a.D;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform branches
    const int NP = AF_P * H;  // producer workgroups; then H reducers, then the Wo workgroups
    if constexpr (WO) {
        if (wg >= NP + H) {
            // ---- a Wo workgroup (rwkv_graph.inc:382-384, x += Wo . y): waves 0..3 own WOR rows each,
            // loaded now; all 5 waves gather y when the reducers publish it (wo_prepoll: after wave 0
            // has seen one granule per head -- each head's 64 outputs are one store instruction)
            STAMP_BEGIN();
            constexpr int AF_WOR = WOR > 0 ? WOR : 1;
            const int row0 = ((wg - NP - H) * 4 + min(wave, 3)) * AF_WOR;
            WBlk wo[AF_WOR][U];
            float xr = 0.0f;
            if (wave < 4) {
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int r = 0; r < AF_WOR; r++) wo[r][u] = load_unit<WF>(a.wo, min(row0 + r, C - 1), u, lane);
                xr = a.xres[min(row0 + min(lane, AF_WOR - 1), C - 1)];
            }
            // y arrives as Q8 blocks (pub_q8 in the reducers: the bits Wo's fp32-input prologue
            // would produce), KG_STRIDE granules per 32 outputs
            const ActBuf xq = lds_act(smem, act_fmt_for(WF), C);
            const int nb = C >> 5;
            if (a.wo_prepoll) {
                if (wave == 0) {
                    for (int b0 = 0; b0 < nb; b0 += 64)
                        gran_prepoll(a.ygran + (size_t)b0 * KG_STRIDE, min(64, nb - b0), KG_STRIDE, 8, a.ytag, a.err,
                                     a.spin_max, lane);
                    STAMP_XN(2);
                }
                __syncthreads();
            }
            q8_gather_image<(U > 1 ? 4 : 2)>(a.ygran, nb, a.ytag, xq, threadIdx.x, 320, a.err, a.spin_max);
            __syncthreads();
            q8_image_qsum(xq, nb, threadIdx.x, 320);
            __syncthreads();
            if (wave == 0) STAMP_XN(3);
            if (wave < 4) {
                const float s = rows_dot_img<WF, AF_WOR, U>(wo, xq, C, lane);
                if (lane < AF_WOR && row0 + lane < C) a.xres[row0 + lane] = xr + s;  // EPI_ADD
            }
            STAMP_END_NS(6);
            return;
        }
    }
    // [0, 8H): producers (h = b % H, s = b / H; decay-LoRA slots b, b + 8H, ...); [8H, 9H): the
    // reducers, which produce nothing themselves
    const bool red = wg >= NP;
    const int h = red ? wg - NP : wg % H, sidx = red ? 0 : wg / H;
    const int c0 = h * S;
    const Att6Dec & at = a.att;
    const size_t hb = (size_t)h * S * S;
    const int jq = lane & 15, kk = lane >> 4;
    unsigned long long * const gdl = a.gran + 4 * (size_t)C;
    STAMP_BEGIN();
    // the reducer's late scalars (Wo input record, hand-off words, eps) in SGPRs now
    const ActBuf yq = at.yq;
    unsigned * const err = a.err;
    const unsigned spin_max = a.spin_max;
    const float eps = at.eps;
    if (red) {
        pin_act(yq);
        asm volatile("" ::"s"(err), "s"(eps), "s"(spin_max));
    }
    const bool publish = wg != a.skip_wg;  // test hook (Engine debug knob "skip_granule")
    // ---- the reducer's head operands first (state rows, per-channel vectors, decay-tail weights):
    // they stream in with this workgroup's own weight rows
    float4 st[4];
    WBlk wp[4];
    float lnw_c = 0.0f, lnb_c = 0.0f, dec_c = 0.0f, u_c = 0.0f;
    if (red) {
        if (wave < 4) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                st[q] = *(const float4 *)(at.sin + hb + (size_t)(16 * wave + 4 * kk + q) * S + 4 * jq);
        }
        if (wave == 0) {
            lnw_c = at.lnx_w[c0 + lane];
            lnb_c = at.lnx_b[c0 + lane];
            u_c = at.u[c0 + lane];
        }
        if (wave == 4) {
            dec_c = at.decay[c0 + lane];
            const int nb = at.wd2.K >> 5;
#pragma unroll
            for (int l = 0; l < 4; l++) wp[l] = load_wblk<WD>(at.wd2, (size_t)(c0 + lane) * nb + min(l, nb - 1));
        }
    }
    // ---- a producer's rows, each published as a granule: wave w -> matrix (4 s + w) / 8 (r, k, v,
    // g), rows of head h; wave 4 -> decay LoRA rows (EPI_TANH) of its slots wg, wg + 8H, ...
    if (red) {
    } else if (wave < 4) {
        const int wh = sidx * 4 + wave, m = wh >> 3, row0 = c0 + (wh & 7) * AF_R;
        const DMat W = m == 0 ? a.W[0] : m == 1 ? a.W[1] : m == 2 ? a.W[2] : a.W[3];
        const ActBuf x = m == 0 ? a.x[0] : m == 1 ? a.x[1] : m == 2 ? a.x[2] : a.x[3];
        const float v = af_rows<WF, AF_R, U>(W, x, row0, m == 3 ? EPI_SILU : EPI_STORE, lane);
        if (lane < AF_R && publish) gran_put(a.gran + (size_t)m * C + row0 + lane, v);
    } else {
        for (int d = wg; d < D; d += NP) {
            const float v = af_rows<WF, 1, U>(a.wd1, a.xw, d, EPI_TANH, lane);  // in lane 0
            const float v0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
            if (lane < H && publish) gran_put(gdl + (size_t)lane * D + d, v0);  // one copy per head
        }
    }
    if (!red) {
        STAMP_END_NS(6);
        return;
    }
    // ---- reducer.  Waves 0..3 sweep r, k, v, g of the head's channels (lane = channel); wave 4
    // sweeps the decay LoRA values and runs the decay tail (k_att6_dec's arithmetic) meanwhile.
    if (wave < 4) {
        unsigned long long * g = a.gran + (size_t)wave * C + c0 + lane;
        bool live[1] = {true};
        float v[1];
        gran_sweep<1>(g, 0, live, v, err, spin_max);
        float * dst = wave == 0 ? sr : wave == 1 ? sk : wave == 2 ? sv : sg;
        dst[lane] = v[0];
        gran_clear(g);
        if (wave == 0) {
            su[lane] = u_c;
            STAMP_MID();
        }
    } else {
        bool live[2] = {lane < D, lane + 64 < D};
        float v[2];
        unsigned long long * const own = gdl + (size_t)h * D + lane;  // this head's copy
        gran_sweep<2>(own, 64, live, v, err, spin_max);
        if (live[0]) gran_clear(own);
        if (live[1]) gran_clear(own + 64);
        const ActBuf act = lds_act(smem, act_fmt_for(WD), D);
        if (lane < D) emit32(act, 0, lane, v[0]);  // lanes 0..31 / 32..63: whole quantization blocks
        if (lane + 64 < D) emit32(act, 0, lane + 64, v[1]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        // decay tail of channel c0 + lane: w = exp(-exp(Wd2 . dl + decay)), rwkv_graph.inc:357-367
        const float s = decay_row_thread<WD, 4, 4>(at.wd2, c0 + lane, act, at.wd2.K >> 5, wp);
        sw[lane] = rk_expf(-rk_expf(s + dec_c));
    }
    __syncthreads();
    STAMP_X(0);
    // wkv6 (ggml_rwkv_wkv6): keys 16 wave + 4 kk + q, value columns 4 jq + c
    if (wave < 4) {
        const int i0 = 16 * wave + 4 * kk;
        const float4 k4 = *(const float4 *)(sk + i0), u4 = *(const float4 *)(su + i0);
        const float4 r4 = *(const float4 *)(sr + i0), w4 = *(const float4 *)(sw + i0);
        const float4 v4 = *(const float4 *)(sv + 4 * jq);
        const float kq[4] = {k4.x, k4.y, k4.z, k4.w}, uq[4] = {u4.x, u4.y, u4.z, u4.w};
        const float rq[4] = {r4.x, r4.y, r4.z, r4.w}, wq[4] = {w4.x, w4.y, w4.z, w4.w};
        const float vj[4] = {v4.x, v4.y, v4.z, v4.w};
        float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float prev[4] = {st[q].x, st[q].y, st[q].z, st[q].w};
            float nw[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const float kv = vj[c] * kq[q];
                const float temp = kv * uq[q] + prev[c];
                const float t = temp * rq[q];
                p[c] += t;
                nw[c] = prev[c] * wq[q] + kv;
            }
            *(float4 *)(at.sout + hb + (size_t)(i0 + q) * S + 4 * jq) = make_float4(nw[0], nw[1], nw[2], nw[3]);
        }
        *(float4 *)&part[4 * wave + kk][4 * jq] = make_float4(p[0], p[1], p[2], p[3]);
    }
    __syncthreads();
    STAMP_X(1);
    // GroupNorm over the head (ggml_norm, fp64 sums) * ln_x + b, * g; emitted as Wo's input
    if (wave == 0) {
        float sgp[4];
#pragma unroll
        for (int gg = 0; gg < 4; gg++)
            sgp[gg] = (part[4 * gg][lane] + part[4 * gg + 1][lane]) + (part[4 * gg + 2][lane] + part[4 * gg + 3][lane]);
        const float x = (sgp[0] + sgp[2]) + (sgp[1] + sgp[3]);
        const double s = group_tree_sum_d((double)x, S);
        const float mean = (float)div_count(s, S);
        const float d = x - mean;
        const double s2 = group_tree_sum_d((double)(d * d), S);
        const float var = (float)div_count(s2, S);
        const float scale = 1.0f / sqrtf(var + eps);
        float o = d * scale;
        o = o * lnw_c;
        o = o + lnb_c;
        o = o * sg[lane];
        if constexpr (WO) pub_q8(a.ygran, (c0 >> 5) + (lane >> 5), o, a.ytag, lane);  // the head's 2 blocks
        else emit32(yq, 0, c0 + lane, o);
    }
    STAMP_END(6);
}

bool v6_att_fused_supported(const Att6Fused & a) {
    if (a.att.S != 64 || a.C != a.H * 64 || a.att.w || a.att.yq.fmt < 0 || a.att.yq.tiled) return false;
    if (!a.gran) return false;
    const int t = a.W[0].type;
    if (!wtype_quantized(t) || a.wd1.type != t || mv_units(t, a.C) > 2) return false;
    for (int m = 0; m < 4; m++)
        if (a.W[m].type != t || a.W[m].M != a.C || a.W[m].K != a.C || a.x[m].fmt != act_fmt_for(t) || a.x[m].K != a.C)
            return false;
    if (a.wd1.M != a.D || a.wd1.K != a.C || a.xw.fmt != act_fmt_for(t) || a.xw.K != a.C) return false;
    if (!wtype_quantized(a.att.wd2.type) || a.att.wd2.M != a.C || a.att.wd2.K != a.D) return false;
    // the decay tail's PF = 4 units per row and one emission half-wave per 32 decay rows
    if (a.D % 32 || a.D > 128) return false;  // two granules per lane of the sweeping wave
    if (a.wo.qs) {
        // Wo fused: C x C of the same type, rows spread over the 28 H non-reducer waves
        if (a.wo.type != t || a.wo.M != a.C || a.wo.K != a.C || !a.xres || !a.ygran || a.C % 32) return false;
        if (a.wo_rows != 4 && a.wo_rows != 8) return false;
    }
    return a.H <= 64 && a.err;  // one decay-value copy per head: a lane per head
}

template <int WF, int U, int WO>
static void launch_af_wd(hipStream_t st, const Att6Fused & a, int lds) {
    const dim3 grid(AF_P * a.H + a.H + (WO ? a.C / (4 * WO) : 0)), block(320);
    switch (a.att.wd2.type) {
        case W_Q4_0: RK_LAUNCH((k_v6_att_fused<WF, U, W_Q4_0, WO>), grid, block, lds, st, a); break;
        case W_Q4_1: RK_LAUNCH((k_v6_att_fused<WF, U, W_Q4_1, WO>), grid, block, lds, st, a); break;
        case W_Q5_0: RK_LAUNCH((k_v6_att_fused<WF, U, W_Q5_0, WO>), grid, block, lds, st, a); break;
        case W_Q5_1: RK_LAUNCH((k_v6_att_fused<WF, U, W_Q5_1, WO>), grid, block, lds, st, a); break;
        default: RK_LAUNCH((k_v6_att_fused<WF, U, W_Q8_0, WO>), grid, block, lds, st, a); break;
    }
}

bool launch_v6_att_fused(hipStream_t st, const Att6Fused & a) {
    if (!v6_att_fused_supported(a)) {
        fprintf(stderr, "rwkv: fused v6 attention decode: unsupported shape\n");
        return false;
    }
    const bool wo = a.wo.qs != nullptr;
    int lds = lds_bytes_for(act_fmt_for(a.att.wd2.type), a.D);
    if (wo) lds = std::max(lds, lds_bytes_for(act_fmt_for(a.W[0].type), a.C));
    const bool u1 = mv_units(a.W[0].type, a.C) <= 1;
    const bool r4 = a.wo_rows == 4;
#define AF_T(WFv)                                                  \
    do {                                                           \
        if (wo && u1 && r4) launch_af_wd<WFv, 1, 4>(st, a, lds);   \
        else if (wo && u1) launch_af_wd<WFv, 1, 8>(st, a, lds);    \
        else if (wo && r4) launch_af_wd<WFv, 2, 4>(st, a, lds);    \
        else if (wo) launch_af_wd<WFv, 2, 8>(st, a, lds);          \
        else if (u1) launch_af_wd<WFv, 1, 0>(st, a, lds);          \
        else launch_af_wd<WFv, 2, 0>(st, a, lds);                  \
    } while (0)
    switch (a.W[0].type) {
        case W_Q4_0: AF_T(W_Q4_0); break;
        case W_Q4_1: AF_T(W_Q4_1); break;
        case W_Q5_0: AF_T(W_Q5_0); break;
        case W_Q5_1: AF_T(W_Q5_1); break;
        default: AF_T(W_Q8_0); break;
    }
#undef AF_T
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
