// mv_att6c.hip -- v6 decode attention launch, CO-RESIDENT layout (rwkv_graph.inc:349-384): the
// r, k, v, g and decay-LoRA-first-stage rows, the per-head attention core and the output
// projection Wo in one launch of 8 H workgroups -- the same bits as mv_att6f.hip's ordered layout.
//
// Workgroup (h, s) = blockIdx h * 8 + s computes 32 of head h's 256 r / k / v / g rows (4 waves x 8
// rows, k_mva's lane/unit order, wave_sum63 tree and epilogues) and, on a fifth wave, the
// decay-LoRA rows of its slot, each published as a single-reader granule (mv_att6.hpp).  (h, 0) --
// which loads the head's state, decay-tail weights and per-channel operands while its own rows
// stream -- sweeps its head's granules and runs k_att6_dec's arithmetic (decay tail, wkv6,
// GroupNorm, gate), publishing the head's 64 outputs y as two Q8 blocks of granules tagged (layer,
// state parity) -- pub_q8: the bits Wo's fp32-input prologue would produce.  The 7 H other
// workgroups then own Wo: wave gw's rows gw, gw + 28 H, gw + 56 H, whose units it loaded at kernel
// start; it waits for every head's y, gathers the blocks into LDS and adds its rows' dots to x.
//
// Every workgroup waits on workgroups of both lower and higher index, so this layout needs all
// 8 H workgroups resident at once.  One context alone on an idle device has that (8 H <= the 256
// compute units, one workgroup each -- v6_att_co_supported); the engine uses this layout only
// while no other context of the process has work queued on the device (Engine::co_mode) and
// falls back to the ordered layout for good after a hand-off timeout (another process's launches
// holding the compute units).  Bounded spins as in mv_att6f.hip: a timeout sets *err, never a hang.
//
// Measured against the ordered layout (v6-1B6, one context): 665.6 vs 694.7 us/token -- 96 fewer
// workgroups and the Wo rows spread 3 per wave over 224 workgroups instead of 8 per wave over 64.
// y as Q8 blocks instead of fp32 granules (a third of the gather traffic over 224 gatherers, no
// quantization in them): 655.6-656.7 vs 667.1-669.3 us/token.
#include "mv_att6.hpp"

#include <algorithm>

namespace rwkvmi {

__device__ __forceinline__ int af_slot(int sidx, int h, int H) { return sidx > 0 ? (sidx - 1) * H + h : (AF_P - 1) * H + h; }

constexpr int AF_WOR = 3;  // Wo rows per non-reducer wave: ceil(C / (28 H)) with C = 64 H

template <int WF, int U, int WD>
__global__ __launch_bounds__(320) void k_v6_att_co(Att6Fused a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];  // Q8 image of dl (decay tail input)
    __shared__ __attribute__((aligned(16))) float sr[64], sk[64], sv[64], sg[64], sw[64], su[64];
    __shared__ __attribute__((aligned(16))) float part[16][64];
    constexpr int S = 64;
    const int wg = (int)blockIdx.x, h = wg / AF_P, sidx = wg % AF_P, H = a.H, C = a.C, D = a.D;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform branches
    const bool red = sidx == 0;
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
    // ---- this workgroup's rows, each published as a granule: wave w -> matrix (4 s + w) / 8
    // (r, k, v, g), rows of head h; wave 4 -> decay LoRA rows (EPI_TANH) of its slot, the
    // non-reducer workgroups' slots first (slot = (s - 1) H + h for s > 0, 7H + h for the reducers)
    if (wave < 4) {
        const int wh = sidx * 4 + wave, m = wh >> 3, row0 = c0 + (wh & 7) * AF_R;
        const DMat W = m == 0 ? a.W[0] : m == 1 ? a.W[1] : m == 2 ? a.W[2] : a.W[3];
        const ActBuf x = m == 0 ? a.x[0] : m == 1 ? a.x[1] : m == 2 ? a.x[2] : a.x[3];
        const float v = af_rows<WF, AF_R, U>(W, x, row0, m == 3 ? EPI_SILU : EPI_STORE, lane);
        if (lane < AF_R && publish) gran_put(a.gran + (size_t)m * C + row0 + lane, v);
    } else {
        for (int d = af_slot(sidx, h, H); d < D; d += AF_P * H) {
            const float v = af_rows<WF, 1, U>(a.wd1, a.xw, d, EPI_TANH, lane);  // in lane 0
            const float v0 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
            if (lane < H && publish) gran_put(gdl + (size_t)lane * D + d, v0);  // one copy per head
        }
    }
    if (!red) {
        // ---- Wo (rwkv_graph.inc:382-384, x += Wo . y) on the 7 H non-reducer workgroups: wave
        // gw owns rows gw, gw + 28 H, gw + 56 H (k_mva's per-row arithmetic does not depend on
        // which wave computes a row).  Its units are loaded now, under the reducers' attention.
        const int nwo = 28 * H, gw = ((sidx - 1) * H + h) * 4 + wave;
        WBlk wo[AF_WOR][U];
        float xr = 0.0f;
        if (wave < 4) {
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int j = 0; j < AF_WOR; j++) wo[j][u] = load_unit<WF>(a.wo, min(gw + nwo * j, C - 1), u, lane);
            xr = a.xres[min(gw + nwo * min(lane, AF_WOR - 1), C - 1)];
        }
        // Wait for every head: wave 0 polls the d granule of every y block (mv_common.hpp
        // gran_prepoll) -- the other waves park at the barrier, so the 7 H waiting workgroups add
        // little traffic beside the reducers' own sweeps; then all five waves gather y's Q8 blocks
        // (pub_q8 in the reducers: the bits Wo's fp32-input prologue would produce) into LDS
        const ActBuf xq = lds_act(smem, act_fmt_for(WF), C);
        const int nb = C >> 5;
        if (wave == 0) {
            for (int b0 = 0; b0 < nb; b0 += 64)
                gran_prepoll(a.ygran + (size_t)b0 * KG_STRIDE, min(64, nb - b0), KG_STRIDE, 8, a.ytag, err, spin_max,
                             lane);
        }
        __syncthreads();
        q8_gather_image<(U > 1 ? 4 : 2)>(a.ygran, nb, a.ytag, xq, tid, 320, err, spin_max);
        __syncthreads();
        q8_image_qsum(xq, nb, tid, 320);
        __syncthreads();
        if (wave < 4) {
            float acc[AF_WOR], acc2[AF_WOR];
#pragma unroll
            for (int j = 0; j < AF_WOR; j++) acc[j] = acc2[j] = 0.0f;
#pragma unroll
            for (int u = 0; u < U; u++) {
                const AUnit xu = load_act_unit<WF, true>(xq, u, lane);
                const bool uv = unit_valid<WF>(C, u, lane);
#pragma unroll
                for (int j = 0; j < AF_WOR; j++) {
                    float t = acc[j], t2 = acc2[j];
                    dot_unit<WF>(wo[j][u], xu, t, t2);
                    acc[j] = uv ? t : acc[j];
                    acc2[j] = uv ? t2 : acc2[j];
                }
            }
            constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
            float sr_[AF_WOR];
#pragma unroll
            for (int j = 0; j < AF_WOR; j++)
                sr_[j] = one ? wave_sum63(acc[j]) + wave_sum63(acc2[j]) : wave_sum63(acc[j]) + 0.0f;
            const float s = lane_row_sum<AF_WOR>(sr_, lane);
            const int row = gw + nwo * lane;
            if (lane < AF_WOR && row < C) a.xres[row] = xr + s;  // EPI_ADD
        }
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
        pub_q8(a.ygran, (c0 >> 5) + (lane >> 5), o, a.ytag, lane);  // the head's 2 blocks
    }
    STAMP_END(6);
}

bool v6_att_co_supported(const Att6Fused & a) {
    // the ordered layout's shapes, Wo fused, rows spread over the 28 H non-reducer waves; and the
    // whole grid resident at one workgroup per CU (the C > 2048 forms hold up to 223 VGPRs: one
    // 5-wave workgroup per CU), so 8 H <= the device's compute units
    if (!v6_att_fused_supported(a) || !a.wo.qs || a.C % 512 || AF_P * a.H > kQgCUs) return false;
    return (a.C + 28 * a.H - 1) / (28 * a.H) <= AF_WOR;
}

template <int WF, int U>
static void launch_co_wd(hipStream_t st, const Att6Fused & a, int lds) {
    const dim3 grid(AF_P * a.H), block(320);
    switch (a.att.wd2.type) {
        case W_Q4_0: RK_LAUNCH((k_v6_att_co<WF, U, W_Q4_0>), grid, block, lds, st, a); break;
        case W_Q4_1: RK_LAUNCH((k_v6_att_co<WF, U, W_Q4_1>), grid, block, lds, st, a); break;
        case W_Q5_0: RK_LAUNCH((k_v6_att_co<WF, U, W_Q5_0>), grid, block, lds, st, a); break;
        case W_Q5_1: RK_LAUNCH((k_v6_att_co<WF, U, W_Q5_1>), grid, block, lds, st, a); break;
        default: RK_LAUNCH((k_v6_att_co<WF, U, W_Q8_0>), grid, block, lds, st, a); break;
    }
}

bool launch_v6_att_co(hipStream_t st, const Att6Fused & a) {
    if (!v6_att_co_supported(a)) {
        fprintf(stderr, "rwkv: co-resident v6 attention decode: unsupported shape\n");
        return false;
    }
    const int lds = std::max(lds_bytes_for(act_fmt_for(a.att.wd2.type), a.D), lds_bytes_for(act_fmt_for(a.W[0].type), a.C));
    const bool u1 = mv_units(a.W[0].type, a.C) <= 1;
#define AC_T(WFv)                                   \
    do {                                            \
        if (u1) launch_co_wd<WFv, 1>(st, a, lds);   \
        else launch_co_wd<WFv, 2>(st, a, lds);      \
    } while (0)
    switch (a.W[0].type) {
        case W_Q4_0: AC_T(W_Q4_0); break;
        case W_Q4_1: AC_T(W_Q4_1); break;
        case W_Q5_0: AC_T(W_Q5_0); break;
        case W_Q5_1: AC_T(W_Q5_1); break;
        default: AC_T(W_Q8_0); break;
    }
#undef AC_T
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
