// mv_sigmaa.hip -- v6 decode: layer l's channel-mix value + receptance rows (k_mvsig's work,
// rwkv_graph.inc:513-531) and layer l + 1's maa LoRA (k_v6_maa_dec4's work, rwkv_graph.inc:306-346)
// in ONE launch, the co-resident form (Engine::co_mode only).
//
// Before: k_mvsig (x += sigmoid(Wr . xr) * (Wv . k)), a kernel boundary, then the next layer's maa
// launch re-reads x for its LayerNorm.  Here workgroup b (512 threads, one row per wave) computes
// rows 8 b .. 8 b + 7 of x exactly as k_mvsig does (k_mva's lane/unit order and wave_sum63 tree per
// product, EPI_SIGMUL_ADD), stores them and publishes each as a granule {tag, value} (one 8-byte
// agent-scope store); workgroups [0, 5 C / 64) then run the maa workgroup (mv_maa.hpp) with x
// gathered from those granules -- its W1 rows and W2 columns stream while the last rows of x arrive.
// The bits equal the k_mvsig + k_v6_maa_dec4 pair.  The maa workgroups wait on workgroups of every
// index, so all C / 8 must be resident at once (<= the compute units, one per CU; checked by
// sig_maa_supported) -- the engine uses this launch only while the context has the device alone.
// Spins are bounded (timeout: *err).
#include "mv_maa.hpp"

#include <algorithm>

namespace rwkvmi {

template <int WF, int U, int U2, int LNP>
__global__ __launch_bounds__(512) void k_sig_maa(SigMaa a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float s_lora[64];
    __shared__ double ln_part[16];
    const MVHot & hv = a.hv;
    const MVHot & hr = a.hr;
    DMat W, W2;
    W.type = W2.type = WF;
    W.M = W2.M = hv.M;
    W.K = hv.K;
    W2.K = hr.K;
    W.qs = hv.qs, W.qh = hv.qh, W.sc = hv.sc;
    W2.qs = hr.qs, W2.qh = hr.qh, W2.sc = hr.sc;
    ActBuf ak, ar;
    ak.K = hv.K, ak.q = (int8_t *)hv.aq, ak.d = (float *)hv.ad, ak.s = (float *)hv.as, ak.qsum = (int *)hv.aqsum;
    ar.K = hr.K, ar.q = (int8_t *)hr.aq, ar.d = (float *)hr.ad, ar.s = (float *)hr.as, ar.qsum = (int *)hr.aqsum;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int M = hv.M, bx = (int)blockIdx.x;
    STAMP_BEGIN();
    // ---- k_mvsig's row (R = 1): value units, receptance units, their activations, x[row]
    const int row = min(bx * 8 + wave, M - 1);
    WBlk w[U], w2[U2];
#pragma unroll
    for (int u = 0; u < U; u++) w[u] = load_unit<WF>(W, row, u, lane);
#pragma unroll
    for (int u = 0; u < U2; u++) w2[u] = load_unit<WF>(W2, row, u, lane);
    AUnit x[U], x2[U2];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = load_act_unit<WF, false>(ak, u, lane);
#pragma unroll
    for (int u = 0; u < U2; u++) x2[u] = load_act_unit<WF, false>(ar, u, lane);
    const float yv = hv.y[row];
    __builtin_amdgcn_sched_barrier(0);
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    float sr, sv;
    {
        float acc = 0.0f, acc2 = 0.0f;
#pragma unroll
        for (int u = 0; u < U2; u++) {
            const bool valid = unit_valid<WF>(W2.K, u, lane);
            float t = acc, t2 = acc2;
            dot_unit<WF>(w2[u], x2[u], t, t2);
            acc = valid ? t : acc;
            acc2 = valid ? t2 : acc2;
        }
        sr = one ? wave_sum63(acc) + wave_sum63(acc2) : wave_sum63(acc) + 0.0f;
    }
    {
        float acc = 0.0f, acc2 = 0.0f;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool valid = unit_valid<WF>(W.K, u, lane);
            float t = acc, t2 = acc2;
            dot_unit<WF>(w[u], x[u], t, t2);
            acc = valid ? t : acc;
            acc2 = valid ? t2 : acc2;
        }
        sv = one ? wave_sum63(acc) + wave_sum63(acc2) : wave_sum63(acc) + 0.0f;
    }
    const float s1[1] = {sr}, s2[1] = {sv};
    const float rr = lane_row_sum<1>(s1, lane), vv = lane_row_sum<1>(s2, lane);
    const float v = yv + sigmoidf_(rr) * vv;  // EPI_SIGMUL_ADD, aux = the receptance row
    if (lane == 0 && bx * 8 + wave < M) {
        hv.y[bx * 8 + wave] = v;
        __hip_atomic_store((gran_u64_t *)(a.xg + bx * 8 + wave), ((unsigned long long)a.xtag << 32) | __float_as_uint(v),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    STAMP_MID();
    // ---- the next layer's maa workgroup (cx, n), x from the granules
    if (bx < a.nm) {
        const int nx = a.maa.C >> 6, n = bx / nx;
        maa_dec4_body<WF, U2, LNP, 64, true>(a.maa, bx - n * nx, n, smem, s_lora, ln_part, a.xg, a.xtag, a.err,
                                             a.spin_max);
    }
    STAMP_END_NS(10);
}

bool sig_maa_supported(const SigMaa & a) {
    const int t = a.hv.qs ? a.wtype : -1;
    if (!wtype_quantized(t) || a.maa.w1.type != t || !a.xg || !a.err) return false;
    const int C = a.hv.M;
    if (C != a.maa.C || a.hr.M != C || a.hr.K != C || C % 64 || C > 4096 || a.hv.K % 32) return false;
    if (mv_units(t, a.hv.K) > 8 || mv_units(t, C) > 2) return false;
    if (!v6_maa_dec_supported(C, a.maa.D, t) || a.maa.D > 32 || (int)a.maa.w1.M != 5 * a.maa.D || (int)a.maa.w1.K != C)
        return false;
    // every maa workgroup waits on all C / 8 row workgroups: all resident at one per CU
    return C / 8 <= kQgCUs && a.nm == 5 * (C / 64) && a.nm <= C / 8;
}

template <int WF, int U>
static void launch_sm_u(hipStream_t st, const SigMaa & a, bool u2, bool lnp64, int lds) {
    const dim3 grid(a.hv.M / 8), block(512);
    if (!u2) RK_LAUNCH((k_sig_maa<WF, U, 1, 32>), grid, block, lds, st, a);
    else if (!lnp64) RK_LAUNCH((k_sig_maa<WF, U, 2, 32>), grid, block, lds, st, a);
    else RK_LAUNCH((k_sig_maa<WF, U, 2, 64>), grid, block, lds, st, a);
}

template <int WF>
static void launch_sm_t(hipStream_t st, const SigMaa & a, int u, bool u2, bool lnp64, int lds) {
    if (u <= 1) launch_sm_u<WF, 1>(st, a, u2, lnp64, lds);
    else if (u <= 2) launch_sm_u<WF, 2>(st, a, u2, lnp64, lds);
    else if (u <= 4) launch_sm_u<WF, 4>(st, a, u2, lnp64, lds);
    else launch_sm_u<WF, 8>(st, a, u2, lnp64, lds);
}

bool launch_sig_maa(hipStream_t st, const SigMaa & a) {
    if (!sig_maa_supported(a)) {
        fprintf(stderr, "rwkv: channel mix + next maa decode launch: unsupported shape\n");
        return false;
    }
    const int C = a.hv.M, u = mv_units(a.wtype, a.hv.K);
    const bool u2 = mv_units(a.wtype, C) > 1, lnp64 = C > 2048;
    const int lds = a.maa.xa_off + C * 4;
    switch (a.wtype) {
        case W_Q4_0: launch_sm_t<W_Q4_0>(st, a, u, u2, lnp64, lds); break;
        case W_Q4_1: launch_sm_t<W_Q4_1>(st, a, u, u2, lnp64, lds); break;
        case W_Q5_0: launch_sm_t<W_Q5_0>(st, a, u, u2, lnp64, lds); break;
        case W_Q5_1: launch_sm_t<W_Q5_1>(st, a, u, u2, lnp64, lds); break;
        default: launch_sm_t<W_Q8_0>(st, a, u, u2, lnp64, lds); break;
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
