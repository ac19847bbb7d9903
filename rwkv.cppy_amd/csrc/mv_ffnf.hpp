// mv_ffnf.hpp -- the decode channel mix in ONE launch (rwkv_graph.inc:484-531 for v4/v5/v6,
// :533-543 for v7): LayerNorm + token shift + the FFN key rows (relu^2) and receptance rows, then
// the FFN value rows with y = x + sigmoid(r) * (Wv . k)  (v7: y = x + Wv . k).
//
// Before: the key / receptance group (k_mv, LayerNorm prologue, the key emitted as the value's Q8
// input) and the value launch (k_mvsig or k_mva) -- a kernel boundary, then the value launch's
// own weight stream (8.3 MB for v6-1B6) before its first dot.  Here the value rows' workgroups sit
// in the same grid AFTER every producer: they load their Wv rows at kernel start, so those bytes
// stream in while the producers run, and they wait for the key only.
//
//   [0, np)           producers: k_mv's emitting LayerNorm group (mv_body_split: 4 image waves, 4
//                     streaming waves x 8 rows, one 32-row Q8 block per workgroup).  The key's
//                     blocks are published as KG_STRIDE granules each (pub_q8: emit32's bits), the
//                     receptance rows as one granule per row.
//   [np, np + C/16)   consumers: 8 waves x FF_RC value rows.  Wave 0 polls the d granule of every
//                     key block; then all waves gather the blocks into the LDS activation image
//                     (the qsum -- an exact integer sum -- recomputed), each wave its rows'
//                     receptance granules; the rows' dots are k_mva's arithmetic (rows_dot_img), the
//                     epilogue EPI_SIGMUL_ADD's (EPI_ADD for v7).  Same bits as the two launches.
//
// Progress without co-residency: consumers wait only on producers, which have lower indices and
// never wait.  Races on x: producers read all of x (the LayerNorm) before they publish; a consumer
// reads and writes only its own rows of x, after every key block is published -- so no producer
// can read a row a consumer has already written.  Spins are bounded (timeout: *err).
#pragma once
#include "mv_common.hpp"

namespace rwkvmi {

constexpr int FF_RC = 2;  // value rows per consumer wave (8 waves: 16 rows per consumer workgroup)

// CO: the co-resident form (Engine::co_mode only) -- no consumer workgroups: every producer
// workgroup, once its key / receptance rows are published, runs value rows bx * 8 + wave (one per
// wave; needs 8 np >= C), issuing their weights right then, so they stream while the last key
// blocks arrive.  Its waits point at higher-index workgroups too: all np must be resident at once.
template <int WF, int UV, int FORM, bool HASR, int LNP, bool CO = false>
__global__ __launch_bounds__(512) void k_ffn_fused(FfnFused f) {
    constexpr int RC = CO ? 1 : FF_RC;  // value rows per consumer wave
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float red[32];
    const int bx = (int)blockIdx.x;
    if (bx < f.np) {
        const int e = (HASR && bx >= f.e[1].block0) ? 1 : 0;
        const MVEntry & Ent = f.e[e];
        const int b0 = e ? f.e[1].block0 : 0;
        const GranPub pub{f.kg, f.rg, f.tag};
        STAMP_BEGIN();
        mv_body_split<WF, 4, 1, MVK_LN, FORM, true, 4, LNP, true>(Ent, bx - b0, b0, 0, smem, red, 0, &pub);
        if constexpr (!CO) {
            STAMP_END(9);
            return;
        }
    }
    STAMP_BEGIN();
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int C = f.wv.M, F = f.wv.K, nb = F >> 5;
    const unsigned tag = f.tag;
    unsigned * const err = f.err;
    const unsigned spin_max = f.spin_max;
    const int row0 = ((CO ? bx : bx - f.np) * 8 + wave) * RC;
    // ---- this wave's value rows (all their units) and residual rows, in flight at once -- after
    // wdelay ticks of the 100 MHz clock, so they do not share the memory system with the
    // producers' key / receptance rows (whose arrival is on the critical path)
    if (!CO && f.wdelay > 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)f.wdelay) __builtin_amdgcn_s_sleep(8);
    }
    WBlk w[RC][UV];
#pragma unroll
    for (int u = 0; u < UV; u++)
#pragma unroll
        for (int r = 0; r < RC; r++) w[r][u] = load_unit<WF>(f.wv, min(row0 + r, C - 1), u, lane);
    const int myrow = min(row0 + min(lane, RC - 1), C - 1);
    const float xr = f.x[myrow];
    const ActBuf img = lds_act(smem, act_fmt_for(WF), F);
    // ---- wait: wave 0 polls the d granule of every key block (64 blocks per rolling poll)
    if (wave == 0 && f.prepoll) {
        for (int b0 = 0; b0 < nb; b0 += 64)
            gran_prepoll(f.kg + (size_t)b0 * KG_STRIDE, min(64, nb - b0), KG_STRIDE, 8, tag, err, spin_max, lane);
        STAMP_XN(0);
    }
    __syncthreads();
    // ---- gather: granule g = tid + 512 i (g < KG_STRIDE nb); each wave re-reads its granules until
    // every tag matches (and lanes r < FF_RC their rows' receptance)
    constexpr int GI = (KG_STRIDE * 64 * UV + 511) / 512;  // granules per thread (nb <= 64 UV)
    const int ng = KG_STRIDE * nb;
    unsigned pay[GI];
    float rr = 0.0f;
    for (unsigned it = 0;; it++) {
        unsigned long long x[GI];
#pragma unroll
        for (int i = 0; i < GI; i++) {
            const int g = tid + 512 * i;
            x[i] = (unsigned long long)tag << 32;
            if (g < ng) x[i] = __hip_atomic_load((gran_u64_t *)(f.kg + g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        unsigned long long xr8 = (unsigned long long)tag << 32;
        if (HASR) xr8 = __hip_atomic_load((gran_u64_t *)(f.rg + myrow), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = (unsigned)(xr8 >> 32) == tag;
#pragma unroll
        for (int i = 0; i < GI; i++) {
            pay[i] = (unsigned)x[i];
            ok = ok && (unsigned)(x[i] >> 32) == tag;
        }
        rr = __uint_as_float((unsigned)xr8);
        if (__all(ok)) break;
        if (it >= spin_max) {
            __hip_atomic_store((gran_u32_t *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    if (wave == 0) STAMP_XN(1);
#pragma unroll
    for (int i = 0; i < GI; i++) {
        const int g = tid + 512 * i;
        if (g < ng) {
            const int b = g / KG_STRIDE, j = g - b * KG_STRIDE;
            if (j < 8) *(unsigned *)(img.q + (size_t)b * 32 + 4 * j) = pay[i];
            else if (j == 8) img.d[b] = __uint_as_float(pay[i]);
            else if (img.fmt == A_Q8_1) img.s[b] = __uint_as_float(pay[i]);
        }
    }
    __syncthreads();
    for (int b = tid; b < nb; b += 512) {
        const int4 lo = *(const int4 *)(img.q + (size_t)b * 32), hi = *(const int4 *)(img.q + (size_t)b * 32 + 16);
        const int ws[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        int s = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) s = __builtin_amdgcn_sdot4(ws[k], 0x01010101, s, false);
        img.qsum[b] = s;
    }
    __syncthreads();
    STAMP_MID();
    // ---- the value rows: k_mva's arithmetic; EPI_SIGMUL_ADD (aux = the receptance row) / EPI_ADD
    const float s = rows_dot_img<WF, RC, UV>(w, img, F, lane);
    const float v = HASR ? xr + sigmoidf_(rr) * s : xr + s;
    if (lane < RC && row0 + lane < C) f.x[row0 + lane] = v;
    STAMP_END(9);
}

template <int WF>
bool launch_ffn_fused_t(hipStream_t st, const FfnFused & f, int form, bool hasr, int uv, int lnp, dim3 grid, int lds) {
#define FF_L(UVv, F_, R_, P_)                                                                    \
    do {                                                                                         \
        if (f.co) RK_LAUNCH((k_ffn_fused<WF, UVv, F_, R_, P_, true>), grid, dim3(512), lds, st, f); \
        else RK_LAUNCH((k_ffn_fused<WF, UVv, F_, R_, P_, false>), grid, dim3(512), lds, st, f);     \
    } while (0)
#define FF_U(F_, R_, P_)                  \
    do {                                  \
        if (uv <= 1) FF_L(1, F_, R_, P_); \
        else if (uv <= 2) FF_L(2, F_, R_, P_); \
        else if (uv <= 4) FF_L(4, F_, R_, P_); \
        else FF_L(8, F_, R_, P_);         \
    } while (0)
#define FF_P(F_, R_)                      \
    do {                                  \
        if (lnp <= 32) FF_U(F_, R_, 32);  \
        else FF_U(F_, R_, 64);            \
    } while (0)
    if (form == 0 && hasr) FF_P(0, true);
    else if (form == 1 && hasr) FF_P(1, true);
    else if (form == 1) FF_P(1, false);
    else return false;
#undef FF_P
#undef FF_U
#undef FF_L
    return true;
}

}  // namespace rwkvmi
