// mv_maa.hpp -- the v6 decode maa LoRA workgroup (rwkv_graph.inc:306-346) as a device function:
// k_v6_maa_dec4 (its own launch) and k_sig_maa (behind the previous layer's channel mix in the same
// launch, mv_sigmaa.hip) run the same code.
//
// One workgroup (cx, n) of 512 threads, D <= 32: the two roles run as separate straight paths
// that meet only at the barriers.  Waves 4..7 load the LayerNorm inputs, compute the statistics
// (no weight load ahead of them in their instruction stream: a load's issue blocks the wave once
// the CU's share of the memory system is saturated) and store the Q8 activation image and the
// fp32 xa image; waves 0..3 issue their R = 8 W1 rows (rows n*D + 8 wave + r) and their W2
// columns at once, dot the rows after the image barrier (k_mv's lane/unit order and wave_sum63
// tree: the lora values are bit-identical), and wave 0 mixes CPW = 64 channels.
//
// XG: the residual stream x is read from granules {tag, value} (xg, tag xtag) written in the same
// launch, each re-read until its tag matches (bounded: *err), instead of from a.x.
// EMB (layer 0): x = LN0(emb[*a.tok]) -- k_embed_ln's loads, chunk sums in chunk order and ln_apply,
// so the same bits -- exchanged through one more barrier; workgroup (0, 0) stores it to a.xout.
#pragma once
#include "mv_common.hpp"

namespace rwkvmi {

template <int WF, int U, int LNP, int CPW, bool XG, bool EMB = false>
__device__ __forceinline__ void maa_dec4_body(const MaaDec & a, int bx, int n, char * smem, float * s_lora,
                                              double * ln_part, const unsigned long long * xg, unsigned xtag,
                                              unsigned * err, unsigned spin_max) {
    constexpr int R = 8, DM = 32;
    const int C = a.C, D = a.D, K = C;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const ActBuf act = lds_act(smem, act_fmt_for(WF), K);
    float * s_xa = (float *)(smem + a.xa_off);
    constexpr int LCW = LNP > 32 ? 2 : 1;
    const int nch = (K + LN_CHUNK - 1) / LN_CHUNK;
    if (wave >= 4) {
        const int pw = wave - 4;
        MVEntry E;
        E.x = a.x;
        E.carry = a.carry;
        E.lnw = a.lnw;
        E.lnb = a.lnb;
        E.mu = a.maa_x;
        E.carry_out = a.carry_out;
        E.f = nullptr;
        ChunkIn ci[LCW];
        int kc[LCW];
#pragma unroll
        for (int q = 0; q < LCW; q++) {
            kc[q] = (pw + 4 * q) * LN_CHUNK + lane * 8;
            chunk_load<MVK_LN, 1>(E, min(kc[q], K - 8), ci[q]);
        }
        if constexpr (EMB) {
            __shared__ double e_part[2][8];
            const size_t tk = *a.tok;
            float w0[LCW][8], b0[LCW][8];
#pragma unroll
            for (int q = 0; q < LCW; q++) {
                ln_load8(w0[q], a.ln0w, kc[q], K);
                ln_load8(b0[q], a.ln0b, kc[q], K);
                const int k = min(kc[q], K - 8);
                if (a.emb.type == W_F16) {
                    const int4 raw = *(const int4 *)((const __half *)a.emb.qs + tk * K + k);
                    const __half * h = (const __half *)&raw;
#pragma unroll
                    for (int j = 0; j < 8; j++) ci[q].x[j] = __half2float(h[j]);
                } else {
                    ln_load8(ci[q].x, (const float *)a.emb.qs + tk * K, k, K);
                }
            }
#pragma unroll
            for (int q = 0; q < LCW; q++)
                if (pw + 4 * q < nch) {
                    double c1, c2;
                    ln_chunk_sums(ci[q].x, kc[q] < K, c1, c2);
                    if (lane == 0) {
                        e_part[0][pw + 4 * q] = c1;
                        e_part[1][pw + 4 * q] = c2;
                    }
                }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // (E) LN0 statistics
            double s1 = 0.0, s2 = 0.0;
            for (int q = 0; q < nch; q++) s1 += e_part[0][q], s2 += e_part[1][q];
            float m0, sc0;
            ln_finish(s1, s2, K, 1e-5f, m0, sc0);
#pragma unroll
            for (int q = 0; q < LCW; q++) {
#pragma unroll
                for (int j = 0; j < 8; j++) ci[q].x[j] = ln_apply(ci[q].x[j], m0, sc0, w0[q][j], b0[q][j]);
                if (bx == 0 && n == 0 && pw + 4 * q < nch && kc[q] < K) {
                    *(float4 *)(a.xout + kc[q]) = make_float4(ci[q].x[0], ci[q].x[1], ci[q].x[2], ci[q].x[3]);
                    *(float4 *)(a.xout + kc[q] + 4) = make_float4(ci[q].x[4], ci[q].x[5], ci[q].x[6], ci[q].x[7]);
                }
            }
        }
        if constexpr (XG) {
            // one granule per chunk first (a wave-uniform address: one request per poll), so the
            // waiting waves do not load the row producers' lines 512 times over
#pragma unroll
            for (int q = 0; q < LCW; q++)
                if (pw + 4 * q < nch) {
                    const unsigned long long * g0 = xg + (pw + 4 * q) * LN_CHUNK;
                    for (unsigned it = 0; it < spin_max; it++) {
                        const unsigned long long v = __hip_atomic_load((gran_u64_t *)g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((unsigned)(v >> 32) == xtag) break;
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
            // this lane's 8 elements of x from their granules (the plain loads above read the
            // previous values of x: replaced)
#pragma unroll
            for (int q = 0; q < LCW; q++) {
                const unsigned long long * g = xg + min(kc[q], K - 8);
                for (unsigned it = 0;; it++) {
                    unsigned long long v[8];
#pragma unroll
                    for (int j = 0; j < 8; j++)
                        v[j] = __hip_atomic_load((gran_u64_t *)(g + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bool ok = true;
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        ci[q].x[j] = __uint_as_float((unsigned)v[j]);
                        ok = ok && (unsigned)(v[j] >> 32) == xtag;
                    }
                    if (__all(ok || pw + 4 * q >= nch)) break;
                    if (it >= spin_max) {
                        __hip_atomic_store((gran_u32_t *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
        }
        // LayerNorm statistics (chunk association, one pass); the chunk sums meet in LDS
#pragma unroll
        for (int q = 0; q < LCW; q++)
            if (pw + 4 * q < nch) {
                double c1, c2;
                ln_chunk_sums(ci[q].x, kc[q] < K, c1, c2);
                if (lane == 0) {
                    ln_part[pw + 4 * q] = c1;
                    ln_part[8 + pw + 4 * q] = c2;
                }
            }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        double s1 = 0.0, s2 = 0.0;
        for (int q = 0; q < nch; q++) s1 += ln_part[q], s2 += ln_part[8 + q];
        float mean, scale;
        ln_finish(s1, s2, K, 1e-5f, mean, scale);
        const bool write_carry = bx == 0 && n == 0;
#pragma unroll
        for (int q = 0; q < LCW; q++) {
            if (pw + 4 * q >= nch) continue;
            if (kc[q] < K) {
#pragma unroll
                for (int j = 0; j < 8; j++) s_xa[kc[q] + j] = ln_apply(ci[q].x[j], mean, scale, ci[q].w[j], ci[q].b[j]);
            }
            chunk_store<WF, MVK_LN, 1>(E, act, ci[q], mean, scale, write_carry, kc[q], kc[q] < K, lane);
        }
        __syncthreads();  // (1) activation image ready
        __syncthreads();  // (2) lora_n ready
    } else {
        const ActBuf ao = a.out[n];
        pin_act(ao);
        const DMat & W = a.w1;
        asm volatile("" ::"s"(W.qs), "s"(W.sc), "s"(W.qh));
        // ---- rows n*D + wave*R + r of W1 and this thread's mix channel: W2 column, carry, maa
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
        const int c = bx * CPW + tid;
        const bool cval = tid < CPW && (int)(bx * CPW + (tid & ~31)) < C;  // half-wave uniform
        const int cc = min(c, C - 1);
        float w2v[DM];
        const float * w2 = a.w2t + (size_t)n * D * C + cc;
#pragma unroll
        for (int i = 0; i < DM; i++) w2v[i] = w2[(size_t)min(i, D - 1) * C];  // rows >= D: skipped below
        const float carry_c = a.carry[cc];
        const float mu_c = a.maa[n][cc];
        if constexpr (EMB) asm volatile("s_barrier" ::: "memory");  // (E)
        asm volatile("s_barrier" ::: "memory");  // the image waves' statistics exchange
        __syncthreads();  // (1) activation image ready
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
        // k_v6_mix5_dec's arithmetic: m = fma chain over i in order
        const float xa = s_xa[cc];
        const float sx = carry_c - xa;
        float m = 0.0f;
#pragma unroll
        for (int i = 0; i < DM; i++)
            if (i < D) m = fmaf(w2v[i], s_lora[i], m);
        if (cval) emit32(ao, 0, c, (m + mu_c) * sx + xa);
    }
}

}  // namespace rwkvmi
