// kernels.hip -- gfx950 kernels for the RWKV eval hot path.
//
// Numerics mirror the reference's CPU path (rwkv_graph.inc + ggml CPU ops), restated in
// oracle/oracle.c, and are compiled with -ffp-contract=off so every multiply/add rounds
// where the reference rounds; fused multiply-adds appear only where ggml's x86 kernels use
// them (the quantized block accumulation).
#include "kernels.hpp"

#include <algorithm>
#include <type_traits>
#include "device_common.hpp"

#include <stdio.h>

namespace rwkvmi {



template <int WF, int RPW, int NT>
__device__ __forceinline__ void mm_accumulate(const MMEntry & E, int row0, int t0, int T, int lane,
                                              float (&acc)[RPW][NT], float (&acc2)[RPW][NT]) {
    const DMat & W = E.W;
    const int K = W.K, M = W.M;
    if constexpr (WF == W_F32) {
        for (int k = lane * 4; k < K; k += 256) {
            float4 x[NT];
#pragma unroll
            for (int n = 0; n < NT; n++)
                x[n] = (t0 + n < T) ? *(const float4 *)(E.in.f + (size_t)(t0 + n) * K + k) : make_float4(0, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < RPW; r++) {
                const int row = row0 + r;
                if (row < M) {
                    const float4 w = *(const float4 *)((const float *)W.qs + (size_t)row * K + k);
#pragma unroll
                    for (int n = 0; n < NT; n++) {
                        float a = acc[r][n];
                        a = fmaf(w.x, x[n].x, a);
                        a = fmaf(w.y, x[n].y, a);
                        a = fmaf(w.z, x[n].z, a);
                        a = fmaf(w.w, x[n].w, a);
                        acc[r][n] = a;
                    }
                }
            }
        }
    } else if constexpr (WF == W_F16) {
        for (int k = lane * 8; k < K; k += 512) {
            int4 x[NT];
#pragma unroll
            for (int n = 0; n < NT; n++)
                x[n] = (t0 + n < T) ? *(const int4 *)(E.in.h + (size_t)(t0 + n) * K + k) : make_int4(0, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < RPW; r++) {
                const int row = row0 + r;
                if (row < M) {
                    const int4 w = *(const int4 *)((const __half *)W.qs + (size_t)row * K + k);
#pragma unroll
                    for (int n = 0; n < NT; n++) {
                        acc[r][n] = dot8_f16(w, x[n], acc[r][n]);
                    }
                }
            }
        }
    } else {
        const int nb = K >> 5;
        for (int b = lane; b < nb; b += 64) {
            int4 alo[NT], ahi[NT];
            float dx[NT], sx[NT];
            int qs[NT];
#pragma unroll
            for (int n = 0; n < NT; n++) {
                if (t0 + n < T) {
                    const int4 * ap = (const int4 *)(E.in.q + (size_t)(t0 + n) * K + (size_t)b * 32);
                    alo[n] = ap[0];
                    ahi[n] = ap[1];
                    const size_t bi = (size_t)(t0 + n) * nb + b;
                    dx[n] = E.in.d[bi];
                    qs[n] = E.in.qsum[bi];
                    sx[n] = (WF == W_Q4_1 || WF == W_Q5_1) ? E.in.s[bi] : 0.0f;
                } else {
                    alo[n] = make_int4(0, 0, 0, 0);
                    ahi[n] = alo[n];
                    dx[n] = 0.0f;
                    qs[n] = 0;
                    sx[n] = 0.0f;
                }
            }
#pragma unroll
            for (int r = 0; r < RPW; r++) {
                const int row = row0 + r;
                if (row < M) {
#pragma unroll
                    for (int n = 0; n < NT; n++) {
                        float dw, mw;
                        const int sumi = block_dot<WF>(W, row, b, nb, alo[n], ahi[n], qs[n], dw, mw);
                        acc[r][n] = fmaf(dw * dx[n], (float)sumi, acc[r][n]);
                        if constexpr (WF == W_Q4_1 || WF == W_Q5_1) acc2[r][n] = fmaf(mw, sx[n], acc2[r][n]);  // exact product
                    }
                }
            }
        }
    }
}

template <int WF, int RPW, int NT>
__global__ __launch_bounds__(256) void k_mm(MMGroup g) {
    constexpr int RW = 4 * RPW;  // rows per workgroup
    __shared__ float red[NT][RW];
    __shared__ float red2[NT][RW];
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MMEntry & E = g.e[e];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int rowwg = ((int)blockIdx.x - E.block0) * RW;
    const int row0 = rowwg + wave * RPW;
    const int T = g.T;
    // grid.y splits the tokens into spans (a multiple of NT each): every output keeps its own
    // arithmetic, the small-M groups (LoRA first stages, 18 row blocks) just get more workgroups
    const int span = ((T + (int)gridDim.y - 1) / (int)gridDim.y + NT - 1) / NT * NT;
    const int tb = (int)blockIdx.y * span, te = min(T, tb + span);
    for (int t0 = tb; t0 < te; t0 += NT) {
        float acc[RPW][NT], acc2[RPW][NT];
#pragma unroll
        for (int r = 0; r < RPW; r++)
#pragma unroll
            for (int n = 0; n < NT; n++) acc[r][n] = acc2[r][n] = 0.0f;
        mm_accumulate<WF, RPW, NT>(E, row0, t0, T, lane, acc, acc2);
#pragma unroll
        for (int r = 0; r < RPW; r++)
#pragma unroll
            for (int n = 0; n < NT; n++) {
                const float s = wave_sum63(acc[r][n]);
                float s2 = 0.0f;
                if constexpr (WF == W_Q4_1 || WF == W_Q5_1) s2 = wave_sum63(acc2[r][n]);
                if (lane == 63) {
                    red[n][wave * RPW + r] = s;
                    red2[n][wave * RPW + r] = s2;
                }
            }
        __syncthreads();
        const int tid = threadIdx.x;
        if (tid < RW * NT) {
            const int n = tid / RW, r = tid % RW;
            const int t = t0 + n, row = rowwg + r;
            // (t < T) is uniform across each 32-lane half-wave since RW is a multiple of 32
            // whenever emission is used (RPW == 8).
            if (t < T) {
                const float acc_v = red[n][r] + red2[n][r];
                float v = 0.0f;
                if (row < E.W.M) {
                    v = apply_epi(E, t, row, acc_v);
                    if (E.y) E.y[(size_t)t * E.ldy + row] = v;
                }
                if (E.emit) emit32(E.out, t, row, v);
            }
        }
        __syncthreads();
    }
}

template <int WF>
static bool launch_mm_wf(hipStream_t st, MMGroup & g) {
    bool emit = false;
    for (int i = 0; i < g.n; i++) emit |= g.e[i].emit != 0;
    const int T = g.T;
    // Emission needs 32 rows per workgroup (one quantization block per half-wave).
    const int rpw = emit ? 8 : 2;
    const int rw = 4 * rpw;
    int blocks = 0;
    for (int i = 0; i < g.n; i++) {
        if (g.e[i].emit && (g.e[i].W.M % 32 != 0)) {
            fprintf(stderr, "rwkv: emitting matmul needs M %% 32 == 0 (M=%d)\n", g.e[i].W.M);
            return false;
        }
        if (g.e[i].W.K % 32 != 0) {
            fprintf(stderr, "rwkv: matmul needs K %% 32 == 0 (K=%d)\n", g.e[i].W.K);
            return false;
        }
        g.e[i].block0 = blocks;
        blocks += (g.e[i].W.M + rw - 1) / rw;
    }
    if (blocks == 0) return true;
    dim3 grid(blocks), block(256);
    if (T == 1) {
        if (emit) RK_LAUNCH((k_mm<WF, 8, 1>), grid, block, 0, st, g);
        else RK_LAUNCH((k_mm<WF, 2, 1>), grid, block, 0, st, g);
    } else {
        // token spans so that the grid has ~4096 workgroups (at most one span per 4 tokens)
        // (batched decode, T <= 16 over >= 256 row blocks: one span, every weight read once)
        const int gy = (T <= 16 && blocks >= 256) ? 1 : std::max(1, std::min((T + 3) / 4, 4096 / blocks));
        const dim3 grid2(blocks, gy);
        if (emit) RK_LAUNCH((k_mm<WF, 8, 4>), grid2, block, 0, st, g);
        else RK_LAUNCH((k_mm<WF, 2, 4>), grid2, block, 0, st, g);
    }
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- small-K matmul
// F16 / F32 weights whose rows fit one unit per lane of k_mm (K <= 512 halves / 256 floats: the v7
// LoRA second stages, K = 64..480), T >= 2.  k_mm gives each output a whole wave, most of whose
// lanes hold no unit (K = 96: 12 of 64) and then a 6-step DPP reduction.  Here one THREAD computes
// one output: the lane partials p[l] = dot over unit l (k_mm's per-lane arithmetic, from 0) and
// wave_sum63's perfect binary tree over them.  Lanes without a unit contribute +0, and a partial
// is never -0 (every chain starts from +0), so the zero leaves change no bit and the tree is
// folded only over the NL leading leaves (NL = the next power of two): results equal k_mm's.
// Workgroup = 64 rows (one per lane) x MMS_TB tokens (waves take every 4th token); the rows'
// weights and the tokens' activations are staged in LDS.
constexpr int MMS_TB = 16;

template <int WF>
__device__ __forceinline__ float small_leaf(const char * wrow, const char * xrow, int l, int nl) {
    float p = 0.0f;
    if (l < nl) {
        const int4 w = *(const int4 *)(wrow + 16 * l), x = *(const int4 *)(xrow + 16 * l);
        if constexpr (WF == W_F16) {
            p = dot8_f16(w, x, 0.0f);
        } else {
            p = fmaf(__int_as_float(w.x), __int_as_float(x.x), p);
            p = fmaf(__int_as_float(w.y), __int_as_float(x.y), p);
            p = fmaf(__int_as_float(w.z), __int_as_float(x.z), p);
            p = fmaf(__int_as_float(w.w), __int_as_float(x.w), p);
        }
    }
    return p;
}

// Leaves in groups of 8 (a perfect 8-leaf tree each), the groups folded as they are produced (a
// binary counter: lv[k] holds the pending left subtree of 8 * 2^k leaves) -- the same perfect
// binary tree over NL leaves with few live registers.
template <int WF, int NL>
__device__ __forceinline__ float small_row_dot(const char * wrow, const char * xrow, int nl) {
    float lv[3];
    float v = 0.0f;
#pragma unroll 1
    for (int g = 0; g < NL / 8; g++) {
        float p[8];
#pragma unroll
        for (int l = 0; l < 8; l++) p[l] = small_leaf<WF>(wrow, xrow, 8 * g + l, nl);
        v = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
#pragma unroll
        for (int k = 0; (8 << k) < NL; k++) {
            if (g & (1 << k)) {
                v = lv[k] + v;
            } else {
                lv[k] = v;
                break;
            }
        }
    }
    return v;  // the last group closed every level: the root
}

template <int WF>
__global__ __launch_bounds__(256) void k_mm_small(MMGroup g, int wstride) {
    extern __shared__ __attribute__((aligned(16))) char sm[];
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MMEntry & E = g.e[e];
    const int M = E.W.M, K = E.W.K, T = g.T;
    constexpr int ES = WF == W_F16 ? 2 : 4;       // element bytes
    const int rowb = K * ES, nl = rowb / 16;       // bytes per row, units (lanes of k_mm)
    const int row0 = ((int)blockIdx.x - E.block0) * 64, t0 = (int)blockIdx.y * MMS_TB;
    char * ws = sm;                                // [64][wstride]
    char * xs = sm + 64 * wstride;                 // [MMS_TB][rowb]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const char * wg = (const char *)E.W.qs;
    const char * xg = (const char *)(WF == W_F16 ? (const void *)E.in.h : (const void *)E.in.f);
    // (row, unit) of flat index i: i / nl through a float reciprocal (exact: i < 2^12, nl <= 64)
    const float rnl = 1.0f / (float)nl;
    for (int i = tid; i < 64 * nl; i += 256) {
        const int r = (int)(((float)i + 0.5f) * rnl), u = i - r * nl;
        const int row = min(row0 + r, M - 1);
        *(int4 *)(ws + r * wstride + 16 * u) = *(const int4 *)(wg + (size_t)row * rowb + 16 * u);
    }
    for (int i = tid; i < MMS_TB * nl; i += 256) {
        const int t = (int)(((float)i + 0.5f) * rnl), u = i - t * nl;
        const int tt = min(t0 + t, T - 1);
        *(int4 *)(xs + t * rowb + 16 * u) = *(const int4 *)(xg + (size_t)tt * rowb + 16 * u);
    }
    __syncthreads();
    const int row = row0 + lane;
    const char * wrow = ws + lane * wstride;
    for (int tl = wave; tl < MMS_TB; tl += 4) {
        const int t = t0 + tl;
        if (t >= T) break;  // wave-uniform
        const char * xrow = xs + tl * rowb;
        float s;
        if (nl <= 8) s = small_row_dot<WF, 8>(wrow, xrow, nl);
        else if (nl <= 16) s = small_row_dot<WF, 16>(wrow, xrow, nl);
        else if (nl <= 32) s = small_row_dot<WF, 32>(wrow, xrow, nl);
        else s = small_row_dot<WF, 64>(wrow, xrow, nl);
        // k_mm: red + red2 (red2 = 0 for float weights)
        const float acc = s + 0.0f;
        float v = 0.0f;
        if (row < M) {
            v = apply_epi(E, t, row, acc);
            if (E.y) E.y[(size_t)t * E.ldy + row] = v;
        }
        // a half-wave = 32 consecutive rows of token t (M % 32 == 0 when emitting)
        if (E.emit && row0 + (lane & 32) < M) emit32(E.out, t, row, v);
    }
}

// true (and launched) when every entry is an F16 / F32 matrix with one unit per k_mm lane
static bool launch_mm_small(hipStream_t st, MMGroup & g, int wtype) {
    if (g.T < 2 || (wtype != W_F16 && wtype != W_F32)) return false;
    const int ES = wtype == W_F16 ? 2 : 4;
    int blocks = 0, kmax = 0;
    for (int i = 0; i < g.n; i++) {
        const MMEntry & e = g.e[i];
        if (e.W.type != wtype || e.W.K * ES > 1024 || (e.W.K * ES) % 16 || e.in.fmt != act_fmt_for(wtype) ||
            (e.emit && e.W.M % 32))
            return false;
        kmax = std::max(kmax, e.W.K);
    }
    for (int i = 0; i < g.n; i++) {
        g.e[i].block0 = blocks;
        blocks += (g.e[i].W.M + 63) / 64;
    }
    const int wstride = kmax * ES + 16;  // padded row: 16-byte reads of 16 lanes spread over banks
    const size_t lds = (size_t)64 * wstride + (size_t)MMS_TB * kmax * ES;
    const dim3 grid(blocks, (g.T + MMS_TB - 1) / MMS_TB);
    if (wtype == W_F16) RK_LAUNCH(k_mm_small<W_F16>, grid, dim3(256), lds, st, g, wstride);
    else RK_LAUNCH(k_mm_small<W_F32>, grid, dim3(256), lds, st, g, wstride);
    return hipGetLastError() == hipSuccess;
}

bool launch_mm_group(hipStream_t st, MMGroup & g, int wtype) {
    bool fmm = false;
    if (!launch_fmm_group(st, g, wtype, &fmm)) return false;
    if (fmm) return true;
    if (launch_mm_small(st, g, wtype)) return true;
    switch (wtype) {
        case W_F32: return launch_mm_wf<W_F32>(st, g);
        case W_F16: return launch_mm_wf<W_F16>(st, g);
        case W_Q4_0: return launch_mm_wf<W_Q4_0>(st, g);
        case W_Q4_1: return launch_mm_wf<W_Q4_1>(st, g);
        case W_Q5_0: return launch_mm_wf<W_Q5_0>(st, g);
        case W_Q5_1: return launch_mm_wf<W_Q5_1>(st, g);
        case W_Q8_0: return launch_mm_wf<W_Q8_0>(st, g);
        default:
            fprintf(stderr, "rwkv: unsupported weight type %d\n", wtype);
            return false;
    }
}

// --------------------------------------------------------------------------- timing helper
__global__ void k_delay(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

bool launch_delay(hipStream_t st, int us) {
    RK_LAUNCH(k_delay, dim3(1), dim3(64), 0, st, (unsigned long long)us * 100ull);  // 100 MHz clock
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- LayerNorm family

// One token row per workgroup.  Every wave loads the embedding row straight into registers in the
// LayerNorm chunk layout (lane l: elements 512 c + 8 l .. + 7) and computes the statistics itself
// (ln_stats_regs: ln_stats_wave's association, the same bits as the sequence kernels); wave w then
// normalizes and stores chunks w, w + 4, ...  The LayerNorm weights are loaded at kernel start, before
// the token id returns: two dependent memory round trips (token, row) instead of a store / reload of
// the row through L2 between them.
constexpr int EMB_NC = 8;  // chunks held per lane: n_embed <= 4096
__global__ __launch_bounds__(256) void k_embed_ln(const uint32_t * tokens, DMat emb, const float * w,
                                                  const float * b, float * x) {
    STAMP_BEGIN();
    const int t = blockIdx.x, C = emb.K, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nc = (C + LN_CHUNK - 1) / LN_CHUNK;
    float wv[2][8], bv[2][8];  // this wave's chunks w and w + 4
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const int c = wave + 4 * q;
        if (c < nc) {
            ln_load8(wv[q], w, c * LN_CHUNK + lane * 8, C);
            ln_load8(bv[q], b, c * LN_CHUNK + lane * 8, C);
        }
    }
    const size_t tok = tokens[t];
    float v[EMB_NC][8];
#pragma unroll
    for (int c = 0; c < EMB_NC; c++) {
        if (c >= nc) break;
        const int k = min(c * LN_CHUNK + lane * 8, C - 8);
        if (emb.type == W_F16) {
            const __half * p = (const __half *)emb.qs + tok * C + k;
            const int4 raw = *(const int4 *)p;
            const __half * h = (const __half *)&raw;
#pragma unroll
            for (int j = 0; j < 8; j++) v[c][j] = __half2float(h[j]);
        } else {
            ln_load8(v[c], (const float *)emb.qs + tok * C, k, C);
        }
    }
    float mean, scale;
    ln_stats_regs<EMB_NC>(v, nc, C, 1e-5f, mean, scale);
    float * xr = x + (size_t)t * C;
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const int c = wave + 4 * q;
        if (c >= nc) continue;
        const int k = c * LN_CHUNK + lane * 8;
        if (k >= C) continue;
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = ln_apply(v[c][j], mean, scale, wv[q][j], bv[q][j]);
        *(float4 *)(xr + k) = make_float4(o[0], o[1], o[2], o[3]);
        *(float4 *)(xr + k + 4) = make_float4(o[4], o[5], o[6], o[7]);
    }
    STAMP_END(5);
}

// Rows wider than EMB_NC chunks (n_embed > 4096, e.g. RWKV-4 14B at 5120): the same statistics
// association (ln_stats_wave's chunk order, 4 chunks in flight) with the row re-read from HBM per
// group of chunks, every wave on its own (no exchange), then wave w normalizes chunks w, w + 4, ...
__device__ __forceinline__ void emb_load8(float (&v)[8], const DMat & emb, size_t tok, int k) {
    const int C = emb.K;
    if (emb.type == W_F16) {
        const int4 raw = *(const int4 *)((const __half *)emb.qs + tok * C + min(k, C - 8));
        const __half * h = (const __half *)&raw;
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = __half2float(h[j]);
    } else {
        ln_load8(v, (const float *)emb.qs + tok * C, k, C);
    }
}
__global__ __launch_bounds__(256) void k_embed_ln_wide(const uint32_t * tokens, DMat emb, const float * w,
                                                       const float * b, float * x) {
    const int t = blockIdx.x, C = emb.K, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nc = (C + LN_CHUNK - 1) / LN_CHUNK;
    const size_t tok = tokens[t];
    double s1 = 0.0, s2 = 0.0;
    for (int c0 = 0; c0 < nc; c0 += 4) {
        float v[4][8];
#pragma unroll
        for (int c = 0; c < 4; c++) emb_load8(v[c], emb, tok, min(c0 + c, nc - 1) * LN_CHUNK + lane * 8);
        double c1[4], c2[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            c1[c] = c2[c] = 0.0;
            if (c0 + c < nc) ln_chunk_sums(v[c], (c0 + c) * LN_CHUNK + lane * 8 < C, c1[c], c2[c]);
        }
#pragma unroll
        for (int c = 0; c < 4; c++)
            if (c0 + c < nc) s1 += c1[c], s2 += c2[c];
    }
    float mean, scale;
    ln_finish(s1, s2, C, 1e-5f, mean, scale);
    float * xr = x + (size_t)t * C;
    for (int c = wave; c < nc; c += 4) {
        const int k = c * LN_CHUNK + lane * 8;
        if (k >= C) continue;
        float v[8], wv[8], bv[8], o[8];
        emb_load8(v, emb, tok, k);
        ln_load8(wv, w, k, C);
        ln_load8(bv, b, k, C);
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = ln_apply(v[j], mean, scale, wv[j], bv[j]);
        *(float4 *)(xr + k) = make_float4(o[0], o[1], o[2], o[3]);
        *(float4 *)(xr + k + 4) = make_float4(o[4], o[5], o[6], o[7]);
    }
}

bool launch_embed_ln(hipStream_t st, const uint32_t * tokens, int T, const DMat & emb, const float * w,
                     const float * b, float * x) {
    if (emb.K % 8 || (emb.type != W_F16 && emb.type != W_F32)) {
        fprintf(stderr, "rwkv: embedding row of %d elements (type %d) unsupported\n", emb.K, emb.type);
        return false;
    }
    if (emb.K > EMB_NC * LN_CHUNK) RK_LAUNCH(k_embed_ln_wide, dim3(T), dim3(256), 0, st, tokens, emb, w, b, x);
    else RK_LAUNCH(k_embed_ln, dim3(T), dim3(256), 0, st, tokens, emb, w, b, x);
    HIP_OK(hipGetLastError());
    return true;
}

// Token-row kernels that emit Q8 activations into sequence-GEMM token tiles run TOKS_PER_WG
// consecutive tokens per workgroup (one 256-thread group each): a tile record's 64-byte sectors
// hold 16-byte pieces of 4 consecutive tokens, so the four partial writes of a sector meet in one
// XCD's L2 instead of leaving four L2s as four partial-line write-backs.
constexpr int TOKS_PER_WG = 4;

// emit32 for an output known at compile time to be Q8 sequence-GEMM token tiles (TQ 1: Q8_0,
// 2: Q8_1) of row length K: store32's tiled values, no runtime format dispatch
template <int TQ>
__device__ __forceinline__ void emit32_tile(uint8_t * tq, int K, int t, int k, float v) {
    const Q32 r = quant32(v);
    uint8_t * rec = tq + ((size_t)(t / QG_TOK) * (K >> 5) + (k >> 5)) * qg_a_bytes(TQ == 2);
    const int tl = t % QG_TOK;
    rec[((k >> 4) & 1) * QG_TOK * 16 + tl * 16 + (k & 15)] = (uint8_t)(int8_t)r.q;
    if ((k & 31) == 0) {
        ((float *)(rec + QG_A_D))[tl] = f16_round(r.d);
        if constexpr (TQ == 2) ((float *)(rec + QG_A_S))[tl] = f16_round(r.d * (float)r.sum);
    }
}

// TQ of a set of outputs: 1 / 2 when all are Q8_0 / Q8_1 token tiles of row length K, else 0
static int tile_q(const ActBuf * outs, int n, int K) {
    if (n < 1) return 0;
    for (int i = 0; i < n; i++)
        if (!outs[i].tiled || outs[i].fmt != outs[0].fmt || outs[i].K != K ||
            (outs[i].fmt != A_Q8_0 && outs[i].fmt != A_Q8_1))
            return 0;
    return outs[0].fmt == A_Q8_1 ? 2 : 1;
}

// rwkv_carry_x (rwkv_graph.inc:56-82) + the token-shift mixes of each version.
template <int TQ>
__global__ __launch_bounds__(1024) void k_ln_mix(LnMixArgs a) {
    // LayerNorm statistics of the workgroup's TOKS_PER_WG + 1 rows (its tokens and the one before),
    // one wave per row (the canonical one-wave association), shared through LDS
    __shared__ float s_mean[TOKS_PER_WG + 1], s_scale[TOKS_PER_WG + 1];
    const int tg = threadIdx.x >> 8, t = blockIdx.x * TOKS_PER_WG + tg, C = a.C, tid = threadIdx.x & 255;
    const int wave = threadIdx.x >> 6;
    if (wave <= TOKS_PER_WG) {
        const int rt = (int)blockIdx.x * TOKS_PER_WG - 1 + wave;
        if (rt >= 0 && rt < a.T) {
            float m, sc;
            ln_stats_any(a.x + (size_t)rt * C, C, 1e-5f, m, sc);
            if ((threadIdx.x & 63) == 0) {
                s_mean[wave] = m;
                s_scale[wave] = sc;
            }
        }
    }
    __syncthreads();
    if (t >= a.T) return;  // whole 256-thread token groups
    const float * xt = a.x + (size_t)t * C;
    const float mean = s_mean[tg + 1], scale = s_scale[tg + 1];
    const float pmean = t > 0 ? s_mean[tg] : 0.0f, pscale = t > 0 ? s_scale[tg] : 0.0f;
    // channel blocks of 256 split over grid.y (short sequences / batched decode: more workgroups);
    // LNM_CB blocks at a time: all their loads are issued before the first store
    constexpr int LNM_CB = TQ > 0 ? 4 : 2;  // (4 spills in the runtime-format emit)
    const int cstride = (int)gridDim.y * 256;
    const int nmu = min(a.n_out, 6);
    for (int cb0 = (int)blockIdx.y * 256; cb0 < C; cb0 += LNM_CB * cstride) {
        float xv[LNM_CB], pv[LNM_CB], wv[LNM_CB], bv[LNM_CB], muv[LNM_CB][6];
#pragma unroll
        for (int j = 0; j < LNM_CB; j++) {
            const int c = min(cb0 + j * cstride + tid, C - 1);
            xv[j] = xt[c];
            wv[j] = a.lnw[c];
            bv[j] = a.lnb[c];
            // batch (a.bs > 0): every token is its own context, shifted against its own carry
            pv[j] = a.bs ? a.carry_in[(size_t)t * a.bs + c] : (t > 0) ? xt[c - C] : a.carry_in[c];
#pragma unroll
            for (int n = 0; n < 6; n++) muv[j][n] = n < nmu ? a.mu[n][c] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < LNM_CB; j++) {
            const int c0 = cb0 + j * cstride, c = c0 + tid;
            if (c0 + (tid & ~63) >= C) continue;  // whole wave out of range (C % 64 == 0)
            const float xa = ln_apply(xv[j], mean, scale, wv[j], bv[j]);
            const float xp = (a.bs || t == 0) ? pv[j] : ln_apply(pv[j], pmean, pscale, wv[j], bv[j]);
            if (a.bs && a.carry_out) a.carry_out[(size_t)t * a.bs + c] = xa;
            else if (t == a.T - 1 && a.carry_out) a.carry_out[c] = xa;
            if (a.out_xa) a.out_xa[(size_t)t * C + c] = xa;
            if (a.out_sx) a.out_sx[(size_t)t * C + c] = xp - xa;
#pragma unroll
            for (int n = 0; n < 6; n++) {
                if (n >= nmu) break;
                const float mu = muv[j][n];
                float v;
                if (a.form == 0) {
                    v = xa * mu + (xp - xp * mu);
                } else {
                    v = (xp - xa) * mu + xa;
                }
                if constexpr (TQ > 0) emit32_tile<TQ>(a.out[n].tq, C, t, c, v);
                else emit32(a.out[n], t, c, v);
            }
        }
    }
}

bool launch_ln_mix(hipStream_t st, const LnMixArgs & a) {
    // long sequences: one channel block row (grid.y = 1; each workgroup computes its rows' LayerNorm
    // statistics itself, so splitting the channels repeats that work: y = 2 / 4 / 8 measured slower)
    // fewer token groups than ~2 per CU (short sequences, batched decode): the channel blocks over
    // grid.y until the grid holds about 512 workgroups
    const int tgs = (a.T + TOKS_PER_WG - 1) / TOKS_PER_WG, cbs = (a.C + 255) / 256;
    const int gy = a.T <= 64 ? cbs : tgs < 256 ? std::min(cbs, (512 + tgs - 1) / tgs) : 1;
    const dim3 grid((a.T + TOKS_PER_WG - 1) / TOKS_PER_WG, gy), block(256 * TOKS_PER_WG);
    const int tq = tile_q(a.out, a.n_out, a.C);
    if (tq == 1) RK_LAUNCH(k_ln_mix<1>, grid, block, 0, st, a);
    else if (tq == 2) RK_LAUNCH(k_ln_mix<2>, grid, block, 0, st, a);
    else RK_LAUNCH(k_ln_mix<0>, grid, block, 0, st, a);
    HIP_OK(hipGetLastError());
    return true;
}

__global__ __launch_bounds__(256) void k_ln_emit(int C, const float * x, const float * w, const float * b, ActBuf out) {
    __shared__ double sh[8];
    const int t = blockIdx.x;  // row t of x -> row t of out
    x += (size_t)t * C;
    float mean, scale;
    ln_stats(x, C, 1e-5f, mean, scale, sh);
    for (int c0 = 0; c0 < C; c0 += blockDim.x) {
        const int c = c0 + threadIdx.x;
        if (c0 + (int)(threadIdx.x & ~63) >= C) continue;
        emit32(out, t, c, ln_apply(x[c], mean, scale, w[c], b[c]));
    }
}

bool launch_ln_emit(hipStream_t st, int C, const float * x, const float * w, const float * b, const ActBuf & out,
                    int rows) {
    RK_LAUNCH(k_ln_emit, dim3(rows), dim3(256), 0, st, C, x, w, b, out);
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v6 mix5
struct Mix5Args {
    int T, C, D;
    const float * lora;
    const float * w2;
    const float * maa[5];
    const float * xa;
    const float * sx;
    ActBuf out[5];
};

// Workgroup = 64 channels x 5 mixes x MIX_TT tokens (32: the per-wave setup over more tokens, 78 -> 76 us
// per v6-1B6 layer), wave n = mixed vector n (w, k, v, r, g):
// each lane holds its channel's W2 column of that mix in registers (D floats, read once per token
// tile); the tile's lora rows sit in LDS as [mix][i][token], so one 16-byte broadcast read gives
// the i-th lora value of 4 tokens.  Per token the D-long fp32 fma chain runs in k_v6_mix5_dec's
// order (sequential over i); 4 tokens' chains run side by side (168 VGPRs: 3 waves per SIMD).
constexpr int MIX_TT = 32;  // (64: 76.8 us)

// TQ > 0: all five outputs are Q8 sequence-GEMM token tiles (TQ = 2: Q8_1); each lane's record
// address is formed once (a workgroup's MIX_TT tokens lie in one QG_TOK-token tile) and the
// per-output emission is quant32 + store (store32's tiled values), no runtime format dispatch.
template <int DM, int TQ, bool EXACT>
__global__ __launch_bounds__(320) void k_v6_mix5(Mix5Args a) {
    static_assert(QG_TOK % MIX_TT == 0 && MIX_TT % 4 == 0, "mix5 token tile");
    __shared__ __attribute__((aligned(16))) float sl[5][DM][MIX_TT];
    const int C = a.C, D = EXACT ? DM : a.D, T = a.T;
    const int tid = threadIdx.x, lane = tid & 63;
    const int n = __builtin_amdgcn_readfirstlane(tid >> 6);
    // this wave's mix: operands selected with compile-time indices (no dynamic kernarg indexing)
    const float * maa_n = a.maa[0];
    ActBuf out_n = a.out[0];
#pragma unroll
    for (int m = 1; m < 5; m++)
        if (n == m) {
            maa_n = a.maa[m];
            out_n = a.out[m];
        }
    const int c = blockIdx.x * 64 + lane;
    const bool cval = (int)(blockIdx.x * 64 + (lane & ~31)) < C;  // half-wave uniform
    const int cc = min(c, C - 1);
    const int t0 = blockIdx.y * MIX_TT, nt = min(MIX_TT, T - t0);
    for (int e = tid; e < 5 * DM * MIX_TT; e += 320) {
        const int tt = e / (5 * DM), f = e % (5 * DM), m = f / DM, i = f % DM;  // coalesced reads
        sl[m][i][tt] = (tt < nt && i < D) ? a.lora[(size_t)(t0 + tt) * 5 * D + m * D + i] : 0.0f;
    }
    float w2v[DM];
    const float mu = maa_n[cc];
#pragma unroll
    for (int i = 0; i < DM; i++) {
        const float t = a.w2[((size_t)n * D + min(i, D - 1)) * C + cc];  // transposed [5][D][C]
        w2v[i] = i < D ? t : 0.0f;
    }
    uint8_t * rec = nullptr;
    int qoff = 0;
    if constexpr (TQ > 0) {
        // record of (token tile t0 / QG_TOK, block c / 32); byte of element c in half (c >> 4) & 1
        const size_t ri = (size_t)(t0 / QG_TOK) * (C >> 5) + (cc >> 5);
        rec = out_n.tq + ri * qg_a_bytes(TQ == 2);
        qoff = ((cc >> 4) & 1) * QG_TOK * 16 + (cc & 15);
    }
    __syncthreads();
    for (int tt = 0; tt < nt; tt += 4) {
        float xa[4], sx[4], acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const size_t ti = (size_t)(t0 + min(tt + j, nt - 1)) * C + cc;
            xa[j] = a.xa[ti];
            sx[j] = a.sx[ti];
        }
#pragma unroll
        for (int i = 0; i < DM; i++) {
            if (EXACT || i < D) {
                const float4 l = *(const float4 *)&sl[n][i][tt];
                acc[0] = fmaf(w2v[i], l.x, acc[0]);
                acc[1] = fmaf(w2v[i], l.y, acc[1]);
                acc[2] = fmaf(w2v[i], l.z, acc[2]);
                acc[3] = fmaf(w2v[i], l.w, acc[3]);
            }
        }
        if (!cval) continue;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (tt + j >= nt) break;
            const float v = (acc[j] + mu) * sx[j] + xa[j];
            if constexpr (TQ > 0) {
                const Q32 q = quant32(v);
                const int tl = (t0 + tt + j) % QG_TOK;
                rec[qoff + tl * 16] = (uint8_t)(int8_t)q.q;
                if ((c & 31) == 0) {
                    ((float *)(rec + QG_A_D))[tl] = f16_round(q.d);
                    if constexpr (TQ == 2) ((float *)(rec + QG_A_S))[tl] = f16_round(q.d * (float)q.sum);
                }
            } else {
                emit32(out_n, t0 + tt + j, c, v);
            }
        }
    }
}

// The same mixes on the f32 MFMA (round 3): m[t][c] = the fmaf chain over i of W2[c][i] * lora[t][i]
// in order from 0 is exactly a chain of v_mfma_f32_16x16x4_f32 over i in quads (C first, k = 0..3
// in order: tools/mfma_f32_probe.hip), so the mixes stay bit-identical to k_v6_mix5 and the decode's
// k_v6_mix5_dec.  Workgroup = 5 waves, wave n = mix n over 32 channels x 64 tokens (2 x 4 tiles of
// 16 x 16; operands straight from L2); the epilogue quantizes each token's 32 channels -- one Q8
// block, held by lanes tok + 16 g of the D layout -- with xor-16/32 lane exchanges (order-free max
// and integer sum, quant32's values) and stores them into the token-tile records (TQ = 1: Q8_0,
// 2: Q8_1).
typedef float mixf4 __attribute__((ext_vector_type(4)));
template <int DM, int TQ>
__global__ __launch_bounds__(320) void k_v6_mix5m(Mix5Args a) {
    const int C = a.C, T = a.T;
    const int lane = threadIdx.x & 63, n = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ml = lane & 15, g = lane >> 4;
    const float * maa_n = a.maa[0];
    ActBuf out_n = a.out[0];
#pragma unroll
    for (int m = 1; m < 5; m++)
        if (n == m) {
            maa_n = a.maa[m];
            out_n = a.out[m];
        }
    const int c0 = blockIdx.x * 32, t0 = blockIdx.y * 64;
    // A operands: W2 (transposed [5][D][C]) of channels c0 + 16 ct + ml, i = 4 j + g
    float wa[2][DM / 4];
#pragma unroll
    for (int ct = 0; ct < 2; ct++)
#pragma unroll
        for (int j = 0; j < DM / 4; j++) wa[ct][j] = a.w2[((size_t)n * DM + 4 * j + g) * C + c0 + 16 * ct + ml];
    mixf4 acc[2][4];
#pragma unroll
    for (int nt = 0; nt < 4; nt++) {
        // B operands: lora[t][n][i] of token t0 + 16 nt + ml, i = 4 j + g
        const size_t tr = (size_t)min(t0 + 16 * nt + ml, T - 1) * 5 * DM + (size_t)n * DM + g;
        float lb[DM / 4];
#pragma unroll
        for (int j = 0; j < DM / 4; j++) lb[j] = a.lora[tr + 4 * j];
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            mixf4 c = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < DM / 4; j++) c = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[ct][j], lb[j], c, 0, 0, 0);
            acc[ct][nt] = c;
        }
    }
    // epilogue: lane holds channels c0 + 16 ct + 4 g + i of token t0 + 16 nt + ml
    const int cb = c0 + 4 * g;
    mixf4 mu[2];
#pragma unroll
    for (int ct = 0; ct < 2; ct++) mu[ct] = *(const mixf4 *)(maa_n + cb + 16 * ct);
    uint8_t * rec = out_n.tq + ((size_t)(t0 / QG_TOK) * (C >> 5) + (c0 >> 5)) * qg_a_bytes(TQ == 2);
#pragma unroll
    for (int nt = 0; nt < 4; nt++) {
        const int t = t0 + 16 * nt + ml;
        const size_t ti = (size_t)min(t, T - 1) * C + cb;
        float v[2][4];
        float am = 0.0f;
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            const mixf4 xa = *(const mixf4 *)(a.xa + ti + 16 * ct), sx = *(const mixf4 *)(a.sx + ti + 16 * ct);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                v[ct][i] = (acc[ct][nt][i] + mu[ct][i]) * sx[i] + xa[i];
                am = fmaxf(am, fabsf(v[ct][i]));
            }
        }
        am = fmaxf(am, __shfl_xor(am, 16));
        am = fmaxf(am, __shfl_xor(am, 32));
        const float id = (am != 0.0f) ? 127.f / am : 0.0f;
        const float d = am / 127.f;
        uint32_t packed[2];
        int sum = 0;
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            packed[ct] = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int q = (int)rintf(v[ct][i] * id);
                sum += q;
                packed[ct] |= ((uint32_t)q & 0xffu) << (8 * i);
            }
        }
        sum += __shfl_xor(sum, 16);
        sum += __shfl_xor(sum, 32);
        if (t < T) {
            const int tl = t % QG_TOK;
#pragma unroll
            for (int ct = 0; ct < 2; ct++) *(uint32_t *)(rec + ct * QG_TOK * 16 + tl * 16 + 4 * g) = packed[ct];
            if (g == 0) {
                ((float *)(rec + QG_A_D))[tl] = f16_round(d);
                if constexpr (TQ == 2) ((float *)(rec + QG_A_S))[tl] = f16_round(d * (float)sum);
            }
        }
    }
}

bool launch_v6_mix5(hipStream_t st, int T, int C, int D, const float * lora, const float * w2,
                    const float * const * maa, const float * xa, const float * sx, const ActBuf * outs) {
    Mix5Args a;
    a.T = T;
    a.C = C;
    a.D = D;
    a.lora = lora;
    a.w2 = w2;
    for (int n = 0; n < 5; n++) {
        a.maa[n] = maa[n];
        a.out[n] = outs[n];
    }
    a.xa = xa;
    a.sx = sx;
    if (D > 64 || C % 32) {
        fprintf(stderr, "rwkv: v6 maa LoRA width %d / n_embed %d unsupported\n", D, C);
        return false;
    }
    const dim3 grid((C + 63) / 64, (T + MIX_TT - 1) / MIX_TT);
    int tq = 0;
    {
        bool all = true;
        for (int n = 0; n < 5; n++)
            all = all && outs[n].tiled && outs[n].fmt == outs[0].fmt && outs[n].K == C &&
                  (outs[n].fmt == A_Q8_0 || outs[n].fmt == A_Q8_1);
        if (all) tq = outs[0].fmt == A_Q8_1 ? 2 : 1;
    }
    // the f32-MFMA form: tiled Q8 outputs, LoRA width 32 or 64, whole 32-channel blocks
    if (tq > 0 && (D == 32 || D == 64) && C % 32 == 0) {
        const dim3 mgrid(C / 32, (T + 63) / 64);
        if (D == 32) {
            if (tq == 1) RK_LAUNCH((k_v6_mix5m<32, 1>), mgrid, dim3(320), 0, st, a);
            else RK_LAUNCH((k_v6_mix5m<32, 2>), mgrid, dim3(320), 0, st, a);
        } else {
            if (tq == 1) RK_LAUNCH((k_v6_mix5m<64, 1>), mgrid, dim3(320), 0, st, a);
            else RK_LAUNCH((k_v6_mix5m<64, 2>), mgrid, dim3(320), 0, st, a);
        }
        HIP_OK(hipGetLastError());
        return true;
    }
#define MIX5_L(DMv, TQv)                                                                  \
    do {                                                                                  \
        if (D == DMv) RK_LAUNCH((k_v6_mix5<DMv, TQv, true>), grid, dim3(320), 0, st, a); \
        else RK_LAUNCH((k_v6_mix5<DMv, TQv, false>), grid, dim3(320), 0, st, a);         \
    } while (0)
    if (D <= 32) {
        if (tq == 1) MIX5_L(32, 1);
        else if (tq == 2) MIX5_L(32, 2);
        else MIX5_L(32, 0);
    } else {
        if (tq == 1) MIX5_L(64, 1);
        else if (tq == 2) MIX5_L(64, 2);
        else MIX5_L(64, 0);
    }
#undef MIX5_L
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v4 wkv
__global__ __launch_bounds__(256) void k_wkv4(int T, int C, const float * r, const float * k, const float * v,
                                              const float * first, const float * decay, const float * sin,
                                              float * sout, ActBuf out, int bs) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if ((int)(blockIdx.x * blockDim.x + (threadIdx.x & ~63)) >= C) return;
    // batch (bs > 0): token blockIdx.y is its own context with its state at blockIdx.y * bs
    const int t0 = bs ? (int)blockIdx.y : 0, t1 = bs ? t0 + 1 : T;
    sin += (size_t)t0 * bs;
    sout += (size_t)t0 * bs;
    float aa = sin[2 * C + c], bb = sin[3 * C + c], pp = sin[4 * C + c];
    const float fi = first[c], de = decay[c];
    for (int t = t0; t < t1; t++) {
        const size_t i = (size_t)t * C + c;
        const float kt = k[i], vt = v[i];
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
        emit32(out, t, c, r[i] * (an / bn));
    }
    sout[2 * C + c] = aa;
    sout[3 * C + c] = bb;
    sout[4 * C + c] = pp;
}

// Sequence form (T > 1, one context): the same per-channel recurrence, one wave per 64 channels.
// The k / v / r rows of the next WKV4_TT tokens are loaded while the current ones are computed
// (the recurrence's dependent chain no longer waits on a load round trip per token), and the
// outputs of a chunk are emitted after its recurrence steps, off the chain.  Per channel and
// token the operations are k_wkv4's, in its order, so decode and sequence stay bit-identical.
constexpr int WKV4_TT = 16;
__global__ __launch_bounds__(64) void k_wkv4_seq(int T, int C, const float * r, const float * k, const float * v,
                                                 const float * first, const float * decay, const float * sin,
                                                 float * sout, ActBuf out) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    const int cl = min(c, C - 1);
    float aa = sin[2 * C + cl], bb = sin[3 * C + cl], pp = sin[4 * C + cl];
    const float fi = first[cl], de = decay[cl];
    float kn[WKV4_TT], vn[WKV4_TT], rn[WKV4_TT];
    auto load = [&](int t0) {
#pragma unroll
        for (int tt = 0; tt < WKV4_TT; tt++) {
            const size_t i = (size_t)min(t0 + tt, T - 1) * C + cl;
            kn[tt] = k[i];
            vn[tt] = v[i];
            rn[tt] = r[i];
        }
    };
    load(0);
#pragma unroll 1
    for (int t0 = 0; t0 < T; t0 += WKV4_TT) {
        float kc[WKV4_TT], vc[WKV4_TT], rc[WKV4_TT], y[WKV4_TT];
#pragma unroll
        for (int tt = 0; tt < WKV4_TT; tt++) kc[tt] = kn[tt], vc[tt] = vn[tt], rc[tt] = rn[tt];
        if (t0 + WKV4_TT < T) load(t0 + WKV4_TT);
        const int n = min(WKV4_TT, T - t0);
#pragma unroll
        for (int tt = 0; tt < WKV4_TT; tt++) {
            if (tt < n) {  // uniform
                const float kt = kc[tt], vt = vc[tt];
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
                y[tt] = rc[tt] * (an / bn);
            }
        }
#pragma unroll
        for (int tt = 0; tt < WKV4_TT; tt++)
            if (tt < n) emit32(out, t0 + tt, c, y[tt]);
    }
    if (c < C) {
        sout[2 * C + c] = aa;
        sout[3 * C + c] = bb;
        sout[4 * C + c] = pp;
    }
}

bool launch_wkv4(hipStream_t st, int T, int C, const float * r, const float * k, const float * v,
                 const float * first, const float * decay, const float * state_in, float * state_out,
                 const ActBuf & out, int bs) {
    if (T > 1 && !bs && C % 64 == 0) {  // whole waves of channels
        RK_LAUNCH(k_wkv4_seq, dim3((C + 63) / 64), dim3(64), 0, st, T, C, r, k, v, first, decay, state_in,
                           state_out, out);
        HIP_OK(hipGetLastError());
        return true;
    }
    RK_LAUNCH(k_wkv4, dim3((C + 255) / 256, bs ? T : 1), dim3(256), 0, st, T, C, r, k, v, first, decay,
                       state_in, state_out, out, bs);
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- wkv6 (v5/v6)
// One workgroup per head; lane group (j, g): j = value index, g splits the key index i.
// The state column S[i][j] for the lane's IPG keys lives in registers across all T tokens.
template <int IPG>
__global__ void k_wkv6(int T, int H, int S, int G, const float * k, const float * v, const float * r,
                       const float * u, const float * w, int w_per_token, const float * sin, float * sout,
                       float * y, int bs) {
    const int h = blockIdx.x;
    const int j = threadIdx.x / G, g = threadIdx.x % G;
    const int C = H * S;
    if (bs) {  // batch: context blockIdx.z, one token
        const size_t o = (size_t)blockIdx.z * C;
        k += o, v += o, r += o, y += o;
        if (w_per_token) w += o;
        sin += (size_t)blockIdx.z * bs;
        sout += (size_t)blockIdx.z * bs;
        T = 1;
    }
    float st[IPG];
    const size_t hb = (size_t)h * S * S;
#pragma unroll
    for (int ii = 0; ii < IPG; ii++) st[ii] = sin[hb + (size_t)(g * IPG + ii) * S + j];
    float uu[IPG];
#pragma unroll
    for (int ii = 0; ii < IPG; ii++) uu[ii] = u[h * S + g * IPG + ii];
    for (int t = 0; t < T; t++) {
        const size_t th = (size_t)t * C + (size_t)h * S;
        const float * wt = w + (w_per_token ? (size_t)t * C : 0) + (size_t)h * S;
        const float vj = v[th + j];
        float acc = 0.0f;
#pragma unroll
        for (int ii = 0; ii < IPG; ii++) {
            const int i = g * IPG + ii;
            const float kv = vj * k[th + i];
            const float prev = st[ii];
            const float temp = kv * uu[ii] + prev;
            acc += temp * r[th + i];
            st[ii] = prev * wt[i] + kv;
        }
        acc = group_sum(acc, G);
        if (g == 0) y[th + j] = acc;
    }
#pragma unroll
    for (int ii = 0; ii < IPG; ii++) sout[hb + (size_t)(g * IPG + ii) * S + j] = st[ii];
}

static int pick_groups(int S) {
    int G = 256 / S;
    if (G > S) G = S;
    if (G < 1) G = 1;
    return G;
}

typedef float f2_t __attribute__((ext_vector_type(2)));

// Head size 64 (every released v5/v6 model), four keys per lane.  Workgroup = 4 waves over 16
// value columns of one head, grid (H, 4).  Lane (g = lane >> 4, jl = (lane >> 2) & 3, q = lane & 3)
// of wave wv owns column j = 16*blockIdx.y + 4*wv + jl for keys i = 16g + 4q + e (e < 4): the
// per-element arithmetic is k_att6_dec's (packed pairs, the same IEEE mul / add per element, no
// contraction).  The output sum has k_att6_dec's association exactly: each lane sums its 4 keys
// in order starting from 0 (p_q), the quad folds them as (p0 + p1) + (p2 + p3) (DPP quad
// permutes xor 1, xor 2; float addition commutes, so every lane of the quad holds the same bits),
// and the 4 key groups are folded with fold_g4 ((s0 + s2) + (s1 + s3)): 8 dependent VALU ops per
// token instead of a 16-add chain through the lanes.  Chunks of 64 tokens of k, r, w and v
// are staged in LDS with coalesced loads, the next chunk in flight while this one runs.

// Sum over the four lane groups g = lane >> 4: partner g ^ 2 (permlane32 swap), then g ^ 1
// (permlane16 swap) -- the (p0 + p2) + (p1 + p3) of group_sum(., 4) on adjacent lanes.
__device__ __forceinline__ float fold_g4(float v) {
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
    v = __int_as_float(a[0]) + __int_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float(b[0]) + __int_as_float(b[1]);
}

// v + (v of lane ^ 1) and v + (v of lane ^ 2) inside each quad
__device__ __forceinline__ float quad_add_x1(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_add_x2(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}

// acc continued over the lane's 4 terms in order
__device__ __forceinline__ float chain4(float acc, const f2_t (&x)[2]) {
    acc += x[0].x;
    acc += x[0].y;
    acc += x[1].x;
    acc += x[1].y;
    return acc;
}

// wkv6 chunk: 64 tokens, so the next chunk's loads have a whole chunk of compute to land in
constexpr int WKV6_TC = 64;
constexpr int WKV6_PAD = 8;  // >= 2 * the token group

template <bool WPT, int NWV>
__global__ __launch_bounds__(64 * NWV) void k_wkv6_s64(int T, int H, const float * k, const float * v, const float * r,
                                                       const float * u, const float * w, const float * sin, float * sout,
                                                       float * y, int bs) {
    constexpr int S = 64;
    if (bs) {  // batch: context blockIdx.z, one token
        const size_t o = (size_t)blockIdx.z * H * S;
        k += o, v += o, r += o, y += o;
        if (WPT) w += o;
        sin += (size_t)blockIdx.z * bs;
        sout += (size_t)blockIdx.z * bs;
        T = 1;
    }
    constexpr int CW = 4 * NWV, NT = 64 * NWV, QQ = WKV6_TC * 16 / NT;
    // WKV6_PAD rows past the chunk: a full chunk's look-ahead reads need no clamp (their tokens
    // are never used)
    constexpr int RW = WKV6_TC + WKV6_PAD;
    __shared__ __attribute__((aligned(16))) float sk[RW][S], sr[RW][S], sw[WPT ? RW : 1][S], sv[RW][CW],
        sy[WKV6_TC][CW];
    const int h = blockIdx.x, jb = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int q = lane & 3, jl = (lane >> 2) & 3, g = lane >> 4;
    const int jc = 4 * wv + jl, j = jb * CW + jc, i0 = g * 16 + 4 * q;
    const int C = H * S;
    const size_t hb = (size_t)h * S * S;
    f2_t st[2], uu[2], wc[2];
#pragma unroll
    for (int p = 0; p < 2; p++) {
        const int i = i0 + 2 * p;
        st[p] = f2_t{sin[hb + (size_t)i * S + j], sin[hb + (size_t)(i + 1) * S + j]};
        uu[p] = f2_t{u[h * S + i], u[h * S + i + 1]};
        wc[p] = WPT ? f2_t{0.f, 0.f} : f2_t{w[h * S + i], w[h * S + i + 1]};
    }
    // chunk staging: k/r/w rows of 64 floats = 16 float4 per token; thread moves float4
    // #(tid & 15) of tokens (tid >> 4) + (NT/16) qq, qq < QQ; v: CW columns = NWV float4 per
    // token, threads < WKV6_TC*NWV move float4 #(tid % NWV) of token tid / NWV
    // QQ == 4 (4 waves, the default): the chunk's rows in named registers -- as arrays they are
    // kept in scratch
    float4 pk[QQ == 4 ? 1 : QQ], pr[QQ == 4 ? 1 : QQ], pw[WPT && QQ != 4 ? QQ : 1], pv;
    float4 k0, k1, k2, k3, r0, r1, r2, r3, w0, w1, w2, w3;
#define WKV6_LD(QI, KV, RV, WV)                                                                           \
    do {                                                                                                  \
        const int t = min(t0 + (tid >> 4) + (NT / 16) * (QI), T - 1);                                     \
        const size_t base = (size_t)t * C + (size_t)h * S + 4 * (tid & 15);                               \
        KV = *(const float4 *)(k + base);                                                                 \
        RV = *(const float4 *)(r + base);                                                                 \
        if constexpr (WPT) WV = *(const float4 *)(w + base);                                              \
    } while (0)
#define WKV6_ST(QI, KV, RV, WV)                                                                           \
    do {                                                                                                  \
        const int tt = (tid >> 4) + (NT / 16) * (QI);                                                     \
        *(float4 *)&sk[tt][4 * (tid & 15)] = KV;                                                          \
        *(float4 *)&sr[tt][4 * (tid & 15)] = RV;                                                          \
        if constexpr (WPT) *(float4 *)&sw[tt][4 * (tid & 15)] = WV;                                       \
    } while (0)
    auto load_chunk = [&](int t0) __attribute__((always_inline)) {
        if constexpr (QQ == 4) {
            WKV6_LD(0, k0, r0, w0);
            WKV6_LD(1, k1, r1, w1);
            WKV6_LD(2, k2, r2, w2);
            WKV6_LD(3, k3, r3, w3);
        } else {
#pragma unroll
            for (int qq = 0; qq < QQ; qq++) WKV6_LD(qq, pk[qq], pr[qq], pw[qq]);
        }
        const int tv = min(tid, WKV6_TC * NWV - 1);
        const int t = min(t0 + tv / NWV, T - 1);
        pv = *(const float4 *)(v + (size_t)t * C + (size_t)h * S + jb * CW + 4 * (tv % NWV));
    };
    auto store_chunk = [&]() __attribute__((always_inline)) {
        if constexpr (QQ == 4) {
            WKV6_ST(0, k0, r0, w0);
            WKV6_ST(1, k1, r1, w1);
            WKV6_ST(2, k2, r2, w2);
            WKV6_ST(3, k3, r3, w3);
        } else {
#pragma unroll
            for (int qq = 0; qq < QQ; qq++) WKV6_ST(qq, pk[qq], pr[qq], pw[qq]);
        }
        if (tid < WKV6_TC * NWV) *(float4 *)&sv[tid / NWV][4 * (tid % NWV)] = pv;
    };
#undef WKV6_LD
#undef WKV6_ST
    struct Tok {
        f2_t k[2], r[2], w[2];
        float v;
    };
    auto read_tok = [&](Tok & o, int tt) __attribute__((always_inline)) {
        const float4 a = *(const float4 *)&sk[tt][i0];
        const float4 b = *(const float4 *)&sr[tt][i0];
        o.k[0] = f2_t{a.x, a.y}, o.k[1] = f2_t{a.z, a.w};
        o.r[0] = f2_t{b.x, b.y}, o.r[1] = f2_t{b.z, b.w};
        if constexpr (WPT) {
            const float4 c = *(const float4 *)&sw[tt][i0];
            o.w[0] = f2_t{c.x, c.y}, o.w[1] = f2_t{c.z, c.w};
        }
        o.v = sv[tt][jc];
    };
    load_chunk(0);
    for (int t0 = 0; t0 < T; t0 += WKV6_TC) {
        store_chunk();
        __syncthreads();
        if (t0 + WKV6_TC < T) load_chunk(t0 + WKV6_TC);  // in flight during this chunk
        const int n = min(WKV6_TC, T - t0);
        // Tokens in groups of TG: the state updates run token after token, then the TG output
        // chains (independent of each other) are interleaved step by step.
        constexpr int TG = 4;
        static_assert(2 * TG <= WKV6_PAD, "look-ahead rows");
        // FULL: a whole chunk (n == WKV6_TC), every token valid
        auto group = [&](const Tok (&o)[TG], int tt0, auto full) __attribute__((always_inline)) {
            constexpr bool FULL = decltype(full)::value;
            f2_t x[TG][2];
#pragma unroll
            for (int e = 0; e < TG; e++) {
                const bool val = FULL || tt0 + e < n;
                const f2_t vj = f2_t{o[e].v, o[e].v};
                f2_t kv[2];
#pragma unroll
                for (int p = 0; p < 2; p++) kv[p] = vj * o[e].k[p];
#pragma unroll
                for (int p = 0; p < 2; p++) x[e][p] = kv[p] * uu[p];
#pragma unroll
                for (int p = 0; p < 2; p++) x[e][p] = x[e][p] + st[p];
#pragma unroll
                for (int p = 0; p < 2; p++) x[e][p] = x[e][p] * o[e].r[p];
#pragma unroll
                for (int p = 0; p < 2; p++) {
                    f2_t ns = st[p] * (WPT ? o[e].w[p] : wc[p]);
                    ns = ns + kv[p];
                    st[p] = val ? ns : st[p];
                }
            }
            // p_q (4 keys in order), (p0 + p1) + (p2 + p3) over the quad, TG sums side by side
            float acc[TG];
#pragma unroll
            for (int e = 0; e < TG; e++) acc[e] = chain4(0.0f, x[e]);
#pragma unroll
            for (int e = 0; e < TG; e++) acc[e] = quad_add_x1(acc[e]);
#pragma unroll
            for (int e = 0; e < TG; e++) acc[e] = quad_add_x2(acc[e]);
            // every lane of the column holds the same sum: all write it to the chunk's y tile
#pragma unroll
            for (int e = 0; e < TG; e++) {
                acc[e] = fold_g4(acc[e]);
                if (FULL || tt0 + e < n) sy[tt0 + e][jc] = acc[e];
            }
        };
        // two operand sets in turn: the next group's LDS reads overlap this group's arithmetic
        Tok A[TG], B[TG];
        if (n == WKV6_TC) {
            const std::integral_constant<bool, true> full;
#pragma unroll
            for (int e = 0; e < TG; e++) read_tok(A[e], e);
            for (int tt = 0; tt < WKV6_TC; tt += 2 * TG) {
#pragma unroll
                for (int e = 0; e < TG; e++) read_tok(B[e], tt + TG + e);
                group(A, tt, full);
#pragma unroll
                for (int e = 0; e < TG; e++) read_tok(A[e], tt + 2 * TG + e);
                group(B, tt + TG, full);
            }
        } else {
            const std::integral_constant<bool, false> part;
#pragma unroll
            for (int e = 0; e < TG; e++) read_tok(A[e], min(e, n - 1));
            for (int tt = 0; tt < n; tt += 2 * TG) {
#pragma unroll
                for (int e = 0; e < TG; e++) read_tok(B[e], min(tt + TG + e, n - 1));
                group(A, tt, part);
                if (tt + TG >= n) break;
#pragma unroll
                for (int e = 0; e < TG; e++) read_tok(A[e], min(tt + 2 * TG + e, n - 1));
                group(B, tt + TG, part);
            }
        }
        __syncthreads();
        // the chunk's y tile [n tokens][CW columns], one float4 per thread
        {
            const int tk = tid / NWV;
            if (tk < n)
                *(float4 *)(y + (size_t)(t0 + tk) * C + (size_t)h * S + jb * CW + 4 * (tid % NWV)) =
                    *(const float4 *)&sy[tk][4 * (tid % NWV)];
        }
    }
#pragma unroll
    for (int p = 0; p < 2; p++) {
        const int i = i0 + 2 * p;
        sout[hb + (size_t)i * S + j] = st[p].x;
        sout[hb + (size_t)(i + 1) * S + j] = st[p].y;
    }
}

int g_wkv6_nwv = 4;  // waves per workgroup of k_wkv6_s64 (tools/wkv_probe.hip varies it)

bool launch_wkv6(hipStream_t st, int T, int H, int S, const float * k, const float * v, const float * r,
                 const float * u, const float * w, int w_per_token, const float * state_in, float * state_out,
                 float * y, int bs) {
    const int nz = bs ? T : 1;
    if (S == 64) {
#define WKV6_L(P, N) RK_LAUNCH((k_wkv6_s64<P, N>), dim3(H, 16 / (N), nz), dim3(64 * (N)), 0, st, T, H, k, v, r, u, w, state_in, state_out, y, bs)
        const int nwv = g_wkv6_nwv;
        if (w_per_token) {
            if (nwv == 1) WKV6_L(true, 1);
            else if (nwv == 2) WKV6_L(true, 2);
            else WKV6_L(true, 4);
        } else {
            if (nwv == 1) WKV6_L(false, 1);
            else if (nwv == 2) WKV6_L(false, 2);
            else WKV6_L(false, 4);
        }
#undef WKV6_L
        HIP_OK(hipGetLastError());
        return true;
    }
    const int G = pick_groups(S), IPG = S / G;
    dim3 grid(H, 1, nz), block(S * G);
    switch (IPG) {
        case 1: RK_LAUNCH(k_wkv6<1>, grid, block, 0, st, T, H, S, G, k, v, r, u, w, w_per_token, state_in, state_out, y, bs); break;
        case 2: RK_LAUNCH(k_wkv6<2>, grid, block, 0, st, T, H, S, G, k, v, r, u, w, w_per_token, state_in, state_out, y, bs); break;
        case 4: RK_LAUNCH(k_wkv6<4>, grid, block, 0, st, T, H, S, G, k, v, r, u, w, w_per_token, state_in, state_out, y, bs); break;
        case 8: RK_LAUNCH(k_wkv6<8>, grid, block, 0, st, T, H, S, G, k, v, r, u, w, w_per_token, state_in, state_out, y, bs); break;
        case 16: RK_LAUNCH(k_wkv6<16>, grid, block, 0, st, T, H, S, G, k, v, r, u, w, w_per_token, state_in, state_out, y, bs); break;
        case 32: RK_LAUNCH(k_wkv6<32>, grid, block, 0, st, T, H, S, G, k, v, r, u, w, w_per_token, state_in, state_out, y, bs); break;
        default: fprintf(stderr, "rwkv: unsupported head size %d\n", S); return false;
    }
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v7
// Per token: thread per channel, heads are S consecutive channels (S <= 64, power of two).
__global__ __launch_bounds__(256) void k_v7_prep(int T, int H, int S, float * k, const float * a, const float * r,
                                                 const float * k_k, const float * k_a, const float * r_k, float * nb,
                                                 float * bb, float * bonus) {
    const int t = blockIdx.x, C = H * S;
    // one 256-channel block (whole heads) per grid.y: no serial walk over the channel blocks
    {
        const int c0 = (int)blockIdx.y * blockDim.x, c = c0 + threadIdx.x;
        if (c0 + (int)(threadIdx.x & ~63) >= C) return;  // whole wave out of range
        const size_t i = (size_t)t * C + c;
        const float kv = k[i];
        const float kkr = kv * k_k[c];
        const float sum = group_sum(kkr * kkr, S);
        const float scale = 1.0f / fmaxf(sqrtf(sum), 1e-12f);
        const float kk = kkr * scale;
        const float av = a[i];
        const float ka = kv * k_a[c];
        const float kadj = kv + (av * ka - ka);
        k[i] = kadj;
        nb[i] = -kk;
        bb[i] = kk * av;
        const float bsum = group_sum((kadj * r[i]) * r_k[c], S);
        if ((c % S) == 0) bonus[(size_t)t * H + c / S] = bsum;
    }
}

bool launch_v7_prep(hipStream_t st, int T, int H, int S, float * k, const float * a, const float * r,
                    const float * k_k, const float * k_a, const float * r_k, float * nb, float * bb, float * bonus) {
    if (S > 64 || (S & (S - 1))) {
        fprintf(stderr, "rwkv: v7 head size %d unsupported\n", S);
        return false;
    }
    RK_LAUNCH(k_v7_prep, dim3(T, (H * S + 255) / 256), dim3(256), 0, st, T, H, S, k, a, r, k_k, k_a, r_k, nb,
                       bb, bonus);
    HIP_OK(hipGetLastError());
    return true;
}

// state [h][i(value)][j(key)]; lane group (i, g): g splits j.
template <int JPG>
__global__ void k_wkv7(int T, int H, int S, int G, const float * r, const float * w, const float * k,
                       const float * v, const float * a, const float * b, const float * sin, float * sout,
                       float * y, int bs) {
    const int h = blockIdx.x;
    const int i = threadIdx.x / G, g = threadIdx.x % G;
    const int C = H * S;
    if (bs) {  // batch: context blockIdx.z, one token
        const size_t o = (size_t)blockIdx.z * C;
        r += o, w += o, k += o, v += o, a += o, b += o, y += o;
        sin += (size_t)blockIdx.z * bs;
        sout += (size_t)blockIdx.z * bs;
        T = 1;
    }
    const size_t hb = (size_t)h * S * S + (size_t)i * S + g * JPG;
    float st[JPG];
#pragma unroll
    for (int jj = 0; jj < JPG; jj++) st[jj] = sin[hb + jj];
    for (int t = 0; t < T; t++) {
        const size_t th = (size_t)t * C + (size_t)h * S + g * JPG;
        float sa = 0.0f;
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) sa += a[th + jj] * st[jj];
        sa = group_sum(sa, G);
        const float vi = v[(size_t)t * C + (size_t)h * S + i];
        float acc = 0.0f;
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) {
            const float kv = vi * k[th + jj];
            const float ns = st[jj] * w[th + jj] + kv + sa * b[th + jj];
            st[jj] = ns;
            acc += ns * r[th + jj];
        }
        acc = group_sum(acc, G);
        if (g == 0) y[(size_t)t * C + (size_t)h * S + i] = acc;
    }
#pragma unroll
    for (int jj = 0; jj < JPG; jj++) sout[hb + jj] = st[jj];
}

// Head size 64: keys in 16 groups of 4 (k_att7_dec's split for S = 64, G = 16).  Workgroup = 4
// waves over 16 value rows of one head, grid (H, 4); lane (g = lane & 15, il = 4 wv + (lane >> 4))
// owns row i = 16 blockIdx.y + il, keys j = 4g .. 4g + 3.  Per token: sa = sum_j a_j s_ij (4 terms
// in order from 0, then the 16 groups folded by the butterfly xor 8, 4, 2, 1 -- DPP row rotations,
// every lane of the row ends with the same bits), the state update, and the output sum the same
// way.  r, w, k, a, b (and v) come in 16-token chunks staged in a double-buffered LDS tile (the next
// chunk in registers while the current one runs); y goes through an LDS tile, one store per chunk.
constexpr int WKV7_TC = 16;

// v + v(lane + 8 mod 16) + ... over a 16-lane DPP row: the butterfly of group_sum(., 16)
__device__ __forceinline__ float row_bfly16(float v) {
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, false));
    return v;
}

__global__ __launch_bounds__(256) void k_wkv7_s64(int T, int H, const float * r, const float * w, const float * k,
                                                  const float * v, const float * a, const float * b,
                                                  const float * sin, float * sout, float * y, int bs) {
    constexpr int S = 64;
    if (bs) {  // batch: context blockIdx.z, one token
        const size_t o = (size_t)blockIdx.z * H * S;
        r += o, w += o, k += o, v += o, a += o, b += o, y += o;
        sin += (size_t)blockIdx.z * bs;
        sout += (size_t)blockIdx.z * bs;
        T = 1;
    }
    __shared__ __attribute__((aligned(16))) float sr[2][WKV7_TC][S], sw[2][WKV7_TC][S], sk[2][WKV7_TC][S],
        sa_[2][WKV7_TC][S], sb[2][WKV7_TC][S], sv[2][WKV7_TC][16], sy[2][WKV7_TC][16];
    const int h = blockIdx.x, ib = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int g = lane & 15, il = 4 * wv + (lane >> 4), i = ib * 16 + il;
    const int C = H * S;
    const size_t hb = (size_t)h * S * S + (size_t)i * S + 4 * g;
    float st[4];
#pragma unroll
    for (int e = 0; e < 4; e++) st[e] = sin[hb + e];  // (state slices need not be 16-byte aligned)
    // staging: thread moves float4 #(tid & 15) of token (tid >> 4) of the five key-indexed rows;
    // threads < 64 one float4 of v (token tid >> 2, rows 4 (tid & 3) ..)
    float4 q0, q1, q2, q3, q4, qv;
    const int c4 = 4 * (tid & 15), tl = tid >> 4;
    auto load = [&](int t0) __attribute__((always_inline)) {
        const int t = min(t0 + tl, T - 1);
        const size_t base = (size_t)t * C + (size_t)h * S + c4;
        q0 = *(const float4 *)(r + base);
        q1 = *(const float4 *)(w + base);
        q2 = *(const float4 *)(k + base);
        q3 = *(const float4 *)(a + base);
        q4 = *(const float4 *)(b + base);
        if (tid < 64) {
            const int tv = min(t0 + (tid >> 2), T - 1);
            qv = *(const float4 *)(v + (size_t)tv * C + (size_t)h * S + ib * 16 + 4 * (tid & 3));
        }
    };
    auto store = [&](int bf) __attribute__((always_inline)) {
        *(float4 *)&sr[bf][tl][c4] = q0;
        *(float4 *)&sw[bf][tl][c4] = q1;
        *(float4 *)&sk[bf][tl][c4] = q2;
        *(float4 *)&sa_[bf][tl][c4] = q3;
        *(float4 *)&sb[bf][tl][c4] = q4;
        if (tid < 64) *(float4 *)&sv[bf][tid >> 2][4 * (tid & 3)] = qv;
    };
    load(0);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int t0 = 0; t0 < T; t0 += WKV7_TC) {
        const int n = min(WKV7_TC, T - t0);
        const bool nx = t0 + WKV7_TC < T;
        if (nx) load(t0 + WKV7_TC);  // in flight during this chunk
        // token tt's operands are in registers while token tt + 1's are read (the LDS latency stays
        // off the recurrence's critical path); whole chunks fully unrolled
        struct Op {
            float4 a, k, w, b, r;
            float v;
        };
        auto rd = [&](Op & o, int tt) __attribute__((always_inline)) {
            o.a = *(const float4 *)&sa_[buf][tt][4 * g];
            o.k = *(const float4 *)&sk[buf][tt][4 * g];
            o.w = *(const float4 *)&sw[buf][tt][4 * g];
            o.b = *(const float4 *)&sb[buf][tt][4 * g];
            o.r = *(const float4 *)&sr[buf][tt][4 * g];
            o.v = sv[buf][tt][il];
        };
        auto tok = [&](const Op & o, int tt) __attribute__((always_inline)) {
            float sa = 0.0f;
            sa += o.a.x * st[0];
            sa += o.a.y * st[1];
            sa += o.a.z * st[2];
            sa += o.a.w * st[3];
            sa = row_bfly16(sa);
            const float kk[4] = {o.k.x, o.k.y, o.k.z, o.k.w}, ww[4] = {o.w.x, o.w.y, o.w.z, o.w.w};
            const float bb[4] = {o.b.x, o.b.y, o.b.z, o.b.w}, rr[4] = {o.r.x, o.r.y, o.r.z, o.r.w};
            float acc = 0.0f;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const float kv = o.v * kk[e];
                const float ns = st[e] * ww[e] + kv + sa * bb[e];
                st[e] = ns;
                acc += ns * rr[e];
            }
            acc = row_bfly16(acc);
            if (g == 0) sy[buf][tt][il] = acc;
        };
        Op cur, nxt;
        rd(cur, 0);
        if (n == WKV7_TC) {
            // two tokens ahead: token tt + 2's LDS reads are issued before token tt's chain, so the
            // recurrence never waits on the LDS
            Op ring[3];
            ring[0] = cur;
            rd(ring[1], 1);
#pragma unroll
            for (int tt = 0; tt < WKV7_TC; tt++) {
                if (tt + 2 < WKV7_TC) rd(ring[(tt + 2) % 3], tt + 2);
                tok(ring[tt % 3], tt);
            }
        } else {
#pragma unroll 1
            for (int tt = 0; tt < n; tt++) {
                rd(nxt, min(tt + 1, n - 1));
                tok(cur, tt);
                cur = nxt;
            }
        }
        if (nx) store(buf ^ 1);
        __syncthreads();
        // the chunk's y tile [n tokens][16 rows]: threads < 64 one float4
        if (tid < 64 && (tid >> 2) < n)
            *(float4 *)(y + (size_t)(t0 + (tid >> 2)) * C + (size_t)h * S + ib * 16 + 4 * (tid & 3)) =
                *(const float4 *)&sy[buf][tid >> 2][4 * (tid & 3)];
        buf ^= 1;
    }
#pragma unroll
    for (int e = 0; e < 4; e++) sout[hb + e] = st[e];
}

bool launch_wkv7(hipStream_t st, int T, int H, int S, const float * r, const float * w, const float * k,
                 const float * v, const float * a, const float * b, const float * state_in, float * state_out,
                 float * y, int bs) {
    const int nz = bs ? T : 1;
    if (S == 64) {
        RK_LAUNCH(k_wkv7_s64, dim3(H, 4, nz), dim3(256), 0, st, T, H, r, w, k, v, a, b, state_in, state_out, y,
                           bs);
        HIP_OK(hipGetLastError());
        return true;
    }
    const int G = pick_groups(S), JPG = S / G;
    dim3 grid(H, 1, nz), block(S * G);
    switch (JPG) {
        case 1: RK_LAUNCH(k_wkv7<1>, grid, block, 0, st, T, H, S, G, r, w, k, v, a, b, state_in, state_out, y, bs); break;
        case 2: RK_LAUNCH(k_wkv7<2>, grid, block, 0, st, T, H, S, G, r, w, k, v, a, b, state_in, state_out, y, bs); break;
        case 4: RK_LAUNCH(k_wkv7<4>, grid, block, 0, st, T, H, S, G, r, w, k, v, a, b, state_in, state_out, y, bs); break;
        case 8: RK_LAUNCH(k_wkv7<8>, grid, block, 0, st, T, H, S, G, r, w, k, v, a, b, state_in, state_out, y, bs); break;
        case 16: RK_LAUNCH(k_wkv7<16>, grid, block, 0, st, T, H, S, G, r, w, k, v, a, b, state_in, state_out, y, bs); break;
        case 32: RK_LAUNCH(k_wkv7<32>, grid, block, 0, st, T, H, S, G, r, w, k, v, a, b, state_in, state_out, y, bs); break;
        default: fprintf(stderr, "rwkv: unsupported head size %d\n", S); return false;
    }
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- GroupNorm
template <int TQ>
__global__ __launch_bounds__(1024) void k_groupnorm(int T, int H, int S, float eps, const float * y, const float * w,
                                                    const float * b, int mode, const float * g, const float * v,
                                                    const float * bonus, ActBuf out) {
    const int t = blockIdx.x * TOKS_PER_WG + (threadIdx.x >> 8), C = H * S, tid = threadIdx.x & 255;
    if (t >= T) return;
    // channel block of 256 (4 heads of 64) per grid.y: one channel per thread
    {
        const int c0 = (int)blockIdx.y * 256, c = c0 + tid;
        if (c0 + (tid & ~63) >= C) return;  // whole wave out of range
        const size_t i = (size_t)t * C + c;
        const float x = y[i];
        const double s = group_tree_sum_d((double)x, S);
        const float mean = (float)div_count(s, S);
        const float d = x - mean;
        const double s2 = group_tree_sum_d((double)(d * d), S);
        const float var = (float)div_count(s2, S);
        const float scale = 1.0f / sqrtf(var + eps);
        float o = d * scale;
        o = o * w[c];
        o = o + b[c];
        if (mode == 2) o = o + v[i] * bonus[(size_t)t * H + c / S];
        if (mode >= 1) o = o * g[i];
        if constexpr (TQ > 0) emit32_tile<TQ>(out.tq, C, t, c, o);
        else emit32(out, t, c, o);
    }
}

bool launch_groupnorm(hipStream_t st, int T, int H, int S, float eps, const float * y, const float * w,
                      const float * b, int mode, const float * g, const float * v, const float * bonus,
                      const ActBuf & out) {
    if (S > 64 || (S & (S - 1))) {
        fprintf(stderr, "rwkv: head size %d unsupported by groupnorm\n", S);
        return false;
    }
    const dim3 grid((T + TOKS_PER_WG - 1) / TOKS_PER_WG, (H * S + 255) / 256), block(256 * TOKS_PER_WG);
    const int tq = tile_q(&out, 1, H * S);
    if (tq == 1) RK_LAUNCH(k_groupnorm<1>, grid, block, 0, st, T, H, S, eps, y, w, b, mode, g, v, bonus, out);
    else if (tq == 2) RK_LAUNCH(k_groupnorm<2>, grid, block, 0, st, T, H, S, eps, y, w, b, mode, g, v, bonus, out);
    else RK_LAUNCH(k_groupnorm<0>, grid, block, 0, st, T, H, S, eps, y, w, b, mode, g, v, bonus, out);
    HIP_OK(hipGetLastError());
    return true;
}

__global__ void k_fill(float * p, size_t n, float value) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = value;
}

bool launch_fill(hipStream_t st, float * p, size_t n, float value) {
    if (!n) return true;
    RK_LAUNCH(k_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, n, value);
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi

namespace rwkvmi {

template <int TQ>
__global__ __launch_bounds__(1024) void k_act_from_f32(const float * x, int T, int K, ActBuf out) {
    const int t = blockIdx.x * TOKS_PER_WG + (threadIdx.x >> 8), tid = threadIdx.x & 255;
    if (t >= T) return;
    // 256-channel blocks split over grid.y (v7-2.9B FFN value input, K = 10240: 31 -> 25 us)
    for (int k0 = (int)blockIdx.y * 256; k0 < K; k0 += (int)gridDim.y * 256) {
        const int k = k0 + tid;
        if (k0 + (tid & ~31) >= K) continue;  // half-wave uniform (K % 32 == 0)
        if constexpr (TQ > 0) emit32_tile<TQ>(out.tq, K, t, k, x[(size_t)t * K + k]);
        else emit32(out, t, k, x[(size_t)t * K + k]);
    }
}
bool launch_act_from_f32(hipStream_t st, const float * x, int T, int K, const ActBuf & out) {
    if (K % 32) return false;
    const dim3 grid((T + TOKS_PER_WG - 1) / TOKS_PER_WG, std::min((K + 255) / 256, 8)), block(256 * TOKS_PER_WG);
    const int tq = tile_q(&out, 1, K);
    if (tq == 1) RK_LAUNCH(k_act_from_f32<1>, grid, block, 0, st, x, T, K, out);
    else if (tq == 2) RK_LAUNCH(k_act_from_f32<2>, grid, block, 0, st, x, T, K, out);
    else RK_LAUNCH(k_act_from_f32<0>, grid, block, 0, st, x, T, K, out);
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
