// mv_fmfma.hip -- float-weight (F16 / F32) matmuls over many tokens or contexts on the f32-input
// MFMA, in the decode matvec's association.
//
// The decode matvec (k_mv / k_mva / k_mvb / k_mm) gives lane l of a row the 16-byte units
// k = 8l + 512u (F16: 8 halves) or 4l + 256u (F32: 4 floats), accumulates each unit's elements in
// order with fmaf onto one partial (F16 operands widened exactly), and folds the 64 lane partials
// with wave_sum63's perfect binary tree.  v_mfma_f32_16x16x4_f32 computes, for every (row, column)
// of a 16 x 16 tile, exactly the fmaf chain over its 4 k values in order, starting from the C
// operand (tools/mfma_f32_probe.hip: 307,200 of 307,200 outputs bitwise over three operand
// distributions).  So the partial of class l (the lane-l partial of the matvec) for 16 rows x 16
// tokens is two MFMAs per F16 unit (one per F32 unit) chained on one accumulator, and the classes
// fold with the tree as a binary counter (qgemm.hip's order).  The products of F16 operands are
// exact in f32, so the MFMA runs the same IEEE operations as the matvec: results are bit-identical
// to the single-token decode of every token / context.
//
// Workgroup: 4 waves x 16 rows (64 rows) x 16 * NT tokens; a wave's NT 16 x 16 tiles share its
// weight loads.  Epilogue (apply_epi, y, emit32) in a workgroup pass over the tile from LDS, so an
// emitting group's 32 consecutive rows of a token sit in one half-wave.
#include "mv_common.hpp"

#include <stdlib.h>

namespace rwkvmi {

typedef float fmf4 __attribute__((ext_vector_type(4)));

template <int WF>
struct FUnit;
template <>
struct FUnit<W_F16> {  // 8 halves of a row: the A/B operands of two MFMAs
    int4 v;
    static constexpr int ELEMS = 8, STRIDE = 512;
    __device__ __forceinline__ void load(const void * base, size_t row, int K, int k) {
        v = *(const int4 *)((const __half *)base + row * K + k);
    }
    // element kk (+4 for the second MFMA) of the unit, widened
    __device__ __forceinline__ float get(int j) const {
        const int w = j >> 1 == 0 ? v.x : j >> 1 == 1 ? v.y : j >> 1 == 2 ? v.z : v.w;
        const half2_t h = __builtin_bit_cast(half2_t, w);
        return (float)((j & 1) ? h.y : h.x);
    }
};
template <>
struct FUnit<W_F32> {  // the lane's element of a 4-float unit
    float v;
    static constexpr int ELEMS = 4, STRIDE = 256;
    __device__ __forceinline__ void load(const void * base, size_t row, int K, int k) {
        v = ((const float *)base)[row * K + k];
    }
};

template <int WF, int NT>
__global__ __launch_bounds__(256) void k_fmm(MMGroup g) {
    extern __shared__ float red[];  // [16 * NT tokens][64 rows]
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MMEntry & E = g.e[e];
    const int T = g.T, M = E.W.M, K = E.W.K;
    const int tgroups = (T + 16 * NT - 1) / (16 * NT);
    const int local = (int)blockIdx.x - E.block0;
    const int rt = local / tgroups, tg = local % tgroups;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ml = lane & 15, kk = lane >> 4;
    const int row0 = rt * 64 + wave * 16, tok0 = tg * 16 * NT;
    const size_t arow = (size_t)min(row0 + ml, M - 1);
    size_t xrow[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) xrow[n] = (size_t)min(tok0 + 16 * n + ml, T - 1);
    const void * xin = WF == W_F16 ? (const void *)E.in.h : (const void *)E.in.f;
    constexpr int EL = FUnit<WF>::ELEMS, STR = FUnit<WF>::STRIDE;
    const int units = (K + STR - 1) / STR;

    fmf4 st[6][NT], c[NT], tot[NT];
#pragma unroll 1
    for (int l = 0; l < 64; l++) {
        fmf4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; n++) acc[n] = fmf4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 1
        for (int u = 0; u < units; u++) {
            const int k = EL * l + STR * u;
            if (k >= K) break;  // uniform: the class has no more units (the matvec's unit_valid)
            FUnit<WF> w;
            w.load(E.W.qs, arow, K, WF == W_F16 ? k : k + kk);
            FUnit<WF> x[NT];
#pragma unroll
            for (int n = 0; n < NT; n++) x[n].load(xin, xrow[n], K, WF == W_F16 ? k : k + kk);
            if constexpr (WF == W_F16) {
                const float a0 = w.get(kk), a1 = w.get(kk + 4);
#pragma unroll
                for (int n = 0; n < NT; n++) {
                    acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, x[n].get(kk), acc[n], 0, 0, 0);
                    acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, x[n].get(kk + 4), acc[n], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int n = 0; n < NT; n++) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.v, x[n].v, acc[n], 0, 0, 0);
            }
        }
        // binary counter over the classes (wave_sum63's tree): even classes open level 0, odd
        // classes close ctz(~l) levels
        if ((l & 1) == 0) {
#pragma unroll
            for (int n = 0; n < NT; n++) st[0][n] = acc[n];
        } else {
            const int N = __builtin_ctz(~l);
#pragma unroll
            for (int n = 0; n < NT; n++) c[n] = acc[n];
#pragma unroll
            for (int kx = 0; kx < 6; kx++)
                if (kx < N)
#pragma unroll
                    for (int n = 0; n < NT; n++) c[n] = st[kx][n] + c[n];
#pragma unroll
            for (int kx = 1; kx < 6; kx++)
                if (kx == N)
#pragma unroll
                    for (int n = 0; n < NT; n++) st[kx][n] = c[n];
            if (N == 6)
#pragma unroll
                for (int n = 0; n < NT; n++) tot[n] = c[n];
        }
    }
    // D layout: lane holds rows 4 * kk + i of the wave's 16, token ml of each 16-token tile
#pragma unroll
    for (int n = 0; n < NT; n++)
#pragma unroll
        for (int i = 0; i < 4; i++) red[(16 * n + ml) * 64 + wave * 16 + 4 * kk + i] = tot[n][i] + 0.0f;
    __syncthreads();
    const int rw0 = rt * 64;
    for (int i = threadIdx.x; i < 16 * NT * 64; i += 256) {
        const int t = tok0 + i / 64, row = rw0 + i % 64;
        if (t >= T) break;  // i / 64 only grows: the rest of the pass is past T too (half-waves whole)
        float v = 0.0f;
        if (row < M) {
            v = apply_epi(E, t, row, red[i]);
            if (E.y) E.y[(size_t)t * E.ldy + row] = v;
        }
        if (E.emit && row < M) emit32(E.out, t, row, v);  // M % 32 == 0: half-wave uniform
    }
}

// MFMA float matmul for a group: F16 / F32 weights, T >= 16 tokens (or contexts), every entry's
// input in the weight type's activation format, row-major (not tiled); emitting entries need M % 32
// == 0.  Returns false with *launched = false when the group is outside that (caller keeps k_mm).
bool launch_fmm_group(hipStream_t st, MMGroup & g, int wtype, bool * launched) {
    static const bool on = [] {
        const char * v = getenv("RWKV_MI355X_FMM");  // 0: float matmuls stay on k_mm / k_mvb
        return !(v && v[0] == '0');
    }();
    *launched = false;
    if (!on || (wtype != W_F16 && wtype != W_F32) || g.T < 16) return true;
    for (int i = 0; i < g.n; i++) {
        const MMEntry & e = g.e[i];
        if (e.W.type != wtype || e.W.K % 32 || e.in.tiled || e.in.fmt != act_fmt_for(wtype) || e.in.K != e.W.K)
            return true;
        if (e.emit && e.W.M % 32) return true;
        if (wtype == W_F16 ? !e.in.h : !e.in.f) return true;
    }
    const int NT = g.T >= 32 ? 2 : 1;
    const int tgroups = (g.T + 16 * NT - 1) / (16 * NT);
    int blocks = 0;
    for (int i = 0; i < g.n; i++) {
        g.e[i].block0 = blocks;
        blocks += (g.e[i].W.M + 63) / 64 * tgroups;
    }
    if (!blocks) return true;
    const size_t lds = (size_t)16 * NT * 64 * 4;
    if (wtype == W_F16) {
        if (NT == 2) hipLaunchKernelGGL((k_fmm<W_F16, 2>), dim3(blocks), dim3(256), lds, st, g);
        else hipLaunchKernelGGL((k_fmm<W_F16, 1>), dim3(blocks), dim3(256), lds, st, g);
    } else {
        if (NT == 2) hipLaunchKernelGGL((k_fmm<W_F32, 2>), dim3(blocks), dim3(256), lds, st, g);
        else hipLaunchKernelGGL((k_fmm<W_F32, 1>), dim3(blocks), dim3(256), lds, st, g);
    }
    HIP_OK(hipGetLastError());
    *launched = true;
    return true;
}

}  // namespace rwkvmi
