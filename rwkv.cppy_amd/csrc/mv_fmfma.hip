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
// Workgroup: 4 waves over a 64-row x 64-token tile (a wave: 2 x 2 tiles of 16 x 16).  Operands are
// staged through LDS one stage (16 steps = 16 units per row and per token) at a time: the workgroup
// loads whole 16-byte units with coalesced global loads (the next stage's in flight while the current
// one is multiplied) and writes them as [element pair kk][row][step] dword planes, so an MFMA
// operand is one conflict-free ds_read_b32 per lane.  Epilogue (apply_epi, y, emit32) in a workgroup
// pass over the tile from LDS, so an emitting group's 32 consecutive rows of a token sit in one
// half-wave.
#include "mv_common.hpp"

#include <stdlib.h>

namespace rwkvmi {

typedef float fmf4 __attribute__((ext_vector_type(4)));

// Format constants: a unit is 16 bytes -- F16: 8 halves, two MFMAs (elements kk, kk + 4 of lane
// (m, kk)); F32: 4 floats, one MFMA (element kk).  Lane l of the matvec holds units k = EL l + STR u.
template <int WF>
struct FUnit;
template <>
struct FUnit<W_F16> {
    static constexpr int EL = 8, STR = 512, MF = 2;
    // dword kk of the LDS form: halves (kk, kk + 4) of the unit
    __device__ __forceinline__ static uint32_t pack(const uint4 & v, int kk) {
        const uint32_t lo = kk < 2 ? v.x : v.y, hi = kk < 2 ? v.z : v.w;
        return (kk & 1) ? __builtin_amdgcn_perm(hi, lo, 0x07060302u) : __builtin_amdgcn_perm(hi, lo, 0x05040100u);
    }
    __device__ __forceinline__ static float elem(uint32_t d, int h) {
        return (float)__builtin_bit_cast(_Float16, (uint16_t)(h ? d >> 16 : d));
    }
};
template <>
struct FUnit<W_F32> {
    static constexpr int EL = 4, STR = 256, MF = 1;
    __device__ __forceinline__ static uint32_t pack(const uint4 & v, int kk) {
        return kk == 0 ? v.x : kk == 1 ? v.y : kk == 2 ? v.z : v.w;
    }
    __device__ __forceinline__ static float elem(uint32_t d, int) { return __uint_as_float(d); }
};

constexpr int FM_SU = 16;                 // steps per stage
constexpr int FM_RS = FM_SU + 1;          // dwords per (kk, row) line
constexpr int FM_KS = 64 * FM_RS + 16;    // dwords per kk plane (= 16 mod 32: lanes kk, kk ^ 1 on disjoint banks)
constexpr int FM_OP = 4 * FM_KS;          // one operand tile (64 rows or tokens)
constexpr int FM_BUF = 2 * FM_OP;         // weights + activations

// SPLIT > 1 (grids of few tiles, e.g. the v7 LoRA first stage): workgroup s of a tile walks classes
// [s 64 / SPLIT, (s + 1) 64 / SPLIT) only -- a complete subtree of the class tree -- and stores the
// subtree sums to the entry's partials; k_qg_combine adds the tree's top levels, applies the epilogue
// and emits: the same bits as the unsplit kernel.
template <int WF, int SPLIT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_fmm(MMGroup g) {
    __shared__ uint32_t fsm[2 * FM_BUF];  // [2 buffers][W, X][kk][64][FM_RS]; after the loop: red[64 tok][64 rows]
    using U = FUnit<WF>;
    constexpr int EL = U::EL, STR = U::STR;
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MMEntry & E = g.e[e];
    const int T = g.T, M = E.W.M, K = E.W.K;
    const int tgroups = (T + 63) / 64;
    int local = (int)blockIdx.x - E.block0;
    {
        // consecutive workgroups go round-robin to the 8 XCDs: give the token groups of one row tile
        // consecutive indices on the same XCD, so its L2 serves their shared weight rows
        const int nloc = (g.e[e + 1 < g.n ? e + 1 : e].block0 - E.block0);
        const int ne = e + 1 < g.n ? nloc : (int)gridDim.x - E.block0;
        if (tgroups > 1 && (E.block0 & 7) == 0 && (ne & 7) == 0) local = (local & 7) * (ne >> 3) + (local >> 3);
    }
    const int sidx = local % SPLIT;
    local /= SPLIT;
    const int rt = local / tgroups, tg = local % tgroups;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ml = lane & 15, kk = lane >> 4;
    const int row0 = rt * 64, tok0 = tg * 64;
    const int wr = (wave & 1) * 32, wt = (wave >> 1) * 32;
    const char * wbase = (const char *)E.W.qs;
    const char * xbase = WF == W_F16 ? (const char *)E.in.h : (const char *)E.in.f;
    const int units = (K + STR - 1) / STR;
    // classes holding a unit (K < 64 units: the rest are zero leaves of the tree, folded below)
    const int ncls = units > 1 ? 64 : min(64, (K + EL - 1) / EL);
    // this workgroup's classes [l0, l0 + ncls_w) (SPLIT > 1: ncls = 64, K >= 512)
    const int l0 = sidx * (64 / SPLIT), ncls_w = SPLIT > 1 ? 64 / SPLIT : ncls;
    const int sbase = l0 * units, nsteps = ncls_w * units;
    const int nst = (nsteps + FM_SU - 1) / FM_SU;
    const size_t rowb = (size_t)K * (WF == W_F16 ? 2 : 4);

    // loader: thread tid moves units q = tid + 256 p (p < 4) of each operand: line q >> 4, step q & 15
    uint4 wv[4], xv[4];
    auto gload = [&](int stg) {
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int q = tid + 256 * p, ln = q >> 4, j = q & 15;
            const int s = sbase + min(stg * FM_SU + j, nsteps - 1);
            const int l = s / units, u = s - l * units;
            const int k = min(EL * l + STR * u, K - EL);  // a unit past K: clamped, never multiplied
            const size_t kb = (size_t)k * (WF == W_F16 ? 2 : 4);
            wv[p] = *(const uint4 *)(wbase + (size_t)min(row0 + ln, M - 1) * rowb + kb);
            xv[p] = *(const uint4 *)(xbase + (size_t)min(tok0 + ln, T - 1) * rowb + kb);
        }
    };
    auto lstore = [&](int buf) {
        uint32_t * wb = fsm + buf * FM_BUF;
        uint32_t * xb = wb + FM_OP;
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int q = tid + 256 * p, ln = q >> 4, j = q & 15;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                wb[c * FM_KS + ln * FM_RS + j] = U::pack(wv[p], c);
                xb[c * FM_KS + ln * FM_RS + j] = U::pack(xv[p], c);
            }
        }
    };

    fmf4 st[6][2][2], acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int n = 0; n < 2; n++) acc[i][n] = fmf4{0.0f, 0.0f, 0.0f, 0.0f};
    // binary counter over the classes (wave_sum63's tree): even classes open level 0, odd classes
    // close ctz(~l) levels into level N (the total, N = 6: into level 0, free by then)
#define FMM_CLOSE(NV)                                                                 \
    case NV: {                                                                        \
        _Pragma("unroll") for (int i = 0; i < 2; i++)                                 \
        _Pragma("unroll") for (int n = 0; n < 2; n++) {                               \
            fmf4 v_ = acc[i][n];                                                      \
            _Pragma("unroll") for (int kx = 0; kx < NV; kx++) v_ = st[kx][i][n] + v_; \
            st[NV < 6 ? NV : 0][i][n] = v_;  /* N = 6: the total, kept in level 0 */  \
        }                                                                             \
        break;                                                                        \
    }
#define FMM_FOLD(L)                                                                   \
    do {                                                                              \
        if (((L) & 1) == 0) {                                                         \
            _Pragma("unroll") for (int i = 0; i < 2; i++)                             \
            _Pragma("unroll") for (int n = 0; n < 2; n++) st[0][i][n] = acc[i][n];    \
        } else {                                                                      \
            switch (__builtin_ctz(~(L))) {                                            \
                FMM_CLOSE(1) FMM_CLOSE(2) FMM_CLOSE(3) FMM_CLOSE(4) FMM_CLOSE(5)      \
                default: FMM_CLOSE(6)                                                 \
            }                                                                         \
        }                                                                             \
        _Pragma("unroll") for (int i = 0; i < 2; i++)                                 \
        _Pragma("unroll") for (int n = 0; n < 2; n++) acc[i][n] = fmf4{0.0f, 0.0f, 0.0f, 0.0f}; \
    } while (0)

    gload(0);
    lstore(0);
    __syncthreads();
    int l = l0, u = 0;  // the step being multiplied
#pragma unroll 1
    for (int stg = 0; stg < nst; stg++) {
        if (stg + 1 < nst) gload(stg + 1);  // in flight under this stage's MFMAs
        const uint32_t * wb = fsm + (stg & 1) * FM_BUF + kk * FM_KS;
        const uint32_t * xb = wb + FM_OP;
        const int jn = min(FM_SU, nsteps - stg * FM_SU);
        // step j's operands are in registers while step j + 1's are read
        uint32_t a[2], b[2];
        auto opread = [&](uint32_t (&a_)[2], uint32_t (&b_)[2], int j) {
#pragma unroll
            for (int i = 0; i < 2; i++) a_[i] = wb[(wr + 16 * i + ml) * FM_RS + j];
#pragma unroll
            for (int n = 0; n < 2; n++) b_[n] = xb[(wt + 16 * n + ml) * FM_RS + j];
        };
        opread(a, b, 0);
#pragma unroll 1
        for (int j = 0; j < jn; j++) {
            uint32_t an[2], bn[2];
            opread(an, bn, min(j + 1, jn - 1));
            if (EL * l + STR * u < K) {  // uniform: the matvec's unit_valid
#pragma unroll
                for (int h = 0; h < U::MF; h++) {
                    // the four tiles' chains interleaved: no MFMA waits on the one just issued
#pragma unroll
                    for (int i = 0; i < 2; i++)
#pragma unroll
                        for (int n = 0; n < 2; n++)
                            acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(U::elem(a[i], h), U::elem(b[n], h), acc[i][n], 0, 0, 0);
                }
            }
            if (++u == units) {
                u = 0;
                FMM_FOLD(l - l0);  // the subtree's own counter (l0 = 0 unsplit)
                l++;
            }
#pragma unroll
            for (int i = 0; i < 2; i++) a[i] = an[i], b[i] = bn[i];
        }
        if (stg + 1 < nst) lstore((stg + 1) & 1);
        __syncthreads();
    }
    if constexpr (SPLIT == 1) {
        // classes without units (K < 64 units): zero leaves, which the matvec adds too.  An aligned run
        // of 2^j of them is a +0 node of level j (0 + 0 = +0 all the way up), merged into the counter
        // like any node -- v = st[k] + v while bit k of its position is set -- so the tail costs at most
        // six merges instead of one fold per class.
#pragma unroll 1
        while (l < 64) {
            const int j = __builtin_ctz(l);  // l + 2^j <= 64: l is a multiple of 2^j
            fmf4 v[2][2];
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int n = 0; n < 2; n++) v[i][n] = fmf4{0.0f, 0.0f, 0.0f, 0.0f};
            bool placed = false;
#pragma unroll
            for (int k = 0; k < 6; k++) {
                if (k < j || placed) continue;  // uniform
                if ((l >> k) & 1) {
#pragma unroll
                    for (int i = 0; i < 2; i++)
#pragma unroll
                        for (int n = 0; n < 2; n++) v[i][n] = st[k][i][n] + v[i][n];
                } else {
#pragma unroll
                    for (int i = 0; i < 2; i++)
#pragma unroll
                        for (int n = 0; n < 2; n++) st[k][i][n] = v[i][n];
                    placed = true;
                }
            }
            if (!placed) {  // the root: the total, kept in level 0
#pragma unroll
                for (int i = 0; i < 2; i++)
#pragma unroll
                    for (int n = 0; n < 2; n++) st[0][i][n] = v[i][n];
            }
            l += 1 << j;
        }
    }
#undef FMM_FOLD
#undef FMM_CLOSE
    if constexpr (SPLIT > 1) {
        // the subtree of 64 / SPLIT classes closed at level log2(64 / SPLIT)
        constexpr int LEV = SPLIT == 4 ? 4 : 3;
        float * part = g.part + E.poff + (size_t)sidx * T * M;
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int n = 0; n < 2; n++) {
                const int t = tok0 + wt + 16 * n + ml;
                if (t >= T) continue;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int row = row0 + wr + 16 * i + 4 * kk + q;
                    if (row < M) part[(size_t)t * M + row] = st[LEV][i][n][q];
                }
            }
        return;
    }
    // D layout: lane holds rows 4 * kk + q of a 16-row tile, token ml of a 16-token tile
    float * red = (float *)fsm;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int n = 0; n < 2; n++)
#pragma unroll
            for (int q = 0; q < 4; q++) red[(wt + 16 * n + ml) * 64 + wr + 16 * i + 4 * kk + q] = st[0][i][n][q] + 0.0f;
    __syncthreads();
    for (int i = tid; i < 64 * 64; i += 256) {
        const int t = tok0 + i / 64, row = row0 + i % 64;
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
    *launched = false;
    // below 32 tokens (contexts) the 64-token tile is mostly padding: k_mvb / k_mm_small stay
    if ((wtype != W_F16 && wtype != W_F32) || g.T < 16 || (g.T < 32 && !g.fmm)) return true;
    // short rows over few tokens (the v7 LoRA second stages, K <= 320, in a batched decode step: a
    // few steps against the stage and epilogue overhead) stay on k_mvb (22 us vs 51 us at B = 32);
    // over a sequence k_fmm wins (135 us vs k_mm_small's 177 us at T = 1024)
    for (int i = 0; i < g.n && !g.fmm && g.T < 256; i++)
        if (g.e[i].W.K < 512) return true;
    for (int i = 0; i < g.n; i++) {
        const MMEntry & e = g.e[i];
        if (e.W.type != wtype || e.W.K % 32 || e.in.tiled || e.in.fmt != act_fmt_for(wtype) || e.in.K != e.W.K)
            return true;
        if (e.emit && e.W.M % 32) return true;
        if (wtype == W_F16 ? !e.in.h : !e.in.f) return true;
        const uintptr_t xa = wtype == W_F16 ? (uintptr_t)e.in.h : (uintptr_t)e.in.f;
        if (((uintptr_t)e.W.qs | xa) & 15) return true;  // 16-byte unit loads
    }
    const int tgroups = (g.T + 63) / 64;
    int blocks = 0;
    for (int i = 0; i < g.n; i++) {
        g.e[i].block0 = blocks;
        blocks += (g.e[i].W.M + 63) / 64 * tgroups;
    }
    // a grid of a few workgroups (the v7 LoRA first stage over 32 contexts: 10) is slower than the
    // matvec forms, which spread such shapes over more workgroups
    if (blocks < 128 && !g.fmm) return true;
    // below 2 workgroups per CU: split the class tree (4 or 8 subtrees) when the partials fit
    int split = g.split == 4 || g.split == 8 ? g.split : blocks >= 2 * kQgCUs ? 1 : blocks * 4 >= 2 * kQgCUs ? 4 : 8;
    if (g.split == 1) split = 1;
    if (split > 1) {
        size_t pfl = 0;
        bool ok = g.part != nullptr;
        for (int i = 0; i < g.n; i++) {
            g.e[i].poff = pfl;
            pfl += (size_t)split * g.T * g.e[i].W.M;
            ok = ok && g.e[i].W.K >= 512 && g.e[i].W.M % 32 == 0;
        }
        if (!ok || g.part_floats < pfl) split = 1;
    }
#define FMM_L(WFv)                                                                                               \
    do {                                                                                                         \
        if (split == 4) RK_LAUNCH((k_fmm<WFv, 4>), dim3(blocks * 4), dim3(256), 0, st, g);             \
        else if (split == 8) RK_LAUNCH((k_fmm<WFv, 8>), dim3(blocks * 8), dim3(256), 0, st, g);        \
        else RK_LAUNCH((k_fmm<WFv, 1>), dim3(blocks), dim3(256), 0, st, g);                             \
    } while (0)
    if (split > 1)
        for (int i = 0; i < g.n; i++) g.e[i].block0 *= split;
    if (wtype == W_F16) FMM_L(W_F16);
    else FMM_L(W_F32);
#undef FMM_L
    HIP_OK(hipGetLastError());
    if (split > 1 && !launch_qg_combine(st, g, split)) return false;
    *launched = true;
    return true;
}

}  // namespace rwkvmi
