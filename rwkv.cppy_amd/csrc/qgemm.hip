// qgemm.hip -- token-batched dequant GEMM for the sequence path (T > 1) on int8 MFMA.
//
// Y[t][m] = sum_b d_w[m,b] d_x[t,b] sumi(m,t,b) (+ m_w s_x for the _1 formats), the ggml block
// arithmetic of rwkv_graph.inc's ggml_mul_mat calls with Q8_0/Q8_1 activations.  One
// v_mfma_i32_16x16x32_i8 is exactly one 32-weight quantization block, so the MFMA produces the
// exact integer block dot sumi for a 16x16 (rows x tokens) tile; the fp32 scale arithmetic
// runs in the epilogue of every block and reproduces the decode matvec's association bit for
// bit: the blocks of class l = b mod 64 (lane l of k_mv / k_mm) are chained with fmaf in
// ascending b, and the 64 class sums are folded with wave_sum63's perfect binary tree (a binary
// counter over the classes).  So serial decode and sequence evaluation stay bit-identical.
//
// Workgroup = 4 waves as 2 (rows) x 2 (tokens); a wave owns TI 16-row tiles x 2 16-token tiles.
#include "device_common.hpp"
#include "kernels.hpp"

#include <stdio.h>

namespace rwkvmi {

typedef int v4i_t __attribute__((ext_vector_type(4)));

// 8 int8 weights of `row`, block b, elements k = 8h..8h+7: the A operand of the 16x16x32 MFMA
// (lane = (h << 4) | (row & 15)).  ggml order: low nibble of qs[j] = element j, high = j + 16.
template <int WF>
__device__ __forceinline__ long wfrag(const DMat & W, int row, int b, int nb, int h) {
    const size_t bi = (size_t)row * nb + b;
    if constexpr (WF == W_Q8_0) {
        return *(const long *)(W.qs + bi * 32 + 8 * h);
    } else {
        const uint2 q = *(const uint2 *)(W.qs + bi * 16 + (h & 1) * 8);
        uint32_t lo = q.x, hi = q.y;
        if (h >= 2) {
            lo >>= 4;
            hi >>= 4;
        }
        lo &= 0x0F0F0F0Fu;
        hi &= 0x0F0F0F0Fu;
        if constexpr (WF == W_Q5_0 || WF == W_Q5_1) {
            const uint32_t qh = W.qh[bi] >> (8 * h);
            lo |= spread4(qh & 0xFu);
            hi |= spread4((qh >> 4) & 0xFu);
        }
        // per-byte subtraction without borrows: ((v | 0x80) - off) ^ 0x80 == v - off (mod 256)
        if constexpr (WF == W_Q4_0) {
            lo = ((lo | 0x80808080u) - 0x08080808u) ^ 0x80808080u;
            hi = ((hi | 0x80808080u) - 0x08080808u) ^ 0x80808080u;
        } else if constexpr (WF == W_Q5_0) {
            lo = ((lo | 0x80808080u) - 0x10101010u) ^ 0x80808080u;
            hi = ((hi | 0x80808080u) - 0x10101010u) ^ 0x80808080u;
        }
        return (long)(((unsigned long)hi << 32) | lo);
    }
}

template <int WF, int TI>
struct QOp {
    long a[TI];          // weight fragments per row tile
    long x[2];           // activation fragments per token tile
    uint32_t sc[TI][4];  // scales of the lane's 4 output rows per row tile (d | m << 16)
    float dx[2], sx[2];
};

template <int WF, int TI>
__device__ __forceinline__ void qop_load(QOp<WF, TI> & o, const MMEntry & E, int b, int nb, int rowA0, int rowO0,
                                         int tokB0, int M, int T, int h, int r16) {
    constexpr bool ONE = WF == W_Q4_1 || WF == W_Q5_1;
    const DMat & W = E.W;
    const int K = W.K;
#pragma unroll
    for (int i = 0; i < TI; i++) {
        o.a[i] = wfrag<WF>(W, min(rowA0 + 16 * i + r16, M - 1), b, nb, h);
        const int ro = min(rowO0 + 16 * i + 4 * h, W.ldt - 4);  // 4 consecutive rows, 4-aligned
        if constexpr (ONE) {
            const uint4 s = *(const uint4 *)((const uint32_t *)W.sct + (size_t)b * W.ldt + ro);
            o.sc[i][0] = s.x, o.sc[i][1] = s.y, o.sc[i][2] = s.z, o.sc[i][3] = s.w;
        } else {
            const uint2 s = *(const uint2 *)((const uint16_t *)W.sct + (size_t)b * W.ldt + ro);
            o.sc[i][0] = s.x & 0xFFFFu, o.sc[i][1] = s.x >> 16, o.sc[i][2] = s.y & 0xFFFFu, o.sc[i][3] = s.y >> 16;
        }
    }
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int t = min(tokB0 + 16 * j + r16, T - 1);
        o.x[j] = *(const long *)(E.in.q + (size_t)t * K + (size_t)b * 32 + 8 * h);
        o.dx[j] = E.in.d[(size_t)t * nb + b];
        o.sx[j] = ONE ? E.in.s[(size_t)t * nb + b] : 0.0f;
    }
}

// one block: 2*TI MFMAs, then acc = fmaf(d_w*d_x, sumi, acc) (+ acc2 += m_w*s_x)
template <int WF, int TI>
__device__ __forceinline__ void qop_compute(const QOp<WF, TI> & o, float (&c)[TI][2][4], float (&c2)[TI][2][4]) {
    constexpr bool ONE = WF == W_Q4_1 || WF == W_Q5_1;
    const v4i_t zero = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const v4i_t s = __builtin_amdgcn_mfma_i32_16x16x32_i8(o.a[i], o.x[j], zero, 0, 0, 0);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float dw = h2f((uint16_t)(o.sc[i][q] & 0xFFFFu));
                c[i][j][q] = fmaf(dw * o.dx[j], (float)s[q], c[i][j][q]);
                if constexpr (ONE) {
                    const float mw = h2f((uint16_t)(o.sc[i][q] >> 16));
                    c2[i][j][q] = c2[i][j][q] + mw * o.sx[j];
                }
            }
        }
}

template <int WF, int TI>
__global__ __launch_bounds__(256) void k_qgemm(MMGroup g) {
    constexpr bool ONE = WF == W_Q4_1 || WF == W_Q5_1;
    constexpr int NE = TI * 2 * 4;  // outputs per lane
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MMEntry & E = g.e[e];
    const int M = E.W.M, K = E.W.K, T = g.T, nb = K >> 5;
    const int tilesT = (T + 63) / 64;
    const int local = (int)blockIdx.x - E.block0;
    const int mtile = local / tilesT, ttile = local % tilesT;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r16 = lane & 15, h = lane >> 4;
    const int row0 = mtile * (32 * TI) + (wave & 1) * (16 * TI);  // this wave's first row
    const int tok0 = ttile * 64 + (wave >> 1) * 32;                // this wave's first token

    // binary-counter tree over the 64 classes (levels 0..5), per output
    float st[6][TI][2][4], st2[6][TI][2][4];
    float tot[TI][2][4], tot2[TI][2][4];
    QOp<WF, TI> op;
    if (nb > 0) qop_load<WF, TI>(op, E, 0, nb, row0, row0, tok0, M, T, h, r16);
#pragma unroll 1
    for (int l = 0; l < 64; l++) {
        float c[TI][2][4], c2[TI][2][4];
#pragma unroll
        for (int i = 0; i < TI; i++)
#pragma unroll
            for (int j = 0; j < 2; j++)
#pragma unroll
                for (int q = 0; q < 4; q++) c[i][j][q] = c2[i][j][q] = 0.0f;
#pragma unroll 1
        for (int b = l; b < nb; b += 64) {
            const QOp<WF, TI> cur = op;
            const int bn = b + 64 < nb ? b + 64 : (l + 1 < nb ? l + 1 : -1);
            if (bn >= 0) qop_load<WF, TI>(op, E, bn, nb, row0, row0, tok0, M, T, h, r16);
            qop_compute<WF, TI>(cur, c, c2);
        }
        // fold class l into the tree (wave_sum63's pairs (2i, 2i+1), then pairs of pairs, ...):
        // a binary counter -- class l closes as many levels as l has trailing one bits
        const int n = __builtin_ctz(~l);
#define QG_ELEMS for (int i = 0; i < TI; i++) for (int j = 0; j < 2; j++) for (int q = 0; q < 4; q++)
#define QG_CASE(N, DST, DST2)                                                                    \
    case N: {                                                                                    \
        _Pragma("unroll") QG_ELEMS {                                                             \
            float v = c[i][j][q];                                                                \
            for (int k = 0; k < N; k++) v = st[k][i][j][q] + v;                                  \
            DST[i][j][q] = v;                                                                    \
            if constexpr (ONE) {                                                                 \
                float v2 = c2[i][j][q];                                                          \
                for (int k = 0; k < N; k++) v2 = st2[k][i][j][q] + v2;                           \
                DST2[i][j][q] = v2;                                                              \
            }                                                                                    \
        }                                                                                        \
        break;                                                                                   \
    }
        switch (n) {
            QG_CASE(0, st[0], st2[0])
            QG_CASE(1, st[1], st2[1])
            QG_CASE(2, st[2], st2[2])
            QG_CASE(3, st[3], st2[3])
            QG_CASE(4, st[4], st2[4])
            QG_CASE(5, st[5], st2[5])
            default:
            QG_CASE(6, tot, tot2)
        }
#undef QG_CASE
#undef QG_ELEMS
    }
    (void)NE;
    // epilogue: y[t][m] = epi(total (+ total2)), as k_mm's red + red2
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int t = tok0 + 16 * j + r16;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int m = row0 + 16 * i + 4 * h + q;
                if (t < T && m < M) {
                    const float acc = ONE ? tot[i][j][q] + tot2[i][j][q] : tot[i][j][q] + 0.0f;
                    E.y[(size_t)t * E.ldy + m] = apply_epi(E, t, m, acc);
                }
            }
        }
}

template <int WF>
static void launch_qgemm_wf(hipStream_t st, MMGroup & g, int blocks) {
    constexpr int TI = (WF == W_Q4_1 || WF == W_Q5_1) ? 1 : 2;
    hipLaunchKernelGGL((k_qgemm<WF, TI>), dim3(blocks), dim3(256), 0, st, g);
}

// Every entry must have y (the engine gives emitting entries a scratch y); emission into the
// next matmul's activation format is a separate launch_act_from_f32 pass by the caller.
bool launch_qgemm(hipStream_t st, MMGroup & g, int wtype) {
    const int TI = (wtype == W_Q4_1 || wtype == W_Q5_1) ? 1 : 2;
    const int tilesT = (g.T + 63) / 64;
    int blocks = 0;
    for (int i = 0; i < g.n; i++) {
        MMEntry & e = g.e[i];
        if (e.W.type != wtype || !e.W.sct || e.W.K % 32 || !e.y || e.in.fmt != act_fmt_for(wtype)) {
            fprintf(stderr, "rwkv: qgemm entry %d not supported (type %d)\n", i, e.W.type);
            return false;
        }
        e.block0 = blocks;
        blocks += (e.W.M + 32 * TI - 1) / (32 * TI) * tilesT;
    }
    if (!blocks) return true;
    switch (wtype) {
        case W_Q4_0: launch_qgemm_wf<W_Q4_0>(st, g, blocks); break;
        case W_Q4_1: launch_qgemm_wf<W_Q4_1>(st, g, blocks); break;
        case W_Q5_0: launch_qgemm_wf<W_Q5_0>(st, g, blocks); break;
        case W_Q5_1: launch_qgemm_wf<W_Q5_1>(st, g, blocks); break;
        case W_Q8_0: launch_qgemm_wf<W_Q8_0>(st, g, blocks); break;
        default: fprintf(stderr, "rwkv: qgemm type %d unsupported\n", wtype); return false;
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
