// mv_batch.hip -- the decode matvec over B independent contexts (batched decode).
//
// y[t][m] = W[m] . x[t] for the B activation rows of B contexts (MMGroup, T = B), with the decode
// matvec's per-output arithmetic (k_mva / k_mv: lane l accumulates units l, l+64, ... with the
// same fma chain, wave_sum63 folds the 64 lanes), so context t's outputs are bit-identical to its
// single-context decode.  What changes is the weight traffic: a wave loads its R rows' units into
// registers ONCE (non-temporal, one HBM round trip) and streams the B activation rows past them
// (L2-resident, each prefetched one context ahead), so a step reads every weight byte once for
// all B contexts instead of B times.
//
// Two phases per workgroup: (1) dots -- each wave's R row sums for every context go to LDS
// (red[t][row]); (2) epilogue -- the workgroup's threads apply the epilogue to all (t, row)
// pairs at once (their y / aux operands are independent loads, not a dependent round trip per
// context), and emitting groups (RW = 32 rows = one quantization block) quantize each
// context's 32 outputs as one block of the next matmul's input, as k_mm does.
#include "mv_common.hpp"

namespace rwkvmi {

template <int WF, int R, int U, bool EMIT>
__global__ __launch_bounds__(256) void k_mvb(MMGroup g) {
    constexpr int RW = 4 * R;
    extern __shared__ float red[];  // [T][RW]
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MMEntry & E = g.e[e];
    const int T = g.T, M = E.W.M, K = E.W.K;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int rowwg = ((int)blockIdx.x - E.block0) * RW, row0 = rowwg + wave * R;
    int rows[R];
#pragma unroll
    for (int r = 0; r < R; r++) rows[r] = min(row0 + r, M - 1);
    WBlk w[R][U];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < R; r++) w[r][u] = load_unit<WF>(E.W, rows[r], u, lane);
    // context t's activation row: the [T][K] layout of a non-tiled ActBuf
    auto act_row = [&](int t) {
        ActBuf a = E.in;
        const size_t nb = (size_t)(K >> 5);
        a.q = E.in.q + (size_t)t * K;
        a.d = E.in.d + (size_t)t * nb;
        a.s = E.in.s + (size_t)t * nb;
        a.qsum = E.in.qsum + (size_t)t * nb;
        a.h = E.in.h + (size_t)t * K;
        a.f = E.in.f + (size_t)t * K;
        return a;
    };
    // activation ring: the rows of the next PD contexts are in flight while one is computed
    // (an L2 round trip is several contexts' worth of dots)
    constexpr int PD = U == 1 ? 8 : U == 2 ? 4 : 2;
    AUnit xb[PD][U];
#pragma unroll
    for (int p = 0; p < PD; p++) {
        const ActBuf a = act_row(min(p, T - 1));
#pragma unroll
        for (int u = 0; u < U; u++) xb[p][u] = load_act_unit<WF, false>(a, u, lane);
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
#pragma unroll 1
    for (int t0 = 0; t0 < T; t0 += PD) {
#pragma unroll
        for (int p = 0; p < PD; p++) {
            const int t = t0 + p;
            if (t >= T) break;  // uniform
            AUnit x[U];
#pragma unroll
            for (int u = 0; u < U; u++) x[u] = xb[p][u];
            if (t + PD < T) {
                const ActBuf a = act_row(t + PD);
#pragma unroll
                for (int u = 0; u < U; u++) xb[p][u] = load_act_unit<WF, false>(a, u, lane);
            }
            float acc[R], acc2[R];
#pragma unroll
            for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
#pragma unroll
            for (int u = 0; u < U; u++) {
                const bool valid = unit_valid<WF>(K, u, lane);
#pragma unroll
                for (int r = 0; r < R; r++) {
                    float s = acc[r], s2 = acc2[r];
                    dot_unit<WF>(w[r][u], x[u], s, s2);
                    acc[r] = valid ? s : acc[r];
                    acc2[r] = valid ? s2 : acc2[r];
                }
            }
#pragma unroll
            for (int r = 0; r < R; r++) {
                const float s = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
                if (lane == 63) red[t * RW + wave * R + r] = s;
            }
        }
    }
    __syncthreads();
    // epilogue over every (context, row) of the workgroup; RW = 32 when emitting, so each
    // half-wave holds one context's 32-row block
    for (int i = threadIdx.x; i < T * RW; i += 256) {
        const int t = i / RW, row = rowwg + i % RW;
        float v = 0.0f;
        if (row < M) {
            v = apply_epi(E, t, row, red[i]);
            if (E.y) E.y[(size_t)t * E.ldy + row] = v;
        }
        if constexpr (EMIT) {
            if (E.emit) emit32(E.out, t, row, v);
        }
    }
}

// Shapes: U = 16-byte units per lane (K), R rows per wave; emitting groups need R = 8.
template <int WF>
static bool launch_mvb_wf(hipStream_t st, MMGroup & g, bool emit, int U) {
    // rows per wave: emitting groups need a 32-row block per workgroup; long rows (U >= 4: the
    // FFN value matrix, the head) take fewer rows per wave so the grid still covers the chip
    const int R = emit ? 8 : U <= 2 ? 4 : U <= 4 ? 2 : 1;
    const int RW = 4 * R;
    int blocks = 0;
    for (int i = 0; i < g.n; i++) {
        g.e[i].block0 = blocks;
        blocks += (g.e[i].W.M + RW - 1) / RW;
    }
    if (!blocks) return true;
    const dim3 grid(blocks), block(256);
    const size_t lds = (size_t)g.T * RW * 4;
#define MVB(Rv, Uv, Ev) RK_LAUNCH((k_mvb<WF, Rv, Uv, Ev>), grid, block, lds, st, g)
    if (emit) {
        if (U == 1) MVB(8, 1, true);
        else MVB(8, 2, true);
    } else if (U == 1) {
        MVB(4, 1, false);
    } else if (U == 2) {
        MVB(4, 2, false);
    } else if (U <= 4) {
        MVB(2, 4, false);
    } else {
        MVB(1, 8, false);
    }
#undef MVB
    HIP_OK(hipGetLastError());
    return true;
}

// false (nothing launched) when the shape is outside what k_mvb covers; the caller then uses
// k_mm, which computes the same bits.
bool launch_mvb_group(hipStream_t st, MMGroup & g, int wtype, bool * launched) {
    *launched = false;
    if (g.T < 1 || g.T > 256) return true;
    bool emit = false;
    int umax = 1;
    for (int i = 0; i < g.n; i++) {
        const MMEntry & e = g.e[i];
        if (e.W.type != wtype || e.W.K % 32 || e.in.tiled || e.in.fmt != act_fmt_for(wtype) || e.in.K != e.W.K)
            return true;
        if (e.emit && (e.W.M % 32 || e.out.tiled)) return true;
        emit |= e.emit != 0;
        umax = umax > mv_units(wtype, e.W.K) ? umax : mv_units(wtype, e.W.K);
    }
    const int U = umax <= 1 ? 1 : umax <= 2 ? 2 : umax <= 4 ? 4 : umax <= 8 ? 8 : 0;
    if (!U || (emit && U > 2)) return true;
    bool ok = false;
    switch (wtype) {
        case W_F32: ok = launch_mvb_wf<W_F32>(st, g, emit, U); break;
        case W_F16: ok = launch_mvb_wf<W_F16>(st, g, emit, U); break;
        case W_Q4_0: ok = launch_mvb_wf<W_Q4_0>(st, g, emit, U); break;
        case W_Q4_1: ok = launch_mvb_wf<W_Q4_1>(st, g, emit, U); break;
        case W_Q5_0: ok = launch_mvb_wf<W_Q5_0>(st, g, emit, U); break;
        case W_Q5_1: ok = launch_mvb_wf<W_Q5_1>(st, g, emit, U); break;
        case W_Q8_0: ok = launch_mvb_wf<W_Q8_0>(st, g, emit, U); break;
        default: return true;
    }
    *launched = ok;
    return ok;
}

}  // namespace rwkvmi
