// wkv7_chunk.hip -- chunk-parallel WKV-7 (v7 time mixing, head size 64) for long sequences, behind
// the same switch as the chunked WKV-6 (RWKV_MI355X_WKV_CHUNK, rwkv_mi355x_debug_set "wkv_chunk").
// Not bit-exact with the serial recurrence (k_wkv7_s64, the reference's association,
// rwkv_operators_wkv_v7.inc:37-107): the sums are re-associated, so results agree within fp32
// rounding (tests/test_gpu_wkv_chunk.py states the tolerance against a float64 recurrence).
//
// Recurrence per head, row i of the state (value channel i; j = key channel):
//   c_t = s_{t-1} . a_t;   s_t = s_{t-1} o w_t + c_t b_t + v_t[i] k_t;   y_t[i] = s_t . r_t
// (a = -kk, b = kk * iclr: the transition diag(w) + a b^T is a diagonal-plus-rank-one matrix).  For a
// chunk of L tokens u = 0..L-1 from state s0, with P[u][j] = sum_{p<u} log2 w_p[j] (chunk-local; P[0] =
// 0) every decay product is 2^(P[x] - P[y]) with x >= y, so nothing overflows:
//   c_u = s0 . (a_u 2^P[u]) + sum_{q<u} Ab[u][q] c_q + sum_{q<u} Ak[u][q] v_q
//        Ab[u][q] = sum_j a_u b_q 2^(P[u] - P[q+1]),  Ak the same with k_q
//   -> c = s0 G + M v with N = (I - Ab)^-1 (unit lower triangular), G[j][u] = sum_p N[u][p] a_p[j] 2^P[p],
//      M = N Ak
//   y_u = s0 . (r_u 2^P[u+1]) + sum_{q<=u} Rb[u][q] c_q + sum_{q<=u} Rk[u][q] v_q
//        Rb[u][q] = sum_j r_u b_q 2^(P[u+1] - P[q+1]),  Rk the same with k_q
//   s_L = s0 o 2^P[L] + sum_q (c_q b_q + v_q k_q) o 2^(P[L] - P[q+1])
// v7's decay is w = exp(-0.606531 sigmoid(.)) >= 0.545, so |P| <= 14 over a 16-token chunk and the
// triangular solve is well conditioned (the transition is a contraction).
//
// Three launches per layer; only the second is serial, over chunks:
//   k_wkv7c_prep  (chunk, head): P, the four L x L matrices, N, M, G and the decayed rows of r, b, k
//                 -- every exp2 of the chunk;
//   k_wkv7c_carry (head, 16 rows): per chunk c = s0 G + M v (row sums across the 16 lanes of a DPP
//                 row) and the new state, the chunk-start states stored -- 64 chunk steps at T = 1024
//                 instead of 1024 token steps;
//   k_wkv7c_out   (chunk, head): c again from the stored start state, then y.
#include "device_common.hpp"
#include "kernels.hpp"

namespace rwkvmi {

constexpr int W7C_L = 16;  // tokens per chunk
constexpr int W7C_S = 64;  // head size
// one (chunk, head) record of k_wkv7c_prep's outputs (floats)
constexpr int W7_G = 0;                    // G [64 j][16 u]
constexpr int W7_M = W7_G + W7C_S * W7C_L;  // M [16 u][16 q]
constexpr int W7_RB = W7_M + W7C_L * W7C_L;  // Rb [16 u][16 q]
constexpr int W7_RK = W7_RB + W7C_L * W7C_L; // Rk [16 u][16 q]
constexpr int W7_RT = W7_RK + W7C_L * W7C_L; // r_u 2^P[u+1]        [16 u][64 j]
constexpr int W7_BH = W7_RT + W7C_L * W7C_S; // b_q 2^(P[L]-P[q+1]) [16 q][64 j]
constexpr int W7_KH = W7_BH + W7C_L * W7C_S; // k_q 2^(P[L]-P[q+1]) [16 q][64 j]
constexpr int W7_DL = W7_KH + W7C_L * W7C_S; // 2^P[L]              [64 j]
constexpr int W7_REC = W7_DL + W7C_S;

__device__ __forceinline__ float w7_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__global__ __launch_bounds__(256) void k_wkv7c_prep(int T, int H, const float * r, const float * w, const float * k,
                                                    const float * a, const float * b, float * rec) {
    constexpr int L = W7C_L, S = W7C_S;
    __shared__ float sa[L][S + 1], sb[L][S + 1], sk[L][S + 1], sr[L][S + 1], pm[L + 1][S + 1];
    __shared__ float sAb[L][L + 1], sAk[L][L + 1], sN[L][L + 1];
    const int c = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, C = H * S, t0 = c * L;
    float * const R = rec + ((size_t)c * H + h) * W7_REC;
#pragma unroll
    for (int q = 0; q < (L * S) / 256; q++) {
        const int idx = tid + 256 * q, u = idx >> 6, j = idx & 63, t = t0 + u;
        const bool ok = t < T;  // tokens past the end: zero operands, no decay
        const size_t o = (size_t)min(t, T - 1) * C + (size_t)h * S + j;
        sa[u][j] = ok ? a[o] : 0.0f;
        sb[u][j] = ok ? b[o] : 0.0f;
        sk[u][j] = ok ? k[o] : 0.0f;
        sr[u][j] = ok ? r[o] : 0.0f;
        pm[u + 1][j] = ok ? __builtin_amdgcn_logf(w[o]) : 0.0f;  // v_log_f32: log2
    }
    __syncthreads();
    if (tid < S) {
        float acc = 0.0f;
        pm[0][tid] = 0.0f;
#pragma unroll
        for (int u = 1; u <= L; u++) {
            acc += pm[u][tid];
            pm[u][tid] = acc;
        }
    }
    __syncthreads();
    // the four L x L matrices: thread (u = tid / 16, q = tid % 16)
    {
        const int u = tid >> 4, q = tid & 15;
        float ab = 0.0f, ak = 0.0f, rb = 0.0f, rk = 0.0f;
        if (q <= u) {
#pragma unroll 8
            for (int j = 0; j < S; j++) {
                const float e1 = w7_exp2(pm[u + 1][j] - pm[q + 1][j]);
                rb = fmaf(sr[u][j] * sb[q][j], e1, rb);
                rk = fmaf(sr[u][j] * sk[q][j], e1, rk);
                const float e0 = q < u ? w7_exp2(pm[u][j] - pm[q + 1][j]) : 0.0f;
                ab = fmaf(sa[u][j] * sb[q][j], e0, ab);
                ak = fmaf(sa[u][j] * sk[q][j], e0, ak);
            }
        }
        sAb[u][q] = ab;
        sAk[u][q] = ak;
        R[W7_RB + tid] = rb;
        R[W7_RK + tid] = rk;
    }
    __syncthreads();
    // N = (I - Ab)^-1: column q on lane q (N[u][q] = [u == q] + sum_{q<=p<u} Ab[u][p] N[p][q])
    if (tid < L) {
        const int q = tid;
        for (int u = 0; u < L; u++) {
            float n = u == q ? 1.0f : 0.0f;
            for (int p = q; p < u; p++) n = fmaf(sAb[u][p], sN[p][q], n);
            sN[u][q] = q <= u ? n : 0.0f;
        }
    }
    __syncthreads();
    {
        // M = N Ak: thread (u, q)
        const int u = tid >> 4, q = tid & 15;
        float m = 0.0f;
        for (int p = q + 1; p <= u; p++) m = fmaf(sN[u][p], sAk[p][q], m);
        R[W7_M + tid] = m;
        // G[j][u] = sum_{p<=u} N[u][p] a_p[j] 2^P[p]: thread (j = tid / 4, u = 4 (tid % 4) ..)
        const int j = tid >> 2, u0 = (tid & 3) * 4;
        float at[L];
#pragma unroll
        for (int p = 0; p < L; p++) at[p] = sa[p][j] * w7_exp2(pm[p][j]);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int uu = u0 + e;
            float g = 0.0f;
#pragma unroll
            for (int p = 0; p < L; p++)
                if (p <= uu) g = fmaf(sN[uu][p], at[p], g);
            R[W7_G + j * L + uu] = g;
        }
    }
#pragma unroll
    for (int q = 0; q < (L * S) / 256; q++) {
        const int idx = tid + 256 * q, u = idx >> 6, j = idx & 63;
        R[W7_RT + idx] = sr[u][j] * w7_exp2(pm[u + 1][j]);
        const float e = w7_exp2(pm[L][j] - pm[u + 1][j]);
        R[W7_BH + idx] = sb[u][j] * e;
        R[W7_KH + idx] = sk[u][j] * e;
    }
    if (tid < S) R[W7_DL + tid] = w7_exp2(pm[L][tid]);
}

// v + v(lane + 8 mod 16) + ... over a 16-lane DPP row (every lane of the row ends with the sum)
__device__ __forceinline__ float w7_row_sum16(float v) {
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, false));
    return v;
}

// The chunk-serial part.  Workgroup = (head, 16 value rows); thread (row i = 16 blockIdx.y + tid / 16,
// key columns 4 (tid % 16) ..): the 16 lanes of a row form one DPP row.  A chunk's operands (G, M, the
// decayed b / k rows, 2^P[L], the rows' v) are loaded global -> registers one chunk ahead, then into
// one half of an LDS ring; one barrier per chunk.
__global__ __launch_bounds__(256) void k_wkv7c_carry(int T, int H, const float * v, const float * rec,
                                                     const float * sin, float * sout, float * SC) {
    constexpr int L = W7C_L, S = W7C_S;
    __shared__ __attribute__((aligned(16))) float sG[2][S * L], sBH[2][L * S], sKH[2][L * S], sM[2][L * L],
        sDL[2][S], sv[2][L][16];
    const int h = blockIdx.x, ib = blockIdx.y, tid = threadIdx.x, C = H * S;
    const int rl = tid >> 4, jq = tid & 15, i = ib * 16 + rl, j0 = 4 * jq;
    const int nch = (T + L - 1) / L;
    const size_t sb0 = (size_t)h * S * S + (size_t)i * S + j0;
    float s[4];
#pragma unroll
    for (int e = 0; e < 4; e++) s[e] = sin[sb0 + e];
    float4 rg, rbh, rkh, rm, rdl, rv;
    auto load = [&](int cc) __attribute__((always_inline)) {
        const float * Rc = rec + ((size_t)cc * H + h) * W7_REC;
        rg = *(const float4 *)(Rc + W7_G + 4 * tid);
        rbh = *(const float4 *)(Rc + W7_BH + 4 * tid);
        rkh = *(const float4 *)(Rc + W7_KH + 4 * tid);
        rm = *(const float4 *)(Rc + W7_M + 4 * (tid & 63));
        rdl = *(const float4 *)(Rc + W7_DL + 4 * (tid & 15));
        const int t = cc * L + ((tid & 63) >> 2);
        rv = *(const float4 *)(v + (size_t)min(t, T - 1) * C + (size_t)h * S + ib * 16 + 4 * (tid & 3));
        if (t >= T) rv = make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto store = [&](int bf) __attribute__((always_inline)) {
        *(float4 *)&sG[bf][4 * tid] = rg;
        *(float4 *)&sBH[bf][4 * tid] = rbh;
        *(float4 *)&sKH[bf][4 * tid] = rkh;
        if (tid < 64) {
            *(float4 *)&sM[bf][4 * tid] = rm;
            *(float4 *)&sv[bf][tid >> 2][4 * (tid & 3)] = rv;
        }
        if (tid < 16) *(float4 *)&sDL[bf][4 * tid] = rdl;
    };
    load(0);
    store(0);
    __syncthreads();
    for (int c = 0; c < nch; c++) {
        const int bf = c & 1;
        if (c + 1 < nch) load(c + 1);
        *(float4 *)(SC + ((size_t)c * H + h) * S * S + (size_t)i * S + j0) = make_float4(s[0], s[1], s[2], s[3]);
        // c_u = sum_j s[j] G[j][u] + sum_q M[u][q] v_q[i]: this lane's 4 columns, M's row u = jq on
        // lane jq, then the row sum over the 16 lanes
        float vr[L];
#pragma unroll
        for (int q = 0; q < L; q++) vr[q] = sv[bf][q][rl];
        float cp = 0.0f;
#pragma unroll
        for (int q4 = 0; q4 < L; q4 += 4) {
            const float4 m4 = *(const float4 *)&sM[bf][jq * L + q4];
            cp = fmaf(m4.x, vr[q4], cp);
            cp = fmaf(m4.y, vr[q4 + 1], cp);
            cp = fmaf(m4.z, vr[q4 + 2], cp);
            cp = fmaf(m4.w, vr[q4 + 3], cp);
        }
        float cu[L];
#pragma unroll
        for (int u = 0; u < L; u++) cu[u] = u == jq ? cp : 0.0f;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const float * g = &sG[bf][(j0 + e) * L];
#pragma unroll
            for (int u4 = 0; u4 < L; u4 += 4) {
                const float4 g4 = *(const float4 *)(g + u4);
                cu[u4] = fmaf(s[e], g4.x, cu[u4]);
                cu[u4 + 1] = fmaf(s[e], g4.y, cu[u4 + 1]);
                cu[u4 + 2] = fmaf(s[e], g4.z, cu[u4 + 2]);
                cu[u4 + 3] = fmaf(s[e], g4.w, cu[u4 + 3]);
            }
        }
#pragma unroll
        for (int u = 0; u < L; u++) cu[u] = w7_row_sum16(cu[u]);
        // s <- s o 2^P[L] + sum_u c_u bhat_u + sum_u v_u[i] khat_u
        const float4 dl = *(const float4 *)&sDL[bf][j0];
        float ns[4] = {s[0] * dl.x, s[1] * dl.y, s[2] * dl.z, s[3] * dl.w};
#pragma unroll
        for (int u = 0; u < L; u++) {
            const float4 b4 = *(const float4 *)&sBH[bf][u * S + j0];
            const float4 k4 = *(const float4 *)&sKH[bf][u * S + j0];
            ns[0] = fmaf(vr[u], k4.x, fmaf(cu[u], b4.x, ns[0]));
            ns[1] = fmaf(vr[u], k4.y, fmaf(cu[u], b4.y, ns[1]));
            ns[2] = fmaf(vr[u], k4.z, fmaf(cu[u], b4.z, ns[2]));
            ns[3] = fmaf(vr[u], k4.w, fmaf(cu[u], b4.w, ns[3]));
        }
#pragma unroll
        for (int e = 0; e < 4; e++) s[e] = ns[e];
        if (c + 1 < nch) store(bf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int e = 0; e < 4; e++) sout[sb0 + e] = s[e];
}

// y of one (chunk, head): c = s0 G + M v from the stored chunk-start state, then
// y_u[i] = s0[i] . rt_u + sum_{q<=u} (Rb[u][q] c_q[i] + Rk[u][q] v_q[i]).
__global__ __launch_bounds__(256) void k_wkv7c_out(int T, int H, const float * v, const float * rec, const float * SC,
                                                   float * y) {
    constexpr int L = W7C_L, S = W7C_S;
    __shared__ __attribute__((aligned(16))) float ss[S][S + 4], sG[S][L], sM[L][L], sRb[L][L], sRk[L][L], sRT[L][S],
        sv[L][S], scc[S][L + 1];
    const int c = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, C = H * S, t0 = c * L;
    const float * Rc = rec + ((size_t)c * H + h) * W7_REC;
    const float * s0 = SC + ((size_t)c * H + h) * S * S;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int idx = tid + 256 * q;
        *(float4 *)&ss[idx >> 4][(idx & 15) * 4] = *(const float4 *)(s0 + idx * 4);
        sG[idx >> 4][idx & 15] = Rc[W7_G + idx];
        sRT[idx >> 6][idx & 63] = Rc[W7_RT + idx];
        const int u = idx >> 6, t = t0 + u;
        sv[u][idx & 63] = t < T ? v[(size_t)t * C + (size_t)h * S + (idx & 63)] : 0.0f;
    }
    sM[tid >> 4][tid & 15] = Rc[W7_M + tid];
    sRb[tid >> 4][tid & 15] = Rc[W7_RB + tid];
    sRk[tid >> 4][tid & 15] = Rc[W7_RK + tid];
    __syncthreads();
    {
        // c[i][q]: thread (i = tid / 4, q = 4 (tid % 4) ..)
        const int i = tid >> 2, q0 = (tid & 3) * 4;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int q = q0 + e;
            float acc = 0.0f;
#pragma unroll 16
            for (int j = 0; j < S; j++) acc = fmaf(ss[i][j], sG[j][q], acc);
#pragma unroll
            for (int p = 0; p < L; p++) acc = fmaf(sM[q][p], sv[p][i], acc);
            scc[i][q] = acc;
        }
    }
    __syncthreads();
    // y: thread (u = tid / 16, rows 4 (tid % 16) ..)
    const int u = tid >> 4, i0 = (tid & 15) * 4;
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const int i = i0 + e;
        float acc = 0.0f;
#pragma unroll 16
        for (int j = 0; j < S; j++) acc = fmaf(ss[i][j], sRT[u][j], acc);
#pragma unroll
        for (int q = 0; q < L; q++)
            if (q <= u) acc = fmaf(sRk[u][q], sv[q][i], fmaf(sRb[u][q], scc[i][q], acc));
        o[e] = acc;
    }
    if (t0 + u < T) *(float4 *)(y + (size_t)(t0 + u) * C + (size_t)h * S + i0) = make_float4(o[0], o[1], o[2], o[3]);
}

size_t wkv7_chunked_scratch_floats(int T, int H) {
    const size_t nch = ((size_t)T + W7C_L - 1) / W7C_L;
    return nch * H * W7_REC + nch * H * W7C_S * W7C_S;
}

bool wkv7_chunked_supported(int T, int S, int bs) { return S == W7C_S && bs == 0 && T >= 2; }

bool launch_wkv7_chunked(hipStream_t st, int T, int H, const float * r, const float * w, const float * k,
                         const float * v, const float * a, const float * b, const float * state_in, float * state_out,
                         float * y, float * scratch) {
    if (!wkv7_chunked_supported(T, W7C_S, 0) || H < 1) return false;
    const int nch = (T + W7C_L - 1) / W7C_L;
    float * rec = scratch;
    float * SC = rec + (size_t)nch * H * W7_REC;
    RK_LAUNCH(k_wkv7c_prep, dim3(nch, H), dim3(256), 0, st, T, H, r, w, k, a, b, rec);
    HIP_OK(hipGetLastError());
    RK_LAUNCH(k_wkv7c_carry, dim3(H, W7C_S / 16), dim3(256), 0, st, T, H, v, rec, state_in, state_out, SC);
    HIP_OK(hipGetLastError());
    RK_LAUNCH(k_wkv7c_out, dim3(nch, H), dim3(256), 0, st, T, H, v, rec, SC, y);
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
