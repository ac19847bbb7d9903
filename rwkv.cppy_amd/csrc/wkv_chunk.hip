// wkv_chunk.hip -- chunk-parallel WKV-6 (v5 / v6 time mixing, head size 64) for long sequences,
// behind a switch (RWKV_MI355X_WKV_CHUNK, rwkv_mi355x_debug_set "wkv_chunk").  Not bit-exact with
// the serial recurrence (k_wkv6_s64, the reference's association: rwkv_operators_wkv_v6 /
// ggml_rwkv_wkv6, rwkv_graph.inc:363-371): the sums are re-associated, so results agree within
// fp32 rounding (tests/test_gpu_wkv_chunk.py states the tolerance and checks the whole model
// against the oracle's noise band).
//
// Recurrence per head (state S[i][j], i = key channel, j = value channel):
//   y_t[j] = sum_i r_t[i] (S[i][j] + u[i] k_t[i] v_t[j]);   S[i][j] <- w_t[i] S[i][j] + k_t[i] v_t[j].
// For a chunk of L tokens starting with state S0, with la_t[i] = sum_{q<t} log2 w_q[i] (chunk-local):
//   y_t[j]  = sum_i (r_t[i] 2^la_t[i]) S0[i][j] + sum_{s<=t} B[t][s] v_s[j]
//   B[t][s] = sum_i r_t[i] k_s[i] 2^(la_t[i] - la_{s+1}[i])  (s < t),  B[t][t] = sum_i r_t[i] u[i] k_t[i]
//   S_L     = 2^la_L[i] S0[i][j] + sum_s (k_s[i] 2^(la_L[i] - la_{s+1}[i])) v_s[j]
// Every exponent is <= 0 (w <= 1), so nothing overflows; log2 w is clamped at -40 (w < 1e-12 acts as
// 1e-12: the terms it multiplies are below 1e-12 either way), and chunks are 16 tokens, so |la| stays
// below 640 and the differences keep ~1e-5 relative accuracy in the worst case.
//
// Four launches per layer; only the third is serial, and only over chunks, elementwise:
//   k_wkv6c_prep  (chunk, head): la, RA = r 2^la, KB = k 2^(la_L - la_{s+1}), the L x L matrix B and
//                 AL = 2^la_L -- all the exp work;
//   k_wkv6c_u     (chunk, head): U_c = KB_c^T V_c, the chunk's tokens carried to its end;
//   k_wkv6c_carry (state element): S_{c+1} = AL_c S_c + U_c over the chunks, S_c stored over U_c --
//                 64 dependent fmas per element at T = 1024 instead of 1024 token steps;
//   k_wkv6c_out   (chunk, head): y = RA S_c + B V.
// A first form with the chunk-serial loop doing the whole y product per chunk (one workgroup per
// head and 8 columns) measured slower than the serial kernel (105 vs 90 us at T = 1024, H = 32).
#include "device_common.hpp"
#include "kernels.hpp"

namespace rwkvmi {

constexpr int WKVC_L = 16;  // tokens per chunk
constexpr int WKVC_S = 64;  // head size

template <bool WPT>
__global__ __launch_bounds__(256) void k_wkv6c_prep(int T, int H, const float * k, const float * r, const float * w,
                                                     const float * u, float * RA, float * KB, float * Bm, float * AL) {
    constexpr int L = WKVC_L, S = WKVC_S;
    // rows padded to 65: the B threads read rows t, s + 1 of the same column i
    __shared__ float sk[L][S + 1], sr[L][S + 1], sla[L + 1][S + 1];
    const int c = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, C = H * S;
    const int t0 = c * L;
#pragma unroll
    for (int q = 0; q < (L * S) / 256; q++) {
        const int idx = tid + 256 * q, tt = idx >> 6, i = idx & 63, t = t0 + tt;
        const bool ok = t < T;
        const size_t o = (size_t)t * C + (size_t)h * S + i;
        sk[tt][i] = ok ? k[o] : 0.0f;
        sr[tt][i] = ok ? r[o] : 0.0f;
        const float wv = ok ? (WPT ? w[o] : w[h * S + i]) : 1.0f;
        sla[tt + 1][i] = fmaxf(__builtin_amdgcn_logf(wv), -40.0f);  // v_log_f32 (log2): 0 -> -inf -> -40
    }
    __syncthreads();
    if (tid < S) {  // chunk-local prefix sums of log2 w
        float a = 0.0f;
        sla[0][tid] = 0.0f;
#pragma unroll
        for (int tt = 1; tt <= L; tt++) {
            a += sla[tt][tid];
            sla[tt][tid] = a;
        }
        AL[(size_t)c * C + h * S + tid] = __builtin_amdgcn_exp2f(a);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < (L * S) / 256; q++) {
        const int idx = tid + 256 * q, tt = idx >> 6, i = idx & 63, t = t0 + tt;
        if (t < T) {
            const size_t o = (size_t)t * C + (size_t)h * S + i;
            RA[o] = sr[tt][i] * __builtin_amdgcn_exp2f(sla[tt][i]);
            KB[o] = sk[tt][i] * __builtin_amdgcn_exp2f(sla[L][i] - sla[tt + 1][i]);
        }
    }
    // B[t][s]: thread (t = tid / 16, s = tid % 16); s > t stays 0
    {
        const int tt = tid >> 4, s = tid & 15;
        float acc = 0.0f;
        if (s < tt) {
#pragma unroll 8
            for (int i = 0; i < S; i++) acc += sr[tt][i] * sk[s][i] * __builtin_amdgcn_exp2f(sla[tt][i] - sla[s + 1][i]);
        } else if (s == tt) {
            const float * uh = u + h * S;
#pragma unroll 8
            for (int i = 0; i < S; i++) acc += sr[tt][i] * uh[i] * sk[tt][i];
        }
        Bm[((size_t)c * H + h) * (L * L) + tid] = acc;
    }
}

// Chunk state contributions U_c[i][j] = sum_s KB[s][i] v_s[j] (the chunk's own tokens carried to its
// end), one workgroup per (chunk, head): thread (i = tid / 16 + 16 q, j = 4 (tid % 16) ..) 16 outputs.
__global__ __launch_bounds__(256) void k_wkv6c_u(int T, int H, const float * KB, const float * v, float * US) {
    constexpr int L = WKVC_L, S = WKVC_S;
    __shared__ __attribute__((aligned(16))) float skb[L][S], sv[L][S];
    const int c = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, C = H * S, t0 = c * L;
    {
        const int tt = tid >> 4, i4 = (tid & 15) * 4;
        const bool ok = t0 + tt < T;
        const size_t o = (size_t)(t0 + tt) * C + (size_t)h * S + i4;
        *(float4 *)&skb[tt][i4] = ok ? *(const float4 *)(KB + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        *(float4 *)&sv[tt][i4] = ok ? *(const float4 *)(v + o) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    const int j4 = (tid & 15) * 4;
    float * out = US + ((size_t)c * H + h) * S * S;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = (tid >> 4) + 16 * q;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int s = 0; s < L; s++) {
            const float kb = skb[s][i];
            const float4 vv = *(const float4 *)&sv[s][j4];
            a.x = fmaf(kb, vv.x, a.x);
            a.y = fmaf(kb, vv.y, a.y);
            a.z = fmaf(kb, vv.z, a.z);
            a.w = fmaf(kb, vv.w, a.w);
        }
        *(float4 *)(out + i * S + j4) = a;
    }
}

// The chunk-serial part, elementwise: thread per state element (h, i, j), S <- AL_c[i] S + U_c[i][j]
// over the chunks; the chunk-start states S_c replace U_c in place (read before the write).  The
// U_c / AL_c loads do not depend on the recurrence: D chunks are kept in flight.
__global__ __launch_bounds__(256) void k_wkv6c_carry(int nch, int H, const float * AL, float * US, const float * sin,
                                                     float * sout) {
    constexpr int S = WKVC_S, D = 8;
    const int e = blockIdx.x * 256 + threadIdx.x;  // h * 4096 + i * 64 + j
    const int h = e >> 12, i = (e >> 6) & 63, C = H * S;
    const size_t cs = (size_t)H * S * S;  // one chunk's states
    float * p = US + e;
    const float * al = AL + h * S + i;
    float st = sin[e];
    float u[D], a[D];
#pragma unroll
    for (int d = 0; d < D; d++) {
        u[d] = d < nch ? p[d * cs] : 0.0f;
        a[d] = d < nch ? al[(size_t)d * C] : 0.0f;
    }
    for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const int c = c0 + d;
            if (c < nch) {
                const float uc = u[d], ac = a[d];
                const int cn = c + D;
                u[d] = cn < nch ? p[cn * cs] : 0.0f;
                a[d] = cn < nch ? al[(size_t)cn * C] : 0.0f;
                p[c * cs] = st;
                st = fmaf(ac, st, uc);
            }
        }
    }
    sout[e] = st;
}

// y of one (chunk, head): y[t][j] = sum_i RA[t][i] S_c[i][j] + sum_{s<=t} B[t][s] v_s[j]; thread
// (t = tid / 16, j = 4 (tid % 16) ..) four outputs.
__global__ __launch_bounds__(256) void k_wkv6c_out(int T, int H, const float * RA, const float * Bm, const float * v,
                                                   const float * US, float * y) {
    constexpr int L = WKVC_L, S = WKVC_S;
    __shared__ __attribute__((aligned(16))) float ss[S][S], sra[L][S + 4], sb[L][L + 1], sv[L][S];
    const int c = blockIdx.x, h = blockIdx.y, tid = threadIdx.x, C = H * S, t0 = c * L;
    const float * sc = US + ((size_t)c * H + h) * S * S;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int idx = tid + 256 * q;
        *(float4 *)&ss[idx >> 4][(idx & 15) * 4] = *(const float4 *)(sc + idx * 4);
    }
    {
        const int tt = tid >> 4, i4 = (tid & 15) * 4;
        const bool ok = t0 + tt < T;
        const size_t o = (size_t)(t0 + tt) * C + (size_t)h * S + i4;
        *(float4 *)&sra[tt][i4] = ok ? *(const float4 *)(RA + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        *(float4 *)&sv[tt][i4] = ok ? *(const float4 *)(v + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        sb[tt][tid & 15] = Bm[((size_t)c * H + h) * (L * L) + tid];
    }
    __syncthreads();
    const int tt = tid >> 4, j4 = (tid & 15) * 4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
#pragma unroll 16
    for (int i = 0; i < S; i++) {
        const float ra = sra[tt][i];
        const float4 sv4 = *(const float4 *)&ss[i][j4];
        a.x = fmaf(ra, sv4.x, a.x);
        a.y = fmaf(ra, sv4.y, a.y);
        a.z = fmaf(ra, sv4.z, a.z);
        a.w = fmaf(ra, sv4.w, a.w);
    }
#pragma unroll
    for (int s2 = 0; s2 < L; s2++) {
        if (s2 <= tt) {
            const float bb = sb[tt][s2];
            const float4 vv = *(const float4 *)&sv[s2][j4];
            b.x = fmaf(bb, vv.x, b.x);
            b.y = fmaf(bb, vv.y, b.y);
            b.z = fmaf(bb, vv.z, b.z);
            b.w = fmaf(bb, vv.w, b.w);
        }
    }
    if (t0 + tt < T)
        *(float4 *)(y + (size_t)(t0 + tt) * C + (size_t)h * S + j4) = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

size_t wkv6_chunked_scratch_floats(int T, int H) {
    // B [nch][H][L][L], AL [nch][C], U / S_c [nch][H][64][64]
    const size_t nch = ((size_t)T + WKVC_L - 1) / WKVC_L;
    return nch * H * WKVC_L * WKVC_L + nch * H * WKVC_S + nch * H * WKVC_S * WKVC_S;
}

bool wkv6_chunked_supported(int T, int S, int bs) { return S == WKVC_S && bs == 0 && T >= 2; }

bool launch_wkv6_chunked(hipStream_t st, int T, int H, const float * k, const float * v, const float * r,
                         const float * u, const float * w, int w_per_token, const float * state_in, float * state_out,
                         float * y, float * RA, float * KB, float * scratch) {
    if (T < 1 || H < 1) return false;
    const int nch = (T + WKVC_L - 1) / WKVC_L;
    float * Bm = scratch;
    float * AL = Bm + (size_t)nch * H * WKVC_L * WKVC_L;
    float * US = AL + (size_t)nch * H * WKVC_S;
    if (w_per_token) RK_LAUNCH((k_wkv6c_prep<true>), dim3(nch, H), dim3(256), 0, st, T, H, k, r, w, u, RA, KB, Bm, AL);
    else RK_LAUNCH((k_wkv6c_prep<false>), dim3(nch, H), dim3(256), 0, st, T, H, k, r, w, u, RA, KB, Bm, AL);
    HIP_OK(hipGetLastError());
    RK_LAUNCH(k_wkv6c_u, dim3(nch, H), dim3(256), 0, st, T, H, KB, v, US);
    HIP_OK(hipGetLastError());
    RK_LAUNCH(k_wkv6c_carry, dim3(H * WKVC_S * WKVC_S / 256), dim3(256), 0, st, nch, H, AL, US, state_in, state_out);
    HIP_OK(hipGetLastError());
    RK_LAUNCH(k_wkv6c_out, dim3(nch, H), dim3(256), 0, st, T, H, RA, Bm, v, US, y);
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
