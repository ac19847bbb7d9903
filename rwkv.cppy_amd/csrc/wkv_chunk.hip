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
// Three launches per layer; only the second is serial, and only over chunks, elementwise:
//   k_wkv6c_prep  (chunk, head): la, RA = r 2^la, KB = k 2^(la_L - la_{s+1}), the L x L matrix B and
//                 AL = 2^la_L -- all the exp work;
//   k_wkv6c_carry (head, 4 key rows): S_{c+1} = AL_c S_c + KB_c^T V_c over the chunks, the chunk-start
//                 states S_c stored -- 64 chunk steps at T = 1024 instead of 1024 token steps;
//   k_wkv6c_out   (chunk, head): y = RA S_c + B V.
// Measured (v6-1B6 head count H = 32, rocprofv3 kernel trace of tools/wkv_chunk_time.py): T = 1024
// 21.6 + 32.5 + 17.2 = 71 us against 90.9 us for k_wkv6_s64; T = 4096 64 + 128 + 53 = 245 us against
// 350 us.  Earlier forms, not kept: the chunk-serial loop doing the whole y product per chunk (one
// workgroup per head and 8 columns) 105 us; U_c as its own kernel with an elementwise carry through
// memory 81 us.  The carry is bound by its S_c stores (32 MB at T = 1024) behind the loop-head
// vmcnt(0) the compiler keeps.
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

// The chunk-serial part: S_{c+1} = AL_c S_c + U_c with U_c[i][j] = sum_s KB[s][i] v_s[j] formed on the
// fly; the chunk-start states S_c go to SC for k_wkv6c_out.  Workgroup = (head, 4 key rows), thread
// (row i = 4 blockIdx.y + tid / 64, column j = tid % 64).  Chunks go in groups of G: a group's operands
// (v: 16 x 64, KB: 16 x 4, AL: 4 per chunk) are loaded global -> registers two groups ahead (one
// chunk's work is far shorter than a load's latency), then into one half of an LDS ring; one barrier
// per group, the G U_c products side by side, then the G dependent state steps.
constexpr int WKVC_G = 4;

__global__ __launch_bounds__(256) void k_wkv6c_carry(int T, int H, const float * KB, const float * v, const float * AL,
                                                     const float * sin, float * sout, float * SC) {
    constexpr int L = WKVC_L, S = WKVC_S, G = WKVC_G, D = 2 * G;
    __shared__ __attribute__((aligned(16))) float sv[2][G][L][S], skb[2][G][L][4], sal[2][G][4];
    const int h = blockIdx.x, ib = blockIdx.y, tid = threadIdx.x, C = H * S;
    const int r = tid >> 6, j = tid & 63, i = ib * 4 + r;
    const int nch = (T + L - 1) / L;
    const size_t hb = (size_t)h * S * S;
    float st = sin[hb + (size_t)i * S + j];
    // staging roles: v float4 (token tid / 16, columns 4 (tid % 16) ..); KB (tid < 64: token tid / 4,
    // row tid % 4); AL (tid < 4: row tid)
    const int vt = tid >> 4, vj = (tid & 15) * 4;
    float4 rv[D];
    float rk[D], ra[D];
    // every load unconditional from a clamped address, zeroed (by a select) only when it is stored to
    // LDS: a predicated load, or a select right behind it, makes the compiler wait for the load there
    auto load = [&](int d, int c) __attribute__((always_inline)) {
        const int cc = min(c, nch - 1), t0 = cc * L;
        const int tv = min(t0 + vt, T - 1), tk = min(t0 + (tid >> 2), T - 1);
        rv[d] = *(const float4 *)(v + (size_t)tv * C + (size_t)h * S + vj);
        rk[d] = KB[(size_t)tk * C + (size_t)h * S + ib * 4 + (tid & 3)];
        ra[d] = AL[(size_t)cc * C + (size_t)h * S + ib * 4 + (tid & 3)];
    };
#pragma unroll
    for (int d = 0; d < D; d++) load(d, d);
    // straight-line groups (no early exit: chunks past the end compute zeros and are not stored), so
    // the compiler's load counters stay exact across the loop
    for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
        for (int half = 0; half < 2; half++) {
            const int g0 = c0 + half * G;  // this group's first chunk
#pragma unroll
            for (int e = 0; e < G; e++) {
                const int d = half * G + e;
                const int t0 = (g0 + e) * L;  // token tails and chunks past the end: zeros
                *(float4 *)&sv[half][e][vt][vj] = t0 + vt < T ? rv[d] : make_float4(0.f, 0.f, 0.f, 0.f);
                if (tid < 64) skb[half][e][tid >> 2][tid & 3] = t0 + (tid >> 2) < T ? rk[d] : 0.0f;
                if (tid < 4) sal[half][e][tid] = ra[d];
                load(d, g0 + e + D);
            }
            __syncthreads();
            float u[G];
#pragma unroll
            for (int e = 0; e < G; e++) u[e] = 0.0f;
#pragma unroll
            for (int s = 0; s < L; s++)
#pragma unroll
                for (int e = 0; e < G; e++) u[e] = fmaf(skb[half][e][s][r], sv[half][e][s][j], u[e]);
#pragma unroll
            for (int e = 0; e < G; e++) {
                const int c = g0 + e;
                const bool live = c < nch;
                SC[(((size_t)c * H + h) * S + i) * S + j] = st;  // chunks past the end: padding slots
                const float nst = fmaf(sal[half][e][r], st, u[e]);
                st = live ? nst : st;
            }
        }
    }
    sout[hb + (size_t)i * S + j] = st;
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
    // B [nch][H][L][L], AL [nch][C], S_c [nch rounded up to 2 G][H][64][64]
    const size_t nch = ((size_t)T + WKVC_L - 1) / WKVC_L, ncp = (nch + 2 * WKVC_G - 1) / (2 * WKVC_G) * (2 * WKVC_G);
    return nch * H * WKVC_L * WKVC_L + nch * H * WKVC_S + ncp * H * WKVC_S * WKVC_S;
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
    RK_LAUNCH(k_wkv6c_carry, dim3(H, WKVC_S / 4), dim3(256), 0, st, T, H, KB, v, AL, state_in, state_out, US);
    HIP_OK(hipGetLastError());
    RK_LAUNCH(k_wkv6c_out, dim3(nch, H), dim3(256), 0, st, T, H, RA, Bm, v, US, y);
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
