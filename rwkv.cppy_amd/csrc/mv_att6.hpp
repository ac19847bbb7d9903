// mv_att6.hpp -- pieces shared by the two v6 fused attention decode launches (mv_att6f.hip, the
// ordered layout that needs no co-residency; mv_att6c.hip, the co-resident layout): the producer
// rows (k_mva's arithmetic) and the single-reader granules of the r / k / v / g / decay-LoRA
// hand-off.
#pragma once
#include "mv_common.hpp"

namespace rwkvmi {

typedef __attribute__((address_space(1))) unsigned gunsigned_t;

constexpr int AF_P = 8;   // workgroups per head
constexpr int AF_R = 8;   // rows per wave (4 waves x 8 rows x 8 workgroups = 4 x 64 rows)

// R rows of one matrix by one wave: k_mva's loads, dots, tree and epilogue (lane r: row r)
template <int WF, int R, int U>
__device__ __forceinline__ float af_rows(const DMat & W, const ActBuf & x, int row0, int epi, int lane) {
    const int M = W.M, K = W.K;
    int rows[R];
#pragma unroll
    for (int r = 0; r < R; r++) rows[r] = min(row0 + r, M - 1);
    WBlk w[R][U];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < R; r++) w[r][u] = load_unit<WF>(W, rows[r], u, lane);
    AUnit xu[U];
#pragma unroll
    for (int u = 0; u < U; u++) xu[u] = load_act_unit<WF, false>(x, u, lane);
    __builtin_amdgcn_sched_barrier(0);
    float acc[R], acc2[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = acc2[r] = 0.0f;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const bool valid = unit_valid<WF>(K, u, lane);
#pragma unroll
        for (int r = 0; r < R; r++) {
            float t = acc[r], t2 = acc2[r];
            dot_unit<WF>(w[r][u], xu[u], t, t2);
            acc[r] = valid ? t : acc[r];
            acc2[r] = valid ? t2 : acc2[r];
        }
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    float sr[R];
#pragma unroll
    for (int r = 0; r < R; r++) sr[r] = one ? wave_sum63(acc[r]) + wave_sum63(acc2[r]) : wave_sum63(acc[r]) + 0.0f;
    const float s = lane_row_sum<R>(sr, lane);
    return epi == EPI_SILU ? siluf_(s) : epi == EPI_TANH ? rk_tanhf(s) : s;
}

typedef __attribute__((address_space(1))) unsigned long long gu64_t;

// One granule = {tag 1 (high word), value bits (low word)}, ONE aligned 8-byte sc1 store: the data is
// its own flag (MI355X_MICROARCH.md hand-off R2, guide Guideline 16).  A consumer sweeps its
// granules until every tag reads 1 and then clears them to 0 (sc1), so the next launch can never
// see a stale value: a granule is only ever 0 (empty) or this launch's value.
__device__ __forceinline__ void gran_put(unsigned long long * g, float v) {
    __hip_atomic_store((gu64_t *)g, (1ull << 32) | (unsigned long long)__float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gran_put_tag(unsigned long long * g, float v, unsigned tag) {
    __hip_atomic_store((gu64_t *)g, ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long gran_get(const unsigned long long * g) {
    return __hip_atomic_load((gu64_t *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gran_clear(unsigned long long * g) {
    __hip_atomic_store((gu64_t *)g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave sweeps N granules per lane (stride S) until every tag is set; bounded (timeout: *err, a
// host-mapped word, stored at system scope so the host sees it after the stream synchronises).
template <int N>
__device__ __forceinline__ void gran_sweep(const unsigned long long * g, int stride, bool (&live)[N], float (&v)[N],
                                           unsigned * err, unsigned spin_max) {
    for (unsigned it = 0;; it++) {
        bool ok = true;
        unsigned long long x[N];
#pragma unroll
        for (int k = 0; k < N; k++) x[k] = live[k] ? gran_get(g + k * stride) : (1ull << 32);
#pragma unroll
        for (int k = 0; k < N; k++) {
            v[k] = __uint_as_float((unsigned)x[k]);
            ok = ok && (x[k] >> 32) == 1ull;
        }
        if (__all(ok)) return;
        if (it >= spin_max) {
            __hip_atomic_store((gunsigned_t *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

}  // namespace rwkvmi
