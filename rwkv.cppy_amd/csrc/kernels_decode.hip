// kernels_decode.hip -- single-token (decode) kernels for gfx950.
//
// Decode is a chain of dependent matvecs over HBM-resident weights.  To keep the chain short,
// every matvec workgroup builds its own input in LDS from fp32 vectors that sit in L2 (the
// previous kernel's output): LayerNorm statistics, token-shift mix and the ggml Q8
// activation quantization are recomputed per workgroup (a few KB of L2 reads) instead of
// costing a separate launch.  Per-head attention work (decay LoRA tail, wkv, GroupNorm) is
// one kernel with the head's state in registers.  The matvec itself lives in mv_common.hpp;
// its launch shapes are instantiated per weight type in mv_*.hip.
#include "mv_common.hpp"

namespace rwkvmi {

// instantiated in the mv_*.hip units
extern template bool launch_mv_shape<-1>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
extern template bool launch_mv_shape<W_F16>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
extern template bool launch_mv_shape<W_Q4_0>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
extern template bool launch_mv_shape<W_Q4_1>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
extern template bool launch_mv_shape<W_Q5_0>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
extern template bool launch_mv_shape<W_Q5_1>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
extern template bool launch_mv_shape<W_Q8_0>(hipStream_t, MVGroup &, int, int, int, bool, dim3);

static int g_mv_cus = 256;

// Rows per wave of k_mva: 2.  More rows per wave put more weight loads in flight per lane behind
// fewer workgroups; measured on the v6-1B6 decode chain (128 tokens): 2 rows 853 us/token, 4 rows
// 883, 8 rows 876 -- the launch stays latency bound and two rows keep the most waves issuing.
int mva_rows() { return 2; }
extern int kQgCUs;
void set_mv_device_cus(int n) {
    g_mv_cus = n > 0 ? n : 256;
    kQgCUs = g_mv_cus;
}

bool launch_mv_group(hipStream_t st, MVGroup & g) {
    g.late = 0;  // weight streams start with the image inputs (holding them: v6-1B6 686 vs 678 us/token)
    bool emit = false;
    for (int i = 0; i < g.n; i++) emit |= g.e[i].emit != 0;
    const int src = g.e[0].src, form = g.e[0].form;
    for (int i = 1; i < g.n; i++)
        if (g.e[i].src != src || (src == SRC_LNMIX && g.e[i].form != form)) {
            fprintf(stderr, "rwkv: matvec group mixes input sources / token-shift forms\n");
            return false;
        }
    const bool prologue = src != SRC_ACT;
    const int srck = src == SRC_ACT ? MVK_ACT : src == SRC_F32 ? MVK_F32 : MVK_LN;
    if (emit && src == SRC_LNMIX && form == 2) {
        fprintf(stderr, "rwkv: emitting matvec with a plain LayerNorm input is not instantiated\n");
        return false;
    }
    if (emit && !prologue) {
        fprintf(stderr, "rwkv: emitting matvec needs a prologue source\n");
        return false;
    }
    // rows per wave: 8 when emitting (a 32-row block per workgroup), else 2; the lean
    // activation-input kernel k_mva (one weight type, <= 4 units per lane) takes mva_rows()
    int wfix = g.e[0].W.type;
    for (int i = 1; i < g.n; i++)
        if (g.e[i].W.type != wfix) wfix = -1;
    int umax0 = 1;
    for (int i = 0; i < g.n; i++) umax0 = std::max(umax0, mv_units(g.e[i].W.type, g.e[i].W.K));
    const bool mva = !prologue && !emit && wfix >= 0 && umax0 <= 4;
    // LayerNorm-prologue groups (not emitting) with more than two workgroups per CU at 2 rows per
    // wave (v7 r,k,v: 960; v5 r,k,v,g: 2048) take 4 rows per wave: one round of workgroups fewer
    // (v7-2.9B decode 469 -> 490 tok/s alone, with U = 1 above 513; v5-7B 517 -> 573)
    constexpr int ln_r4 = 1;
    int rows2 = 0;
    for (int i = 0; i < g.n; i++) rows2 += (g.e[i].W.M + 7) / 8;
    const bool r4 = ln_r4 && prologue && !emit && srck == MVK_LN && (g.n > 1 || rows2 <= 8 * g_mv_cus) &&
                    rows2 > 2 * g_mv_cus;
    // ... and 8 rows per wave when even 4 leave more than four workgroups per CU (K > 2048, two units
    // per lane: v5-7B r,k,v,g, 1024 -> 512 workgroups; decode 1557 -> 1535 us/token, bit-exact; v7's
    // r,k,v at 480 workgroups measured neutral and stays at 4).  That shape takes its two units in two
    // round trips (U = 1, launch_mv_shape): at U = 2 it held 153 VGPRs, one workgroup per CU, and its
    // 512 workgroups ran in two rounds (v5-7B decode 1525-1528 -> 1485-1487 us/token)
    constexpr int ln_r8 = 1;
    int lnk = 0;
    for (int i = 0; i < g.n; i++) lnk = std::max(lnk, g.e[i].W.K);
    const bool r8 = ln_r8 && r4 && lnk > 2048 && umax0 == 2 && rows2 > 4 * g_mv_cus;
    const int R = emit ? 8 : mva ? mva_rows() : r8 ? 8 : r4 ? 4 : 2, RW = 4 * R;
    g.rows = R;
    int blocks = 0, umax = 1, lds = 0;
    for (int i = 0; i < g.n; i++) {
        MVEntry & e = g.e[i];
        if (e.W.K % 32) {
            fprintf(stderr, "rwkv: matvec needs K %% 32 == 0 (K=%d)\n", e.W.K);
            return false;
        }
        if (e.src == SRC_LNMIX && (e.W.K % 64 || e.W.K > 64 * 128)) {
            fprintf(stderr, "rwkv: LayerNorm prologue needs K %% 64 == 0 and K <= 8192 (K=%d)\n", e.W.K);
            return false;
        }
        if (e.emit && e.W.M % 32) {
            fprintf(stderr, "rwkv: emitting matvec needs M %% 32 == 0 (M=%d)\n", e.W.M);
            return false;
        }
        if (e.src == SRC_ACT && (e.act.K != e.W.K || e.act.fmt != act_fmt_for(e.W.type))) {
            fprintf(stderr, "rwkv: matvec input format/size mismatch (K=%d vs %d)\n", e.act.K, e.W.K);
            return false;
        }
        e.block0 = blocks;
        blocks += (e.W.M + RW - 1) / RW;
        umax = std::max(umax, mv_units(e.W.type, e.W.K));
        if (e.src != SRC_ACT) lds = std::max(lds, lds_bytes_for(act_fmt_for(e.W.type), e.W.K));
    }
    g.lds_bytes = lds;
    g.units_max = umax;
    for (int i = 0; i < g.n; i++) {
        const MVEntry & e = g.e[i];
        MVHot & h = g.hot[i];
        h.qs = e.W.qs;
        h.qh = e.W.qh;
        h.sc = e.W.sc;
        h.aq = e.act.q;
        h.ad = e.act.d;
        h.as = e.act.s;
        h.aqsum = e.act.qsum;
        h.ahf = e.act.fmt == A_F16 ? (const void *)e.act.h : (const void *)e.act.f;
        h.y = e.y;
        h.aux = e.aux;
        h.bias = e.bias;
        h.M = e.W.M;
        h.K = e.W.K;
        h.epi = e.epi;
        h.steps = (e.aux ? 1 : 0) | (e.bias ? 2 : 0);
    }
    if (!blocks) return true;
    // a single large prologue entry (the head): persistent walk over its row blocks, one
    // LayerNorm per workgroup
    g.stride = 0;
    int grid = blocks;
    if (prologue && g.n == 1 && !emit && blocks > 8 * g_mv_cus) {
        grid = 2 * g_mv_cus;
        g.stride = grid;
    }
    g.grid = grid;
    int U = umax <= 1 ? 1 : umax <= 2 ? 2 : 4;  // 2: K = 2560 (v7-2.9B) quantized rows
    // emitting LayerNorm groups at U = 2 hold 16 weight units per wave (184 VGPRs: one workgroup
    // per CU); with more row blocks than CUs, U = 1 (two round trips, 122 VGPRs, two per CU):
    // v7-2.9B FFN key, 320 workgroups -- decode 469 -> 489 tok/s alone
    constexpr int emit_u1 = 1;
    if (emit_u1 && emit && U == 2 && blocks > g_mv_cus) U = 1;
    // activation-input rows of 5..8 quantized units per lane (v7-2.9B FFN value, K = 10240): all
    // units in one round of loads instead of 4 + the rest
    constexpr int act_u8 = 1;
    if (act_u8 && srck == MVK_ACT && !mva && umax > 4 && umax <= 8 && wfix >= 0 && wtype_quantized(wfix)) U = 8;
    // F16 LayerNorm groups of 5-8 units per lane (v7-2.9B LoRA first stages, K = 2560): one round
    constexpr int f16_u8 = 1;
    if (f16_u8 && srck == MVK_LN && !emit && wfix == W_F16 && R == 2 && umax > 4 && umax <= 8 && lnk > 2048) U = 8;
    bool ok = false;
    switch (wfix) {
        case W_F16: ok = launch_mv_shape<W_F16>(st, g, U, srck, form, emit, dim3(grid)); break;
        case W_Q4_0: ok = launch_mv_shape<W_Q4_0>(st, g, U, srck, form, emit, dim3(grid)); break;
        case W_Q4_1: ok = launch_mv_shape<W_Q4_1>(st, g, U, srck, form, emit, dim3(grid)); break;
        case W_Q5_0: ok = launch_mv_shape<W_Q5_0>(st, g, U, srck, form, emit, dim3(grid)); break;
        case W_Q5_1: ok = launch_mv_shape<W_Q5_1>(st, g, U, srck, form, emit, dim3(grid)); break;
        case W_Q8_0: ok = launch_mv_shape<W_Q8_0>(st, g, U, srck, form, emit, dim3(grid)); break;
        default: ok = launch_mv_shape<-1>(st, g, U, srck, form, emit, dim3(grid)); break;
    }
    if (!ok) return false;
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v6 mix5 (decode)
struct Mix5Dec {
    int C, D;
    const float * xa, * carry, * lora, * w2t;
    const float * maa[5];
    ActBuf out[5];
    // batched decode (grid.z = contexts): context b's xa / sx (xp - xa) rows at + b*C, lora at
    // + b*5D, output row b; carry is then unused
    const float * sx;
};

// grid (C/256, 5[, B]): block (cx, n[, b]) computes mixed vector n for 256 channels from xa = LN(x),
// which the preceding W1 matvec already wrote as the new att_xx carry.  w2t [5][D][C] makes
// the per-channel D-long dots coalesced across lanes; accumulation order matches the oracle
// (one fp32 fma chain, sequential over i).
__global__ __launch_bounds__(256) void k_v6_mix5_dec(Mix5Dec a) {
    const int n = blockIdx.y, C = a.C, D = a.D, b = blockIdx.z;
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if ((int)(blockIdx.x * blockDim.x + (threadIdx.x & ~31)) >= C) return;  // half-wave uniform
    float w2v[64];
    const float * w2 = a.w2t + (size_t)n * D * C + c;
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const float t = w2[(size_t)min(i, D - 1) * C];
        w2v[i] = (i < D) ? t : 0.0f;
    }
    const size_t cb = (size_t)b * C;
    const float xa = a.xa[cb + c], mu = a.maa[n][c];
    const float sx = a.sx ? a.sx[cb + c] : a.carry[c] - xa;
    const float * lv = a.lora + (size_t)b * 5 * D + n * D;
    float m = 0.0f;
#pragma unroll
    for (int i = 0; i < 64; i++)
        if (i < D) m = fmaf(w2v[i], lv[i], m);
    emit32(a.out[n], b, c, (m + mu) * sx + xa);
}

bool launch_v6_mix5_dec(hipStream_t st, int C, int D, const float * xa, const float * carry, const float * lora,
                        const float * w2t, const float * const * maa, const ActBuf * outs, int nb, const float * sx) {
    Mix5Dec a;
    a.C = C;
    a.D = D;
    a.xa = xa;
    a.carry = carry;
    a.lora = lora;
    a.w2t = w2t;
    a.sx = sx;
    for (int n = 0; n < 5; n++) {
        a.maa[n] = maa[n];
        a.out[n] = outs[n];
    }
    if (D > 64 || C % 32 || (nb > 1 && !sx)) {
        fprintf(stderr, "rwkv: v6 maa LoRA width %d / n_embed %d unsupported\n", D, C);
        return false;
    }
    dim3 grid((C + 255) / 256, 5, nb > 1 ? nb : 1);
    RK_LAUNCH(k_v6_mix5_dec, grid, dim3(256), 0, st, a);
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v5/v6 attention (decode)
// One row by one wave, exactly k_mm's loop (any K).
template <int WF>
__device__ __forceinline__ float decay_row_wave(const DMat & W, int row, const ActBuf & act, int lane) {
    float acc = 0.0f, acc2 = 0.0f;
    const int units = mv_units(WF, W.K);
    for (int u = 0; u < units; u++) {
        const WBlk w = load_unit<WF>(W, row, u, lane);
        const AUnit x = load_act_unit<WF, true>(act, u, lane);
        if (unit_valid<WF>(W.K, u, lane)) dot_unit<WF>(w, x, acc, acc2);
    }
    constexpr bool one = WF == W_Q4_1 || WF == W_Q5_1;
    return one ? wave_sum63(acc) + wave_sum63(acc2) : wave_sum63(acc) + 0.0f;
}

// lanes of k_mm that hold a unit of a K-long row, when each holds at most one; else 0
__host__ __device__ inline int one_unit_lanes(int type, int K) {
    const int per = type == W_F32 ? 4 : type == W_F16 ? 8 : 32;
    const int n = K / per;
    return n <= 64 ? n : 0;
}

template <int WF>
__device__ __forceinline__ void decay_rows(const Att6Dec & a, const ActBuf & act, float * sw, int c0, int S) {
    const int tid = threadIdx.x;
    const int nl = one_unit_lanes(WF, a.wd2.K);
    if (nl > 0 && nl <= 16) {
        const WBlk none[1] = {};
        if (tid < S) {
            const float s = decay_row_thread<WF, 0, 16>(a.wd2, c0 + tid, act, nl, none);
            sw[tid] = rk_expf(-rk_expf(s + a.decay[c0 + tid]));
        }
    } else {
        const int lane = tid & 63, nw = blockDim.x >> 6;
        for (int j = tid >> 6; j < S; j += nw) {
            const float s = decay_row_wave<WF>(a.wd2, c0 + j, act, lane);
            if (lane == 63) sw[j] = rk_expf(-rk_expf(s + a.decay[c0 + j]));
        }
    }
}

// One workgroup per head, S*G threads (G = min(256/S, S), as the sequence kernel k_wkv6):
// thread (j = tid % S, g = tid / S) owns state column j for keys i in [g*IPG, (g+1)*IPG) --
// each state load/store instruction covers S consecutive floats.  The per-thread partial y
// sums meet in LDS and are folded with group_sum's butterfly tree, so decode and sequence
// agree bit for bit.  PF > 0: quantized decay LoRA with <= PF units per row, prefetched.
// SS = 64: head size 64 at compile time (straight-line state loop, constant store offsets);
// SS = 0: any head size from a.S.
template <int WF, int PF, int SS>
__global__ __launch_bounds__(256) void k_att6_dec(Att6Dec a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ __attribute__((aligned(16))) float sr[64], sk[64], sv[64], sw[64], su[64];
    __shared__ float part[16][64];
    const int h = blockIdx.x, S = SS ? SS : a.S, G = SS ? 256 / SS : min(256 / S, S), IPG = S / G;
    const int tid = threadIdx.x, j = tid % S, g = min(tid / S, G - 1), c0 = h * S;
    const bool active = SS ? true : tid < S * G;  // SS: the block is exactly S * G threads
    const size_t hb = (size_t)h * S * S;
    // batched decode: context blockIdx.y (its [C] vectors, decay LoRA row and state); 0 in decode
    const int bz = blockIdx.y;
    const size_t cb = (size_t)bz * a.H * S;
    const float * ar = a.r + cb, * ak = a.k + cb, * av = a.v + cb;
    const float * ag = a.g ? a.g + cb : nullptr;
    const float * adl = a.dl ? a.dl + (size_t)bz * a.ldd : nullptr;
    const float * asin = a.sin + (size_t)bz * a.bs;
    float * asout = a.sout + (size_t)bz * a.bs;
    STAMP_BEGIN();
    WBlk wp[PF > 0 ? PF : 1];
    if constexpr (PF > 0) {
        const int nb = a.wd2.K >> 5;
        const int row = c0 + min(tid, S - 1);
#pragma unroll
        for (int l = 0; l < PF; l++) wp[l] = load_wblk<WF>(a.wd2, (size_t)row * nb + min(l, nb - 1));
    }
    // per-channel operands of the decay tail and the GroupNorm epilogue, loaded now so they
    // are not a dependent round trip behind the barriers
    const int cme = c0 + min(tid, S - 1);
    const float lnw_c = a.lnx_w[cme], lnb_c = a.lnx_b[cme];
    const float g_c = ag ? ag[cme] : 1.0f;
    const float dec_c = a.w ? 0.0f : a.decay[cme];
    const float r_c = ar[cme], k_c = ak[cme], v_c = av[cme], u_c = a.u[cme];
    const float w_c = a.w ? a.w[cme] : 0.0f;
    const bool dlo = WF != -2 && !a.w;
    float dl_c = 0.0f;
    if (dlo && tid < a.wd2.K) dl_c = adl[tid];
    // the state columns last: the operand loads above retire first (in-order vmcnt), so the
    // decay tail below runs while the state is still in flight
    float st[16];
#pragma unroll
    for (int ii = 0; ii < 16; ii++)
        st[ii] = ii < IPG && active ? asin[hb + (size_t)(g * IPG + ii) * S + j] : 0.0f;
    if (tid < S) {
        sr[tid] = r_c;
        sk[tid] = k_c;
        sv[tid] = v_c;
        su[tid] = u_c;
        if (a.w) sw[tid] = w_c;
    }
    ActBuf act;
    if (dlo) {
        // v6 decay LoRA tail: w = exp(-exp(Wd2 . dl + decay)), rwkv_graph.inc:357-367
        const int D = a.wd2.K;
        act = lds_act(smem, act_fmt_for(a.wd2.type), D);
        if (PF > 0 || D <= (int)blockDim.x) {  // PF > 0: D <= 32 * PF
            if ((tid & ~31) < D) emit32(act, 0, tid, dl_c);
        } else {
            for (int k0 = 0; k0 < D; k0 += blockDim.x) {
                if (k0 + (tid & ~31) >= D) continue;
                emit32(act, 0, k0 + tid, adl[k0 + tid]);
            }
        }
    }
    __syncthreads();
    STAMP_MID();
    if (WF != -2 && !a.w) {
        if constexpr (WF == -2) {
        } else if constexpr (PF > 0) {
            if (tid < S) {
                const float s = decay_row_thread<WF, PF, PF>(a.wd2, c0 + tid, act, a.wd2.K >> 5, wp);
                sw[tid] = rk_expf(-rk_expf(s + dec_c));
            }
        } else {
            switch (a.wd2.type) {
                case W_F32: decay_rows<W_F32>(a, act, sw, c0, S); break;
                case W_F16: decay_rows<W_F16>(a, act, sw, c0, S); break;
                case W_Q4_0: decay_rows<W_Q4_0>(a, act, sw, c0, S); break;
                case W_Q4_1: decay_rows<W_Q4_1>(a, act, sw, c0, S); break;
                case W_Q5_0: decay_rows<W_Q5_0>(a, act, sw, c0, S); break;
                case W_Q5_1: decay_rows<W_Q5_1>(a, act, sw, c0, S); break;
                case W_Q8_0: decay_rows<W_Q8_0>(a, act, sw, c0, S); break;
                default: break;
            }
        }
        __syncthreads();
    }
    STAMP_X(0);
    // wkv6 for one token (ggml_rwkv_wkv6 semantics, same arithmetic as the sequence kernels).
    // Head size 64 (IPG 16): the group's sum is (p0 + p1) + (p2 + p3) over its four 4-key runs,
    // k_wkv6_s64's association; other head sizes: one sequential run (k_wkv6's).
    if (active) {
        const float vj = sv[j];
        // the group's key operands into registers first (all LDS reads in flight at once; head
        // size 64: 16-byte reads), then the arithmetic -- same operations, same order
        float kq[16], uq[16], rq[16], wq[16];
        if (IPG == 16) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const float4 k4 = *(const float4 *)(sk + g * 16 + 4 * q), u4 = *(const float4 *)(su + g * 16 + 4 * q);
                const float4 r4 = *(const float4 *)(sr + g * 16 + 4 * q), w4 = *(const float4 *)(sw + g * 16 + 4 * q);
                kq[4 * q] = k4.x, kq[4 * q + 1] = k4.y, kq[4 * q + 2] = k4.z, kq[4 * q + 3] = k4.w;
                uq[4 * q] = u4.x, uq[4 * q + 1] = u4.y, uq[4 * q + 2] = u4.z, uq[4 * q + 3] = u4.w;
                rq[4 * q] = r4.x, rq[4 * q + 1] = r4.y, rq[4 * q + 2] = r4.z, rq[4 * q + 3] = r4.w;
                wq[4 * q] = w4.x, wq[4 * q + 1] = w4.y, wq[4 * q + 2] = w4.z, wq[4 * q + 3] = w4.w;
            }
        } else {
#pragma unroll
            for (int ii = 0; ii < 16; ii++) {
                const int i = g * IPG + min(ii, IPG - 1);
                kq[ii] = sk[i], uq[ii] = su[i], rq[ii] = sr[i], wq[ii] = sw[i];
            }
        }
        float acc = 0.0f, p4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int ii = 0; ii < 16; ii++) {
            if (ii < IPG) {
                const int i = g * IPG + ii;
                const float prev = st[ii];
                const float kv = vj * kq[ii];
                const float temp = kv * uq[ii] + prev;
                const float t = temp * rq[ii];
                acc += t;
                p4[ii >> 2] += t;
                asout[hb + (size_t)i * S + j] = prev * wq[ii] + kv;
            }
        }
        part[g][j] = IPG == 16 ? (p4[0] + p4[1]) + (p4[2] + p4[3]) : acc;
    }
    __syncthreads();
    STAMP_X(1);
    // GroupNorm over the head (ggml_norm, fp64 sums) * ln_x (+ b) (* g)
    if (tid < S) {
        float p[16];
#pragma unroll
        for (int q = 0; q < 16; q++) p[q] = q < G ? part[q][tid] : 0.0f;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1)
            if (o < G)
#pragma unroll
                for (int q = 0; q < o; q++) p[q] = p[q] + p[q + o];
        const float x = p[0];
        const double s = group_tree_sum_d((double)x, S);
        const float mean = (float)div_count(s, S);
        const float d = x - mean;
        const double s2 = group_tree_sum_d((double)(d * d), S);
        const float var = (float)div_count(s2, S);
        const float scale = 1.0f / sqrtf(var + a.eps);
        float o = d * scale;
        o = o * lnw_c;
        o = o + lnb_c;
        if (ag) o = o * g_c;
        if (a.yq.fmt >= 0) emit32(a.yq, bz, c0 + tid, o);  // S >= 32: whole half-wave blocks
        else a.y[cb + c0 + tid] = o;
    }
    STAMP_END(3);
}

bool launch_att6_dec(hipStream_t st, const Att6Dec & a) {
    if (a.S > 64 || (a.S & (a.S - 1))) {
        fprintf(stderr, "rwkv: head size %d unsupported\n", a.S);
        return false;
    }
    int G = 256 / a.S;
    if (G > a.S) G = a.S;
    const int threads = a.S * G;
    int lds = 0;
    if (!a.w) {
        const int D = a.wd2.K;
        if (D % 32) {
            fprintf(stderr, "rwkv: v6 decay LoRA width %d unsupported\n", D);
            return false;
        }
        lds = lds_bytes_for(act_fmt_for(a.wd2.type), D);
    }
    if (a.yq.fmt >= 0 && a.S < 32) {
        fprintf(stderr, "rwkv: quantized attention output needs head size >= 32\n");
        return false;
    }
    dim3 grid(a.H, a.nb > 1 ? a.nb : 1), block(std::max(threads, 64));
    const bool pf = !a.w && a.wd2.type >= W_Q4_0 && (a.wd2.K >> 5) <= 4;
    const bool s64 = a.S == 64;
#define ATT6(WFv, PFv)                                                                         \
    do {                                                                                       \
        if (s64) RK_LAUNCH((k_att6_dec<WFv, PFv, 64>), grid, block, lds, st, a);      \
        else RK_LAUNCH((k_att6_dec<WFv, PFv, 0>), grid, block, lds, st, a);           \
    } while (0)
    if (a.w) {
        ATT6(-2, 0);  // v5: no decay LoRA
    } else if (!pf) {
        ATT6(-1, 0);
    } else {
        switch (a.wd2.type) {
            case W_Q4_0: ATT6(W_Q4_0, 4); break;
            case W_Q4_1: ATT6(W_Q4_1, 4); break;
            case W_Q5_0: ATT6(W_Q5_0, 4); break;
            case W_Q5_1: ATT6(W_Q5_1, 4); break;
            default: ATT6(W_Q8_0, 4); break;
        }
    }
#undef ATT6
    HIP_OK(hipGetLastError());
    return true;
}

// Sequence path, v6 decay LoRA tail: w[t][c] = exp(-exp(Wd2[c] . Q8(dl[t]) + decay[c])), one thread
// per channel over DECAY_TT tokens with decay_row_thread -- k_att6_dec's arithmetic, so decode and
// sequence agree bit for bit.  Replaces the f32->Q8 conversion + K = D GEMM launch pair (a 2-block
// GEMM is all fixed cost on the MFMA path).  Workgroup = DECAY_TT tokens x 256 channels: the
// tokens' Q8 images sit in LDS, the thread's Wd2 row units stay in registers across the tokens.
constexpr int DECAY_TT = 4;  // 4: 2048 workgroups at T = 1024 (16: 512, 14.4 us)

template <int WF>
__global__ __launch_bounds__(256) void k_v6_decay_seq(int T, int C, DMat wd2, const float * dl, const float * decay,
                                                      float * w) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t0 = blockIdx.x * DECAY_TT, D = wd2.K, tid = threadIdx.x, nb = D >> 5;
    const int fmt = act_fmt_for(WF), abytes = (lds_bytes_for(fmt, D) + 15) & ~15;
    const int row = min((int)blockIdx.y * 256 + tid, C - 1);
    WBlk wp[4];
#pragma unroll
    for (int l = 0; l < 4; l++) wp[l] = load_wblk<WF>(wd2, (size_t)row * nb + min(l, nb - 1));  // re-read: cached
    const float dec = decay[row];
    // D % 32 == 0, so every 32 consecutive e are one quantization block of one token
    for (int e = tid; e < DECAY_TT * D; e += 256) {
        const int tt = e / D, k = e % D;
        const ActBuf act = lds_act(smem + tt * abytes, fmt, D);
        emit32(act, 0, k, dl[(size_t)min(t0 + tt, T - 1) * D + k]);
    }
    __syncthreads();
    if ((int)blockIdx.y * 256 + tid >= C) return;
    const int nt = min(DECAY_TT, T - t0);
    for (int tt = 0; tt < nt; tt++) {
        const ActBuf act = lds_act(smem + tt * abytes, fmt, D);
        const float s = decay_row_thread<WF, 4, 4>(wd2, row, act, nb, wp);
        w[(size_t)(t0 + tt) * C + row] = rk_expf(-rk_expf(s + dec));
    }
}

bool v6_decay_seq_supported(int wd2_type, int D) {
    return wd2_type >= W_Q4_0 && D % 32 == 0 && D >= 32 && D <= 128;
}

bool launch_v6_decay_seq(hipStream_t st, int T, int C, const DMat & wd2, const float * dl, const float * decay,
                         float * w) {
    if (!v6_decay_seq_supported(wd2.type, wd2.K) || wd2.M != C) {
        fprintf(stderr, "rwkv: v6 decay tail: unsupported shape (%d x %d, type %d)\n", (int)wd2.M, (int)wd2.K,
                (int)wd2.type);
        return false;
    }
    const dim3 grid((T + DECAY_TT - 1) / DECAY_TT, (C + 255) / 256);
    const int lds = DECAY_TT * ((lds_bytes_for(act_fmt_for(wd2.type), wd2.K) + 15) & ~15);
    switch (wd2.type) {
        case W_Q4_0: RK_LAUNCH(k_v6_decay_seq<W_Q4_0>, grid, dim3(256), lds, st, T, C, wd2, dl, decay, w); break;
        case W_Q4_1: RK_LAUNCH(k_v6_decay_seq<W_Q4_1>, grid, dim3(256), lds, st, T, C, wd2, dl, decay, w); break;
        case W_Q5_0: RK_LAUNCH(k_v6_decay_seq<W_Q5_0>, grid, dim3(256), lds, st, T, C, wd2, dl, decay, w); break;
        case W_Q5_1: RK_LAUNCH(k_v6_decay_seq<W_Q5_1>, grid, dim3(256), lds, st, T, C, wd2, dl, decay, w); break;
        default: RK_LAUNCH(k_v6_decay_seq<W_Q8_0>, grid, dim3(256), lds, st, T, C, wd2, dl, decay, w); break;
    }
    HIP_OK(hipGetLastError());
    return true;
}

// --------------------------------------------------------------------------- v7 attention (decode)
template <int JPG>
__global__ __launch_bounds__(1024) void k_att7_dec(Att7Dec a) {
    __shared__ float sr[64], sw[64], sk[64], sv[64], snb[64], sbb[64], sy[64];
    __shared__ float sbonus;
    const int h = blockIdx.x, S = a.S, G = S / JPG;
    const int tid = threadIdx.x, c0 = h * S;
    // batched decode: context blockIdx.y (0 in decode)
    const int bz = blockIdx.y;
    const size_t cb = (size_t)bz * a.H * S;
    const float * asin = a.sin + (size_t)bz * a.bs;
    float * asout = a.sout + (size_t)bz * a.bs;
    // the per-channel operands (prep and GroupNorm epilogue) are loaded first and the state rows
    // after them: the prep below waits only for the operands (in-order vmcnt) while the state is
    // still in flight, and nothing is a dependent round trip behind the barriers
    const bool wact = tid < S * G;
    const int wi = min(tid / G, S - 1), wg = tid % G;
    const size_t wbase = (size_t)h * S * S + (size_t)wi * S + wg * JPG;
    const int cme = c0 + min(tid, S - 1);
    const float lnw_c = a.lnx_w[cme], lnb_c = a.lnx_b[cme], g_c = a.g[cb + cme];
    const float k_c = a.k[cb + cme], kk_c = a.k_k[cme], a_c = a.a[cb + cme], ka_c = a.k_a[cme];
    const float r_c = a.r[cb + cme], w_c = a.w[cb + cme], v_c = a.v[cb + cme], rk_c = a.r_k[cme];
    __builtin_amdgcn_sched_barrier(0);  // keep the state loads behind the operand loads
    float st[JPG];
#pragma unroll
    for (int jj = 0; jj < JPG; jj++) st[jj] = asin[wbase + jj];
    if (tid < S) {
        // prep (rwkv_graph.inc:432-437 + rwkv_operators.inc:40-82)
        const float kv = k_c;
        const float kkr = kv * kk_c;
        const float sum = group_sum(kkr * kkr, S);
        const float scale = 1.0f / fmaxf(sqrtf(sum), 1e-12f);
        const float kk = kkr * scale;
        const float av = a_c;
        const float ka = kv * ka_c;
        const float kadj = kv + (av * ka - ka);
        const float rv = r_c;
        sr[tid] = rv;
        sw[tid] = w_c;
        sk[tid] = kadj;
        sv[tid] = v_c;
        snb[tid] = -kk;
        sbb[tid] = kk * av;
        const float bs = group_sum((kadj * rv) * rk_c, S);
        if (tid == 0) sbonus = bs;
    }
    __syncthreads();
    if (wact) {
        // wkv7 (rwkv_operators_wkv_v7.inc:37-107): state [h][i(value)][j(key)], g splits j
        const int i = wi, g = wg;
        const size_t base = wbase;
        float sa = 0.0f;
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) sa += snb[g * JPG + jj] * st[jj];
        sa = group_sum(sa, G);
        const float vi = sv[i];
        float acc = 0.0f;
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) {
            const int j = g * JPG + jj;
            const float kv = vi * sk[j];
            const float ns = st[jj] * sw[j] + kv + sa * sbb[j];
            asout[base + jj] = ns;
            acc += ns * sr[j];
        }
        acc = group_sum(acc, G);
        if (g == 0) sy[i] = acc;
    }
    __syncthreads();
    if (tid < S) {
        const int c = c0 + tid;
        const float x = sy[tid];
        const double s = group_tree_sum_d((double)x, S);
        const float mean = (float)div_count(s, S);
        const float d = x - mean;
        const double s2 = group_tree_sum_d((double)(d * d), S);
        const float var = (float)div_count(s2, S);
        const float scale = 1.0f / sqrtf(var + 64e-5f);
        float o = d * scale;
        o = o * lnw_c;
        o = o + lnb_c;
        o = o + sv[tid] * sbonus;
        o = o * g_c;
        if (a.yq.fmt >= 0) emit32(a.yq, bz, c, o);  // S >= 32: whole half-wave blocks
        else a.y[cb + c] = o;
    }
}

bool launch_att7_dec(hipStream_t st, const Att7Dec & a) {
    if (a.S > 64 || (a.S & (a.S - 1))) {
        fprintf(stderr, "rwkv: head size %d unsupported\n", a.S);
        return false;
    }
    // keys per lane: 4 at head size 64 (16 groups, k_wkv7_s64's split), else pick_groups' split
    int G = a.S == 64 ? 16 : 256 / a.S;
    if (G > a.S) G = a.S;
    const int JPG = a.S / G;
    const int threads = std::max(64, a.S * G);
    if (a.yq.fmt >= 0 && a.S < 32) {
        fprintf(stderr, "rwkv: quantized attention output needs head size >= 32\n");
        return false;
    }
    dim3 grid(a.H, a.nb > 1 ? a.nb : 1), block(threads);
    switch (JPG) {
        case 1: RK_LAUNCH(k_att7_dec<1>, grid, block, 0, st, a); break;
        case 2: RK_LAUNCH(k_att7_dec<2>, grid, block, 0, st, a); break;
        case 4: RK_LAUNCH(k_att7_dec<4>, grid, block, 0, st, a); break;
        case 8: RK_LAUNCH(k_att7_dec<8>, grid, block, 0, st, a); break;
        case 16: RK_LAUNCH(k_att7_dec<16>, grid, block, 0, st, a); break;
        default: return false;
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
