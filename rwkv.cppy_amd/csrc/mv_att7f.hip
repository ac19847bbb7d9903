// mv_att7f.hip -- v7 decode: the LoRA second stages (w, a, g, v) and the per-head attention core
// (rwkv_graph.inc:416-470, rwkv_operators_wkv_v7.inc:37-107) in ONE launch per layer.
//
// Before: the LoRA second stages were their own matvec launch (four F16 matrices C x D, D = 64..480,
// k_mva over C rows each with their epilogues -- decay, sigmoid + bias, identity, v mix) and
// k_att7_dec read w, a, g, v back from global memory.  Head h only needs its own 64 channels of
// them, so here workgroup h computes those 4 x 64 rows itself (one row per lane group of a wave:
// k_mva's lane/unit order, wave_sum63 tree and epilogue arithmetic, so the values are
// bit-identical) from the four LoRA first-stage vectors (fp32, converted to the weights' input
// format in registers exactly as the matvec prologue converts them), keeps them in LDS and runs k_att7_dec's
// prep, wkv7 and GroupNorm on them.  No hand-off: the LoRA inputs are complete at the launch
// boundary.  One launch and one boundary less per layer; the w/a/g/v round trip through HBM is gone.
#include "mv_common.hpp"

namespace rwkvmi {

// R rows of one matrix by one wave in k_mva's lane/unit order: the weight units first (issued at
// kernel start, before the inputs exist), then the dots and wave_sum63's tree; lane r returns row
// r's sum (wave_sum63(acc) + 0.0f, the non-_1 formats' form)
template <int WF, int R, int U>
__device__ __forceinline__ void a7_load(const DMat & W, int row0, int lane, WBlk (&w)[R][U]) {
    const int M = W.M;
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int r = 0; r < R; r++) w[r][u] = load_unit<WF>(W, min(row0 + r, M - 1), u, lane);
}

// The input unit of lane l in the weights' input format, converted in registers from the fp32
// LoRA first-stage vector exactly as the matvec prologue converts it into LDS (chunk_store: fp16
// halves by to_half, or fp32 as is) and read back (load_act_unit: units clamped to K - EL)
template <int WF, int U>
__device__ __forceinline__ void a7_input(const float * x, int K, int lane, AUnit (&xu)[U]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
        if constexpr (WF == W_F16) {
            const int k = min(lane * 8 + u * 512, K - 8);
            const float4 t0 = *(const float4 *)(x + k), t1 = *(const float4 *)(x + k + 4);
            const float v[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
            int p[4];
#pragma unroll
            for (int j = 0; j < 4; j++)
                p[j] = __builtin_bit_cast(int, __halves2half2(to_half(v[2 * j]), to_half(v[2 * j + 1])));
            xu[u].lo = make_int4(p[0], p[1], p[2], p[3]);
        } else {
            const int k = min(lane * 4 + u * 256, K - 4);
            const float4 t = *(const float4 *)(x + k);
            xu[u].lo = make_int4(__float_as_int(t.x), __float_as_int(t.y), __float_as_int(t.z), __float_as_int(t.w));
        }
    }
}

template <int WF, int R, int U>
__device__ __forceinline__ float a7_dots(const WBlk (&w)[R][U], int K, const AUnit (&xu)[U], int lane) {
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
        }
    }
    float sr[R];
#pragma unroll
    for (int r = 0; r < R; r++) sr[r] = wave_sum63(acc[r]) + 0.0f;
    return lane_row_sum<R>(sr, lane);
}

constexpr int A7_LMAX = 512;  // LoRA width held in LDS per input (F16: one unit per lane)

template <int WF, int U>
__global__ __launch_bounds__(1024) void k_att7_lora(Att7Lora a) {
    constexpr int S = 64, G = 16, JPG = 4;
    __shared__ float sr[64], sw[64], sk[64], sv[64], snb[64], sbb[64], sy[64], sa[64], sg[64];
    __shared__ float sbonus;
    const Att7Dec & at = a.att;
    const int h = blockIdx.x, tid = threadIdx.x, c0 = h * S;
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // this wave's LoRA rows: matrix wave / 4 (w, a, g, v), rows c0 + 16 (wave & 3) .. + 15; their
    // weight units are the kernel's first loads
    const int lm = wave >> 2, lrow0 = c0 + 16 * (wave & 3);
    const bool lon = lm < 3 || a.has_v;
    const DMat LW = lm == 0 ? a.W2[0] : lm == 1 ? a.W2[1] : lm == 2 ? a.W2[2] : a.W2[3];
    WBlk lw[16][U];
    AUnit lx[U];
    if (lon) {
        a7_load<WF, 16, U>(LW, lrow0, lane, lw);
        a7_input<WF, U>(lm == 0 ? a.lin[0] : lm == 1 ? a.lin[1] : lm == 2 ? a.lin[2] : a.lin[3], LW.K, lane, lx);
    }
    // per-channel operands and the state rows first (they stream in under the LoRA rows)
    const int wi = tid / G, wg = tid % G;
    const size_t wbase = (size_t)h * S * S + (size_t)wi * S + wg * JPG;
    const int cme = c0 + (tid & (S - 1));
    const float lnw_c = at.lnx_w[cme], lnb_c = at.lnx_b[cme];
    const float k_c = at.k[cme], kk_c = at.k_k[cme], ka_c = at.k_a[cme];
    const float r_c = at.r[cme], rk_c = at.r_k[cme];
    float st[JPG];
#pragma unroll
    for (int jj = 0; jj < JPG; jj++) st[jj] = at.sin[wbase + jj];
    // LoRA second stages: wave w -> matrix w / 4 (w, a, g, v), rows c0 + 16 (w & 3) .. + 15
    {
        const int m = lm, row0 = lrow0;
        if (lon) {
            const int c = row0 + min(lane, 15);
            EpiIn ep;
            ep.y = m == 3 ? at.v[c] : 0.0f;
            ep.aux = m == 3 ? a.vfirst[c] : 0.0f;
            ep.bias = a.bias[m] ? a.bias[m][c] : 0.0f;
            const float s = a7_dots<WF, 16, U>(lw, LW.K, lx, lane);
            const int epi = m == 0 ? EPI_DECAY7 : m == 1 ? EPI_SIGMOID_BIAS : m == 2 ? EPI_STORE : EPI_VMIX7;
            const float o = epi_apply(epi, s, ep);
            if (lane < 16) {
                float * dst = m == 0 ? sw : m == 1 ? sa : m == 2 ? sg : sv;
                dst[c - c0] = o;
            }
        } else if (m == 3 && lane < 16) {
            sv[row0 - c0 + lane] = at.v[row0 + lane];  // layer 0: no v mix
        }
    }
    __syncthreads();
    // k_att7_dec from here, with w, a, g, v from LDS
    float w_c = 0.0f, a_c = 0.0f, v_c = 0.0f, g_c = 0.0f;
    if (tid < S) {
        w_c = sw[tid];
        a_c = sa[tid];
        v_c = sv[tid];
        g_c = sg[tid];
    }
    __syncthreads();
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
    {
        // wkv7 (rwkv_operators_wkv_v7.inc:37-107): state [h][i(value)][j(key)], g splits j
        const int i = wi, g = wg;
        float sa_ = 0.0f;
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) sa_ += snb[g * JPG + jj] * st[jj];
        sa_ = group_sum(sa_, G);
        const float vi = sv[i];
        float acc = 0.0f;
#pragma unroll
        for (int jj = 0; jj < JPG; jj++) {
            const int j = g * JPG + jj;
            const float kv = vi * sk[j];
            const float ns = st[jj] * sw[j] + kv + sa_ * sbb[j];
            at.sout[wbase + jj] = ns;
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
        if (at.yq.fmt >= 0) emit32(at.yq, 0, c, o);
        else at.y[c] = o;
    }
}

bool att7_lora_supported(const Att7Lora & a) {
    if (a.att.S != 64 || a.att.nb > 1 || a.att.yq.fmt < 0) return false;
    const int t = a.W2[0].type;
    if (t != W_F16 && t != W_F32) return false;
    const int C = a.att.H * 64;
    for (int m = 0; m < 4; m++) {
        if (m == 3 && !a.has_v) continue;
        // one weight unit per lane: F16 K <= 512, F32 K <= 256 (the 16-row register tile)
        const int kmax = t == W_F16 ? A7_LMAX : A7_LMAX / 2;
        if (a.W2[m].type != t || a.W2[m].M != C || a.W2[m].K <= 0 || a.W2[m].K % 8 || a.W2[m].K > kmax) return false;
        if (!a.lin[m]) return false;
    }
    if (a.has_v && !a.vfirst) return false;
    return true;
}

bool launch_att7_lora(hipStream_t st, const Att7Lora & a) {
    if (!att7_lora_supported(a)) {
        fprintf(stderr, "rwkv: fused v7 LoRA + attention decode: unsupported shape\n");
        return false;
    }
    const dim3 grid(a.att.H), block(1024);
    if (a.W2[0].type == W_F16) RK_LAUNCH((k_att7_lora<W_F16, 1>), grid, block, 0, st, a);
    else RK_LAUNCH((k_att7_lora<W_F32, 1>), grid, block, 0, st, a);
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
