// kernels.hpp -- host launchers for the gfx950 kernels (kernels.hip).
#pragma once

#include "common.hpp"

namespace rwkvmi {

// ---- matmul (dequant-matvec / batched) --------------------------------------------------
// Launches one grouped matmul: every entry shares the weight type `wtype`.
bool launch_mm_group(hipStream_t st, MMGroup & g, int wtype);
// int8-MFMA sequence GEMM for quantized weights (qgemm.hip); same results as launch_mm_group.
// Every entry needs y; emission is left to the caller (launch_act_from_f32).
bool launch_qgemm(hipStream_t st, MMGroup & g, int wtype);
// F16 / F32 weights over T >= 16 tokens on the f32 MFMA (mv_fmfma.hip); *launched = false: not covered
bool launch_fmm_group(hipStream_t st, MMGroup & g, int wtype, bool * launched);
bool launch_qg_combine(hipStream_t st, MMGroup & g, int split);
extern int kQgCUs;
// Batched decode matvec (mv_batch.hip): the T rows are T independent contexts; same results as
// launch_mm_group.  *launched = false (and nothing enqueued) for shapes it does not cover.
bool launch_mvb_group(hipStream_t st, MMGroup & g, int wtype, bool * launched);

// ---- elementwise / recurrence kernels -----------------------------------------------------
// x[t] = LN(emb[tokens[t]]; w, b)   (rwkv_graph.inc:654-658)
bool launch_embed_ln(hipStream_t st, const uint32_t * tokens, int T, const DMat & emb,
                     const float * w, const float * b, float * x);

struct LnMixArgs {
    int T, C;
    const float * x;            // [T][C] residual stream
    const float * carry_in;     // [C] previous token's LN output (state *_xx)
    float * carry_out;          // [C] <- LN(x[T-1])
    const float * lnw, * lnb;
    int form;                   // 0: xa*mu + (xp - xp*mu)  (v4/v5)   1: (xp - xa)*mu + xa (v6/v7)
    int n_out;
    const float * mu[6];
    ActBuf out[6];
    float * out_xa;             // optional fp32 [T][C]
    float * out_sx;             // optional fp32 [T][C] (xp - xa)
    size_t bs;                  // 0: one sequence; > 0: batched decode -- token t is context t, its
                                // carries at carry_in/out + t * bs (state floats per context)
};
bool launch_ln_mix(hipStream_t st, const LnMixArgs & a);

// v6: xs[n] = (W2[n] . lora_n + maa[n]) * sx + xa, n = w,k,v,r,g   (rwkv_graph.inc:313-346)
bool launch_v6_mix5(hipStream_t st, int T, int C, int D, const float * lora, const float * w2,
                    const float * const * maa, const float * xa, const float * sx, const ActBuf * outs);

// v4 wkv with aa/bb/pp state (rwkv_graph.inc:119-161); emits r*wkv into `out`.
bool launch_wkv4(hipStream_t st, int T, int C, const float * r, const float * k, const float * v,
                 const float * first, const float * decay, const float * state_in, float * state_out,
                 const ActBuf & out, int bs = 0);

// ggml_rwkv_wkv6 semantics (v5/v6): y[T][C]; w_per_token selects v6 (w [T][C]) vs v5 (w [C]).
// bs > 0 (every wkv launcher): batched decode -- the T tokens are T contexts, one token each,
// context t's state at state_in/out + t * bs.
bool launch_wkv6(hipStream_t st, int T, int H, int S, const float * k, const float * v, const float * r,
                 const float * u, const float * w, int w_per_token, const float * state_in,
                 float * state_out, float * y, int bs = 0);

// Chunk-parallel wkv6 (wkv_chunk.hip, head size 64, T >= 2, no batch): the same recurrence with the
// sums re-associated (not bit-exact with launch_wkv6).  RA / KB: [T][C] scratch; scratch:
// wkv6_chunked_scratch_floats(T, H) floats.
bool wkv6_chunked_supported(int T, int S, int bs);
size_t wkv6_chunked_scratch_floats(int T, int H);
bool launch_wkv6_chunked(hipStream_t st, int T, int H, const float * k, const float * v, const float * r,
                         const float * u, const float * w, int w_per_token, const float * state_in, float * state_out,
                         float * y, float * RA, float * KB, float * scratch);

// Chunk-parallel WKV-7 (wkv7_chunk.hip, head size 64, T >= 2, no batch): the same recurrence with the
// sums re-associated (not bit-exact with launch_wkv7); scratch: wkv7_chunked_scratch_floats(T, H).
bool wkv7_chunked_supported(int T, int S, int bs);
size_t wkv7_chunked_scratch_floats(int T, int H);
bool launch_wkv7_chunked(hipStream_t st, int T, int H, const float * r, const float * w, const float * k,
                         const float * v, const float * a, const float * b, const float * state_in, float * state_out,
                         float * y, float * scratch);

// v7 per-head prep: kk = l2norm(k*k_k); k += a*ka - ka; nb = -kk; bb = kk*a; bonus = sum(k*r*r_k)
bool launch_v7_prep(hipStream_t st, int T, int H, int S, float * k, const float * a, const float * r,
                    const float * k_k, const float * k_a, const float * r_k, float * nb, float * bb,
                    float * bonus);

// rwkv_operators_wkv_v7.inc:37-107
bool launch_wkv7(hipStream_t st, int T, int H, int S, const float * r, const float * w, const float * k,
                 const float * v, const float * a, const float * b, const float * state_in,
                 float * state_out, float * y, int bs = 0);

// GroupNorm over heads + ln_x (+ v7 bonus) (+ gate), emitted as the output projection's input.
// mode 0: none, 1: *g, 2: + v*bonus then *g
bool launch_groupnorm(hipStream_t st, int T, int H, int S, float eps, const float * y, const float * w,
                      const float * b, int mode, const float * g, const float * v, const float * bonus,
                      const ActBuf & out);

// LN of rows x[0..rows) emitted into rows 0..rows of an ActBuf (head input).
bool launch_ln_emit(hipStream_t st, int C, const float * x, const float * w, const float * b, const ActBuf & out,
                    int rows = 1);

// v4 state init value helper: fills n floats with value
bool launch_fill(hipStream_t st, float * p, size_t n, float value);

}  // namespace rwkvmi

namespace rwkvmi {
// x [T][K] fp32 -> activation buffer (emit32 path); used by the self-test entry points.
bool launch_act_from_f32(hipStream_t st, const float * x, int T, int K, const ActBuf & out);
}  // namespace rwkvmi

// ---------------------------------------------------------------------------------------
// Decode (T == 1) kernels: kernels_decode.hip
namespace rwkvmi {

enum MVSrc : int {
    SRC_ACT = 0,    // pre-quantized activation row in global memory (ActBuf, row 0)
    SRC_F32 = 1,    // fp32 vector in global memory; each workgroup quantizes it into LDS
    SRC_LNMIX = 2,  // LN(x) + token shift + mix, computed and quantized into LDS per workgroup
};

struct MVEntry {
    DMat W;
    int src;
    ActBuf act;              // SRC_ACT
    const float * f;         // SRC_F32 [K]
    const float * x;         // SRC_LNMIX residual stream [K]
    const float * carry;     // previous token's LN output (state *_xx)
    const float * lnw, * lnb, * mu;
    int form;                // 0: xa*mu + (xp - xp*mu)   1: (xp - xa)*mu + xa   2: xa (plain LN)
    float * carry_out;       // entry's first workgroup writes xa here (new *_xx state)
    const float * mu2;       // SRC_LNMIX: the entry's first workgroup also emits the mix with mu2
    ActBuf act2_out;         // (same LayerNorm and token shift) into act2_out (row 0, global)
    float * y;               // fp32 [M] (may be null when emitting)
    const float * aux;
    const float * bias;
    int epi;
    int emit;                // emit the post-epilogue values into act_out (needs M % 32 == 0)
    ActBuf act_out;
    int block0;
};

// The scalars k_mva reads, copied out of the entry by launch_mv_group into one contiguous
// record so the kernel fetches them as a few back-to-back wide scalar loads (one round trip).
struct MVHot {
    const uint8_t * qs;
    const uint32_t * qh;
    const void * sc;
    const int8_t * aq;
    const float * ad;
    const float * as;
    const int * aqsum;
    const void * ahf;       // A_F16 halves or A_F32 floats
    float * y;
    const float * aux;      // g_mv_zero-free: null -> step 0 over a zero word (set by the kernel)
    const float * bias;
    int M, K, epi, steps;   // steps: bit0 aux present, bit1 bias present
};

struct MVGroup {
    MVHot hot[MM_MAX_ENTRIES];
    MVEntry e[MM_MAX_ENTRIES];
    int n;
    int lds_bytes;
    int stride;              // set by launch_mv_group: >0 = workgroups walk row blocks
    int grid;                // set by launch_mv_group: workgroups launched
    int units_max;           // set by launch_mv_group: max 16-byte units per lane over entries
    int rows;                // set by launch_mv_group: rows per wave of the launched shape
    int late;                // set by launch_mv_group: weights issued after the image inputs land
};

// Prologue matvecs: RWKV_MI355X_LATE_W=1 makes the streaming waves issue their weights only after
// the image waves' inputs have landed (default 0: measured slower in the split form).
int mv_late_weights();

// Busy-waits about `us` microseconds on the device (kernel timing: lets the host queue a whole
// decode step before the GPU starts it, so event pairs time kernels, not host submission).
bool launch_delay(hipStream_t st, int us);

void set_mv_device_cus(int n);

bool launch_mv_group(hipStream_t st, MVGroup & g);
int mva_rows();

// Decode channel mix (v4/v5/v6): y[row] += sigmoid(Wr[row] . xr) * (Wv[row] . k) in one launch
// (mv_sig.hip, k_mvsig): ev = the value matvec (SRC_ACT, y = the residual stream), er = the
// receptance matvec (SRC_ACT, same rows).  Same bits as the receptance matvec + EPI_SIGMUL_ADD.
bool mv_sigmul_supported(const MVEntry & ev, const MVEntry & er);
bool launch_mv_sigmul(hipStream_t st, const MVEntry & ev, const MVEntry & er);
// The MVHot record of an SRC_ACT entry (the scalars k_mvsig reads)
void mv_fill_hot(const MVEntry & e, MVHot & h);

// v6 token-shift mixes with the maa LoRA (rwkv_graph.inc:308-346); xa = LN(x) is the new
// att_xx carry already written by the W1 matvec prologue; w2t is time_maa_w2 transposed to
// [5][D][C]; emits the five mixed vectors w,k,v,r,g.
// Batched decode: nb > 1 contexts (grid.z), xa / sx [nb][C] (sx = xp - xa), lora [nb][5D].
bool launch_v6_mix5_dec(hipStream_t st, int C, int D, const float * xa, const float * carry, const float * lora,
                        const float * w2t, const float * const * maa, const ActBuf * outs, int nb = 1,
                        const float * sx = nullptr);

// v6 maa LoRA in one launch (mv_maa.hip): LN(x) + token shift -> lora_n = tanh(W1[n] . xxx) ->
// the five mixed vectors w,k,v,r,g, emitted in their matmuls' input formats; writes the new
// att_xx carry.  Bit-identical to the W1 k_mv + launch_v6_mix5_dec pair it replaces.
struct MaaDec {
    int C, D;
    DMat w1;                    // time_maa_w1 (M = 5*D, K = C)
    const float * x;            // residual stream [C]
    const float * carry;        // previous att_xx [C]
    float * carry_out;          // new att_xx [C] (= LN(x)), written by workgroup (0, 0)
    const float * lnw, * lnb;
    const float * maa_x;        // time_maa_x [C]
    const float * w2t;          // time_maa_w2 transposed [5][D][C]
    const float * maa[5];       // time_maa_{w,k,v,r,g} [C]
    ActBuf out[5];
    int xa_off;                 // LDS byte offset of the fp32 xa image
    // layer 0 of a decode (k_v6_maa_dec4 only): x = LN0(emb[*tok]) computed in the launch (k_embed_ln's
    // arithmetic) instead of read from x; workgroup (0, 0) stores it to xout
    const uint32_t * tok;
    DMat emb;
    const float * ln0w, * ln0b;
    float * xout;
};
bool v6_maa_dec_supported(int C, int D, int w1_type);
void v6_maa_dec_args(MaaDec & a, int C, int D, const DMat & w1, const float * x, const float * carry, float * carry_out,
                     const float * lnw, const float * lnb, const float * maa_x, const float * w2t,
                     const float * const * maa, const ActBuf * outs);
bool v6_maa_emb_supported(const MaaDec & a);
bool launch_v6_maa_dec_emb(hipStream_t st, const MaaDec & a);
bool launch_v6_maa_dec(hipStream_t st, int C, int D, const DMat & w1, const float * x, const float * carry,
                       float * carry_out, const float * lnw, const float * lnb, const float * maa_x,
                       const float * w2t, const float * const * maa, const ActBuf * outs);
// v6 decode, co-resident form (mv_sigmaa.hip): layer l's k_mvsig rows (hv: Wv / k / y = x, hr: Wr /
// xr) and layer l + 1's maa workgroups (maa, x gathered from the granules xg the rows publish, tag
// xtag) in one launch of C / 8 workgroups; the same bits as k_mvsig + k_v6_maa_dec4.
struct SigMaa {
    MVHot hv, hr;
    int wtype;
    MaaDec maa;
    int nm;                      // maa workgroups: 5 C / 64
    unsigned long long * xg;     // C granules
    unsigned xtag;
    unsigned * err;
    unsigned spin_max;
};
bool sig_maa_supported(const SigMaa & a);
bool launch_sig_maa(hipStream_t st, const SigMaa & a);

// v5/v6 attention core for one token, one workgroup per head: (v6: decay LoRA second stage
// w = exp(-exp(Wd2 . dl + decay))) + wkv6 + GroupNorm*ln_x (+ *g).  Writes fp32 y [C].
struct Att6Dec {
    int H, S;
    const float * r, * k, * v, * g, * u;
    const float * w;         // v5: w [C]
    DMat wd2;                // v6: time_decay_w2 (M = C, K = D)
    const float * dl;        // v6: tanh(Wd1 . xw) [D]
    const float * decay;     // v6: time_decay [C]
    const float * sin;
    float * sout;
    const float * lnx_w, * lnx_b;
    float eps;
    float * y;
    ActBuf yq;               // fmt >= 0 (needs S >= 32): emit y in the Wo input format instead
    // batched decode (nb > 1 contexts, grid.y): context b's r/k/v/g/y at + b*C, dl at + b*ldd,
    // state at sin/sout + b*bs, yq row b
    int nb, ldd;
    size_t bs;
};
bool launch_att6_dec(hipStream_t st, const Att6Dec & a);

// v6 decode: the r, k, v, g and decay-LoRA first-stage matvecs plus the per-head attention core
// in one launch (mv_att6f.hip); bit-identical to the k_mva group + launch_att6_dec pair.
struct Att6Fused {
    int H, C, D;
    DMat W[4];       // att_r, att_k, att_v, att_g (M = K = C)
    ActBuf x[4];     // their inputs (the maa mixes xr, xk, xv, xg)
    DMat wd1;        // time_decay_w1 (M = D, K = C)
    ActBuf xw;       // its input
    Att6Dec att;     // wd2, decay, u, sin, sout, lnx_w, lnx_b, eps, yq
    unsigned long long * gran;  // 4 C + H D zeroed 8-byte granules: r, k, v, silu(g), tanh(Wd1 . xw)
    unsigned * err;  // set (system scope) on a hand-off timeout: a host-mapped word the engine reads
                     // after every synchronising call (Engine::handoff_check)
    unsigned spin_max;  // sweep bound (passes) before a timeout
    int skip_wg;     // test hook: this producer workgroup publishes nothing (-1: none)
    // Wo fused (wo.qs != null): the reducers publish the head outputs y as granules tagged ytag
    // (unique per layer and state parity, so they need no clearing) instead of emitting Wo's Q8
    // input; the non-reducer workgroups then gather y, quantize it (the matvec prologue's
    // arithmetic) and run Wo's rows with x += Wo . y (EPI_ADD) -- the Wo launch disappears
    DMat wo;
    float * xres;                 // the residual stream x [C]
    unsigned long long * ygran;   // C granules
    unsigned ytag;
    int wo_rows;                  // Wo rows per wave of a Wo workgroup: 4 or 8
    int wo_prepoll;               // 1: one wave polls a granule per head before the gather
};
bool v6_att_fused_supported(const Att6Fused & a);
bool launch_v6_att_fused(hipStream_t st, const Att6Fused & a);
// the same launch in the co-resident layout (mv_att6c.hip: 8 H workgroups that must all be
// resident at once; Wo fused, C % 512 == 0): the same bits, used by Engine::co_mode only
bool v6_att_co_supported(const Att6Fused & a);
bool launch_v6_att_co(hipStream_t st, const Att6Fused & a);
// v4 decode: LN + token shift, r / k / v rows and WKV-4 in one launch, 8 channels per workgroup
// (mv_att4f.hip); the two-launch k_mv + k_wkv4 pair gives the same bits.  Without wf, Wo's input
// is written as fp32 y (Wo quantizes it in its prologue).
bool v4_att_fused_supported(int C, const DMat & Wr, const DMat & Wk, const DMat & Wv, const ActBuf & out);
// wf: Wo in the same launch -- the producers publish their channels' outputs as granules tagged
// ytag (per layer and state parity); Wo workgroups after them in the grid gather all C, quantize
// them as Wo's fp32-input prologue does and run 2 Wo rows per wave, x += Wo . y
struct V4WoFused {
    DMat wo;
    float * xres;
    unsigned long long * ygran;
    unsigned ytag;
    unsigned * err;
    unsigned spin_max;
    // layer 0 of a decode: x = LN0(emb[*tok]) computed in the launch (k_embed_ln's arithmetic)
    const uint32_t * tok;
    DMat emb;
    const float * ln0w, * ln0b;
};
bool launch_v4_att_fused(hipStream_t st, int C, const DMat & Wr, const DMat & Wk, const DMat & Wv, const float * x,
                         const float * carry, float * carry_out, const float * lnw, const float * lnb,
                         const float * mix_r, const float * mix_k, const float * mix_v, const float * first,
                         const float * decay, const float * sin, float * sout, const ActBuf & out, float * y,
                         const V4WoFused * wf = nullptr);

// The decode channel mix in one launch (mv_ffnf.hpp): e[0] the FFN key (SRC_LNMIX, relu^2, emit = 1,
// act_out's format = the value's input format), e[1] the receptance (SRC_LNMIX, EPI_STORE; hasr
// only), wv the FFN value; x += sigmoid(r) * (Wv . relu^2(Wk . xk))  (v7: x += Wv . relu^2(...)).
// kg: KG_STRIDE * F / 32 granules, rg: C granules, both tagged `tag` (unique per layer and state
// parity; the engine clears them whenever the parity flips without a fused decode).
constexpr int KG_STRIDE = 10;  // granules per published Q8 block: 8 q dwords, d, s (Q8_1's d * sum)
struct FfnFused {
    MVEntry e[2];
    DMat wv;
    float * x;
    unsigned long long * kg;
    unsigned long long * rg;
    unsigned tag;
    unsigned * err;
    unsigned spin_max;
    int np;       // producer workgroups (set by launch_ffn_fused)
    int wdelay;   // consumers issue their value rows this many 100 MHz ticks after starting
    int prepoll;  // 1: one wave polls each key block's d granule before the gather
    int co;       // 1: the co-resident form (no consumer workgroups; Engine::co_mode only)
};
bool ffn_fused_supported(const FfnFused & f, int form, bool hasr);
bool launch_ffn_fused(hipStream_t st, FfnFused & f, int form, bool hasr);

// Sequence v6 decay LoRA tail (T >= 2): w[t][c] = exp(-exp(Wd2[c] . Q8(dl[t]) + decay[c])) with
// k_att6_dec's per-row arithmetic; dl fp32 [T][D].  Quantized Wd2 with D <= 512 only.
bool v6_decay_seq_supported(int wd2_type, int D);
bool launch_v6_decay_seq(hipStream_t st, int T, int C, const DMat & wd2, const float * dl, const float * decay,
                         float * w);

// v7 attention core for one token, one workgroup per head: kk/k/a prep, wkv7, GroupNorm,
// + v*sum(k*r*r_k), *g.  Writes fp32 y [C].
struct Att7Dec {
    int H, S;
    const float * r, * w, * k, * v, * a, * g;
    const float * k_k, * k_a, * r_k;
    const float * sin;
    float * sout;
    const float * lnx_w, * lnx_b;
    float * y;
    ActBuf yq;               // fmt >= 0 (needs S >= 32): emit y in the Wo input format instead
    int nb;                  // batched decode: contexts (grid.y), as Att6Dec
    size_t bs;
};
bool launch_att7_dec(hipStream_t st, const Att7Dec & a);

// v7 decode: the LoRA second stages (w, a, g, v: F16 / F32, K <= 512) and the per-head attention
// core in one launch (mv_att7f.hip); bit-identical to the LoRA-out matvec + k_att7_dec pair.
struct Att7Lora {
    Att7Dec att;            // r, k, v (pre-mix), k_k, k_a, r_k, state, ln_x, yq (w, a, g unused)
    DMat W2[4];             // time_w2, time_a2, time_g2, time_v2 (M = C, K = the LoRA widths)
    const float * lin[4];   // their inputs: the LoRA first-stage outputs (fp32 [K])
    const float * bias[4];  // w0, a0, none, v0
    const float * vfirst;   // layer 0's v (the v mix's aux)
    int has_v;              // layers > 0 mix v with v_first
};
bool att7_lora_supported(const Att7Lora & a);
bool launch_att7_lora(hipStream_t st, const Att7Lora & a);

}  // namespace rwkvmi
