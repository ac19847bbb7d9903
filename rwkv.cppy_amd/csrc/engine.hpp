// engine.hpp -- device-resident RWKV model and the per-version forward programs.
#pragma once

#include <string>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"
#include "model_file.hpp"

namespace rwkvmi {

struct DLayer {
    float *ln1_w = nullptr, *ln1_b = nullptr, *ln2_w = nullptr, *ln2_b = nullptr;
    // v4 / v5
    float *att_mix_k = nullptr, *att_mix_v = nullptr, *att_mix_r = nullptr, *att_mix_g = nullptr;
    float *att_first = nullptr, *att_decay = nullptr;  // v4 (per channel)
    float *att_u = nullptr, *att_w = nullptr;          // v5/v6 wkv6 u (faaaa/first) and v5 w, expanded to [C]
    float *att_lnx_w = nullptr, *att_lnx_b = nullptr;
    // v6
    float *maa_x = nullptr, *maa[5] = {nullptr, nullptr, nullptr, nullptr, nullptr}, *maa_w2 = nullptr;
    float *maa_w2t = nullptr;  // time_maa_w2 transposed to [5][D][C] (coalesced per-channel dots)
    float *decay6 = nullptr;
    // v7
    float *x_rwkvag = nullptr, *w0 = nullptr, *a0 = nullptr, *v0 = nullptr, *k_k = nullptr, *k_a = nullptr, *r_k = nullptr;
    // ffn
    float *ffn_mix_k = nullptr, *ffn_mix_r = nullptr, *ffn_maa_k = nullptr, *ffn_maa_r = nullptr, *ffn_x_k = nullptr;
    DMat att_r{}, att_k{}, att_v{}, att_o{}, att_g{}, maa_w1{}, decay_w1{}, decay_w2{};
    DMat w1{}, w2{}, a1{}, a2{}, g1{}, g2{}, v1{}, v2{};
    DMat ffn_k{}, ffn_v{}, ffn_r{};
};

struct DeviceModel {
    int refcount = 0;
    int device = 0;
    uint32_t layer_lo = 0, layer_hi = 0;  // layers whose weights are resident: [layer_lo, layer_hi)
    bool partial() const { return layer_lo != 0 || layer_hi != n_layer; }
    uint32_t n_vocab = 0, n_embed = 0, n_layer = 0;
    int major = 4, minor = 0;
    int64_t H = 0, S = 0;
    int F = 0;          // FFN width
    int maa_D = 0;      // v6 maa LoRA width (per mix)
    int kmax = 0;       // largest matmul K
    size_t state_len = 0;
    DMat emb{}, head{};
    float *ln0_w = nullptr, *ln0_b = nullptr, *lnout_w = nullptr, *lnout_b = nullptr;
    std::vector<DLayer> layers;
    std::vector<void *> allocs;
    double layer_weight_bytes = 0;   // algorithmic bytes of all layer matrices (original block sizes)
    double head_weight_bytes = 0;
    double layer_flops = 0, head_flops = 0;  // 2*M*K per token
    double small_param_bytes = 0;    // fp32 vectors read per token
};

bool upload_model(const ModelFile & mf, DeviceModel & dm, uint32_t layer_begin = 0, uint32_t layer_end = UINT32_MAX);
// repacks one ggml-order matrix into the device layout (allocations recorded in dm.allocs)
bool upload_mat(DeviceModel & dm, const HostTensor * t, DMat & out, bool count_bytes, bool is_head);
void free_model(DeviceModel & dm);

struct ActSlot {
    int8_t * q = nullptr;
    float * d = nullptr;
    float * s = nullptr;
    int * qsum = nullptr;
    __half * h = nullptr;
    float * f = nullptr;
    uint8_t * tq = nullptr;  // sequence-GEMM token-tile records
};

// Per-kernel-class timing collected with hipEvents on the context stream (bench roofline).
struct KernelStat {
    std::string name;
    long long launches = 0;
    double total_ms = 0;
    double total_bytes = 0;   // algorithmic bytes (weights at original block size + activations)
    double total_flops = 0;
};

class Engine : public KLaunchTimer {
  public:
    explicit Engine(DeviceModel * m) : m_(m) {}
    ~Engine();
    bool begin(hipEvent_t * a, hipEvent_t * b) override;
    void end(const char * kernel) override;

    bool init();
    // ABI-level evaluation (host buffers).  tokens host, T >= 1.
    bool eval_once(const uint32_t * tokens, size_t T, const float * state_in, float * state_out, float * logits_out);
    bool eval(const uint32_t * tokens, size_t T, const float * state_in, float * state_out, float * logits_out);
    // device-resident evaluation on the context's own state
    bool eval_device(const uint32_t * tokens, size_t T, bool want_logits, float * logits_out, bool sync);
    bool eval_layers(const uint32_t * tokens, size_t T, uint32_t l0, uint32_t l1, float * x_io, float * vfirst_io,
                     bool want_logits, float * logits_out, bool sync = true);
    // batched decode: B contexts, one token each; states [B][state_len] (host or device, see dev)
    bool eval_batch(const uint32_t * tokens, size_t B, const float * state_in, float * state_out, float * logits_out,
                    bool dev);
    static constexpr int kBatchMax = 256;
    float * device_logits() const { return logits_; }
    bool state_upload(const float * state);
    bool state_download(float * state);
    // the state of layers [l0, l1) only (a pipeline stage's or replica's slice); slice = those
    // layers in the host layout, NULL on upload = fresh state for them
    size_t layer_state_len() const { return m_->major >= 5 ? (size_t)m_->n_embed * (2 + (size_t)m_->S) : 5 * (size_t)m_->n_embed; }
    bool state_upload_layers(const float * slice, uint32_t l0, uint32_t l1);
    bool state_download_layers(float * slice, uint32_t l0, uint32_t l1);
    // state bytes moved host->device / device->host by this context (state APIs and rwkv_eval)
    double io_bytes_h2d() const { return io_h2d_; }
    double io_bytes_d2h() const { return io_d2h_; }
    bool sync();
    hipStream_t stream() const { return stream_; }
    void set_timing(bool on);
    bool mm_launch(MMGroup & g, int wtype);
    const std::vector<KernelStat> & stats();
    float * device_state() const { return dstate_[cur_]; }
    // debugging aid (rwkv_mi355x_debug_buffer): copies a workspace buffer of the last evaluation
    long long debug_copy(const char * name, void * out, size_t bytes);
    // test hooks (rwkv_mi355x_debug_set): "skip_granule" = producer workgroup of k_v6_att_fused that
    // publishes nothing (-1 off), "spin_max" = the hand-off sweep bound; returns false for unknown names
    bool debug_set(const char * name, long long value);
    // false when an in-launch hand-off of the work completed so far timed out: reports it, clears the
    // granules and the flag (the caller fails the evaluation with RWKV_ERROR_CTX)
    bool handoff_check();

  private:
    bool ensure_workspace(int T);
    bool init_state(float * st, size_t n = 0);
    bool forward(int T, const float * sin, float * sout, bool logits);
    bool forward_range(int T, const float * sin, float * sout, uint32_t l0, uint32_t l1, bool logits);
    bool forward_decode(const float * sin, float * sout, bool logits, uint32_t l0 = 0, uint32_t l1 = UINT32_MAX);
    bool mv(MVGroup & g, hipStream_t st = nullptr);
    bool run_tokens(const uint32_t * tokens, size_t T, bool want_logits);
    bool run_tokens_impl(const uint32_t * tokens, size_t T, bool want_logits);
    bool layer_v4(int l, int T, const float * si, float * so);
    bool wkv6(int T, int H, int S, const float * u, const float * w, int wpt, const float * sin, float * sout);
    bool layer_v5(int l, int T, const float * si, float * so);
    bool layer_v6(int l, int T, const float * si, float * so);
    bool layer_v7(int l, int T, const float * si, float * so);
    bool ffn(int l, int T, const float * si, float * so);
    ActBuf A(int slot, const DMat & W) const;
    ActBuf Aview(int slot, int K, int fmt) const;

    DeviceModel * m_;
    hipStream_t stream_ = nullptr;
    double io_h2d_ = 0, io_d2h_ = 0;
    int tcap_ = 0;
    std::vector<void *> ws_allocs_;
    float *x_ = nullptr, *xa_ = nullptr, *sx_ = nullptr, *r_ = nullptr, *k_ = nullptr, *v_ = nullptr, *g_ = nullptr;
    float *w_ = nullptr, *y_ = nullptr, *a_ = nullptr, *nb_ = nullptr, *bb_ = nullptr, *vfirst_ = nullptr;
    float *fr_ = nullptr, *lora_ = nullptr, *bonus_ = nullptr, *logits_ = nullptr;
    float *dsmall_[4] = {nullptr, nullptr, nullptr, nullptr};  // decode LoRA intermediates [kmax]
    uint32_t * dtokens_ = nullptr;
    uint32_t * htokens_ = nullptr;  // pinned
    static constexpr int kSlots = 12;
    ActSlot slots_[kSlots];
    float * dstate_[2] = {nullptr, nullptr};
    int cur_ = 0;
    unsigned * herr_h_ = nullptr;  // hand-off timeout flag, host-mapped (herr_d_ = its device address)
    unsigned * herr_d_ = nullptr;
    unsigned long long * hgran_ = nullptr;  // in-launch hand-off granules (k_v6_att_fused)
    // tagged granules (per layer and state parity, never cleared by their readers): ygran_ [C] head
    // outputs -> fused Wo rows; kgran_ [KG_STRIDE F / 32] FFN key blocks and rgran_ [C] receptance
    // rows -> fused FFN value rows.  One allocation of tgran_n_ granules, cleared as a whole.
    unsigned long long * ygran_ = nullptr;
    unsigned long long * kgran_ = nullptr;
    unsigned long long * rgran_ = nullptr;
    unsigned long long * xgran_ = nullptr;  // [C] v6 x rows -> the next layer's maa (k_sig_maa)
    size_t tgran_n_ = 0;
    size_t hgran_n_ = 0;
    int dbg_skip_gran_ = -1;
    unsigned spin_max_ = 1u << 20;
    // chunk-parallel wkv6 for sequences (wkv_chunk.hip; re-associated, not bit-exact): 0 = serial
    // k_wkv6_s64 (default); RWKV_MI355X_WKV_CHUNK=1 or rwkv_mi355x_debug_set(ctx, "wkv_chunk", 1)
    bool wkv_chunk_ = false;
    float * wkvc_ = nullptr;  // its chunk matrices / chunk states
    bool ensure_wkvc(size_t need);
    size_t wkvc_cap_ = 0;
    hipGraphExec_t graphs_[2][2][2] = {};  // [co-resident layout][cur][logits]
    bool use_graphs_ = true;
    bool split_maa_ = false;       // RWKV_MI355X_SPLIT_MAA=1: v6 decode W1 + mix as two launches
    // Decode fusions (RWKV_MI355X_DECODE_FUSION, a mask read at init; rwkv_mi355x_debug_set
    // "decode_fusion"): every fused launch has an unfused form of the same bits.
    enum : unsigned {
        FUSE_ATT6 = 1,   // k_v6_att_fused (r, k, v, g, decay-LoRA rows + per-head attention)
        FUSE_WO6 = 2,    // + Wo in that launch
        FUSE_ATT4 = 4,   // k_v4_att_fused (LN + r, k, v rows + WKV-4)
        FUSE_WO4 = 8,    // + Wo in that launch
        FUSE_ATT7 = 16,  // k_att7_lora (v7 LoRA second stages + attention)
        FUSE_SIG = 32,   // k_mvsig (FFN value + receptance rows)
        FUSE_FFN = 64,   // k_ffn_fused (the whole channel mix: key, receptance and value rows)
        FUSE_FFNCO = 128,  // its co-resident form, while the co-resident layouts are in use (co_mode)
        FUSE_SIGMAA = 256, // v6: the FFN value rows + the next layer's maa in one launch (co-resident only)
        FUSE_EMBMAA = 512, // the embedding LayerNorm inside layer 0's first launch (v6 maa, v4 attention)
        FUSE_ALL = 1023,
        // the one-launch channel mix measured slower than the key + value pair (same box, separate
        // processes: v6-1B6 716 vs 692 us/token, v4-169M 234 vs 228): off by default
        // (FUSE_FFNCO is added at creation for RWKV-4 only: v4-169M 222.5-223.0 vs 230.5-230.9 us/token,
        // v6-1B6 697.8-699.7 vs 655.9-659.2 -- profiles/r6_ab_ffco_v4.txt, r6_ab_ffco_v6.txt)
        FUSE_DEFAULT = FUSE_ALL & ~FUSE_FFN & ~FUSE_FFNCO,
    };
    unsigned fuse_ = FUSE_DEFAULT;
    // v6 attention launch layout (mv_att6c.hip vs mv_att6f.hip, the same bits).  The co-resident
    // layout needs all its workgroups resident at once: it is used only while this context is the
    // process's only one with work queued on the device (claim_device / the per-device count) and
    // until a hand-off timeout (another process's launches holding the compute units) turns it off
    // for the context.  co_knob_ ("co_mode"): -1 that rule, 0 never, 1 always (tests, A/B).
    int co_knob_ = -1;
    bool co_ok_ = true;       // cleared for good by a hand-off timeout in the co-resident layout
    bool co_ = false;         // the layout the launches being enqueued / captured use
    bool claimed_ = false;    // this context holds one count on its device (released at a sync)
    bool co_retry_ = false;   // the last failed check saw co-resident layout launches
    int co_pending_ = 0;      // co-resident layout decodes enqueued since the last check
    void claim_device();
    void release_device();
    bool choose_co();         // claim the device, pick the layout for the next decode launches
    int wo_rows_ = 8;      // k_v6_att_fused: Wo rows per wave of a Wo workgroup (debug knob "wo_rows": 4 / 8)
    int ffn_wdelay_ = -1;  // k_ffn_fused: consumer weight-issue delay in 100 MHz ticks ("ffn_wdelay"; -1:
                           // the producers' weight bytes at 4 TB/s, so the two streams do not overlap)
    int ffn_prepoll_ = 1;  // k_ffn_fused: poll the key blocks' d granules before the gather ("ffn_prepoll")
    int wo_prepoll_ = 1;   // k_v6_att_fused: one wave polls a granule per head before the gather ("wo_prepoll"; 0: 707.5 -> 708.9 us/token)
    bool generic_decode_ = false;  // RWKV_MI355X_GENERIC_DECODE=1: decode through the T>1 kernels
    hipEvent_t tok_event_ = nullptr;
    bool v7_fused_lora_ = false;  // the decode program runs k_att7_lora (w/a/g/v buffers not written)
    bool last_decode_ = false;    // the last step ran the decode program (debug_copy)
    bool timing_ = false;
    struct Pending {
        int stat;
        hipEvent_t a, b;
        double bytes, flops;
    };

    int add_stat(const std::string & name);
    double kt_bytes_ = 0, kt_flops_ = 0;  // algorithmic work of the next timed launch
    hipEvent_t kt_a_ = nullptr, kt_b_ = nullptr;
    bool mm_dispatch(MMGroup & g, int wtype);
    bool ensure_part(size_t n);
    float * gy_ = nullptr;     // scratch y of emit-only GEMM entries
    size_t gy_cap_ = 0;
    float * part_ = nullptr;   // split-K partials (launch_qgemm, k_fmm)
    size_t part_cap_ = 0;
    float * m2_ = nullptr;     // _1 formats: m*s chain totals (launch_qgemm, k_qg_msum)
    size_t m2_cap_ = 0;
    bool use_mm_ = false;
    bool tile_acts_ = false;  // Aview: Q8 activations in sequence-GEMM tiles (forward, T >= 2)
    // batched decode (eval_batch): state floats per context while a batched forward is built
    // (0 otherwise), the head's output rows, and the engine-owned staging buffers / graphs
    size_t bs_ = 0;
    int batch_gemm_min_ = 16;
    float * head_out_ = nullptr;
    float * bstate_[2] = {nullptr, nullptr};
    float * blogits_ = nullptr;
    size_t bcap_ = 0;
    struct BatchGraph {
        size_t B;
        const float * sin;
        float * sout;
        float * lout;
        hipGraphExec_t ge;
    };
    std::vector<BatchGraph> bgraphs_;
    void drop_batch_graphs();
    // rwkv_eval with host state buffers: the decode as io_chunk_-layer graphs with the state
    // copies of other chunks overlapped (eval_host_chunked)
    bool io_pipeline_ = true;
    int io_chunk_ = 4;
    hipStream_t io_stream_[2] = {nullptr, nullptr};
    std::vector<hipEvent_t> io_ev_;
    hipEvent_t io_entry_ev_ = nullptr;  // work already queued on stream_ at entry (copy streams wait)
    std::vector<hipGraphExec_t> io_graphs_[2][2][2];  // [co-resident layout][cur][logits] per chunk
    bool eval_host_chunked(uint32_t token, const float * state_in, float * state_out, float * logits_out);
    bool pinned_io(const float * state_in, const float * state_out);
    void drop_io_graphs();
    void drop_graphs();
    std::vector<Pending> pending_;
    std::vector<hipEvent_t> event_pool_;
    std::vector<KernelStat> stats_;
    void collect_timing();
};

}  // namespace rwkvmi
