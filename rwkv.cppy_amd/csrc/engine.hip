// engine.hip -- device model upload and the per-version forward programs.
//
// A token step is a fixed sequence of launches on the context's stream.  The T == 1 step
// is captured once into a hipGraph per (state parity, logits) and replayed, so decode pays
// no host launch cost.  Per-layer programs restate rwkv_graph.inc:
//   v4  :84-197 + FFN :484-511      v5  :199-292 + FFN :484-511
//   v6  :294-385 + FFN :513-531     v7  :387-482 + FFN :533-543
#include "engine.hpp"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <string>

#include "kernels.hpp"
#include "stamp.hpp"

namespace rwkvmi {

thread_local KLaunchTimer * g_klt = nullptr;

#ifdef RWKV_STAMP
// Diagnostic builds (stamp.hpp): every kernel translation unit registers a setter for its copy
// of the device-side control block; the rings are dumped to $RWKV_STAMP_OUT when an engine dies.
static std::vector<void (*)(const StampCtl &)> & stamp_setters() {
    static std::vector<void (*)(const StampCtl &)> v;
    return v;
}
int stamp_register(void (*f)(const StampCtl &)) {
    stamp_setters().push_back(f);
    return 0;
}
static StampCtl g_host_stamp = {nullptr, nullptr};
static void stamp_init() {
    if (g_host_stamp.buf) return;
    const size_t bytes = (size_t)kStampCUs * kStampRing * 64;
    if (hipMalloc(&g_host_stamp.buf, bytes) != hipSuccess || hipMalloc(&g_host_stamp.ctr, kStampCUs * 4) != hipSuccess)
        return;
    (void)hipMemset(g_host_stamp.buf, 0, bytes);
    (void)hipMemset(g_host_stamp.ctr, 0, kStampCUs * 4);
    for (auto f : stamp_setters()) f(g_host_stamp);
    (void)hipDeviceSynchronize();
}
static void stamp_dump() {
    const char * out = getenv("RWKV_STAMP_OUT");
    if (!out || !g_host_stamp.buf) return;
    const size_t bytes = (size_t)kStampCUs * kStampRing * 64;
    std::vector<unsigned long long> h(bytes / 8);
    if (hipMemcpy(h.data(), g_host_stamp.buf, bytes, hipMemcpyDeviceToHost) != hipSuccess) return;
    FILE * f = fopen(out, "wb");
    if (!f) return;
    // only the non-empty records: {t0, t1, t2, tag, x0..x3}
    for (size_t i = 0; i < h.size(); i += 8)
        if (h[i]) fwrite(&h[i], 8, 8, f);
    fclose(f);
}
#else
static void stamp_init() {}
static void stamp_dump() {}
#endif

// ------------------------------------------------------------------------- upload

template <typename T>
static T * dalloc(DeviceModel & dm, size_t n) {
    void * p = nullptr;
    if (hipMalloc(&p, n * sizeof(T) + 16) != hipSuccess) return nullptr;
    dm.allocs.push_back(p);
    return (T *)p;
}

static float * upload_vec(DeviceModel & dm, const HostTensor * t) {
    if (!t) return nullptr;
    const uint64_t n = t->nel();
    std::vector<float> v(n);
    if (t->type == W_F32) {
        memcpy(v.data(), t->data.data(), n * 4);
    } else if (t->type == W_F16) {
        for (uint64_t i = 0; i < n; i++) {
            uint16_t h;
            memcpy(&h, t->data.data() + 2 * i, 2);
            v[i] = f16_to_f32(h);
        }
    } else {
        fprintf(stderr, "rwkv: parameter %s must be FP32/FP16\n", t->name.c_str());
        return nullptr;
    }
    float * d = dalloc<float>(dm, n);
    if (!d || hipMemcpy(d, v.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    dm.small_param_bytes += (double)n * 4;
    return d;
}

static float * upload_host_floats(DeviceModel & dm, const std::vector<float> & v) {
    float * d = dalloc<float>(dm, v.size());
    if (!d || hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    dm.small_param_bytes += (double)v.size() * 4;
    return d;
}

// Repack one ggml-order matrix ne=[K, M] into the device layout of common.hpp.
bool upload_mat(DeviceModel & dm, const HostTensor * t, DMat & out, bool count_bytes, bool is_head) {
    if (!t) return true;
    if (t->ndim != 2) {
        fprintf(stderr, "rwkv: %s: matrix expected\n", t->name.c_str());
        return false;
    }
    out.type = (int)t->type;
    out.gt = nullptr;
    out.mt = nullptr;
    out.K = (int)t->ne[0];
    out.M = (int)t->ne[1];
    const size_t M = out.M, K = out.K;
    if (t->type == W_F32 || t->type == W_F16) {
        const size_t bytes = t->data.size();
        uint8_t * d = dalloc<uint8_t>(dm, bytes);
        if (!d || hipMemcpy(d, t->data.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return false;
        out.qs = d;
    } else {
        if (K % 32) {
            fprintf(stderr, "rwkv: %s: K=%zu not a multiple of 32\n", t->name.c_str(), K);
            return false;
        }
        const size_t nb = K / 32, nblk = M * nb, bb = type_block_bytes(t->type);
        const size_t qbytes = (t->type == W_Q8_0) ? 32 : 16;
        std::vector<uint8_t> qs(nblk * qbytes);
        std::vector<uint32_t> qh;
        std::vector<uint16_t> sc16;
        std::vector<uint32_t> sc32;
        const bool q5 = t->type == W_Q5_0 || t->type == W_Q5_1;
        const bool one = t->type == W_Q4_1 || t->type == W_Q5_1;
        if (q5) qh.resize(nblk);
        if (one) sc32.resize(nblk); else sc16.resize(nblk);
        const uint8_t * src = t->data.data();
        for (size_t i = 0; i < nblk; i++) {
            const uint8_t * b = src + i * bb;
            uint16_t d, mm;
            memcpy(&d, b, 2);
            switch (t->type) {
                case W_Q4_0: sc16[i] = d; memcpy(&qs[i * 16], b + 2, 16); break;
                case W_Q4_1: memcpy(&mm, b + 2, 2); sc32[i] = (uint32_t)d | ((uint32_t)mm << 16); memcpy(&qs[i * 16], b + 4, 16); break;
                case W_Q5_0: sc16[i] = d; memcpy(&qh[i], b + 2, 4); memcpy(&qs[i * 16], b + 6, 16); break;
                case W_Q5_1: memcpy(&mm, b + 2, 2); sc32[i] = (uint32_t)d | ((uint32_t)mm << 16); memcpy(&qh[i], b + 4, 4); memcpy(&qs[i * 16], b + 8, 16); break;
                case W_Q8_0: sc16[i] = d; memcpy(&qs[i * 32], b + 2, 32); break;
                default: return false;
            }
        }
        uint8_t * dq = dalloc<uint8_t>(dm, qs.size());
        if (!dq || hipMemcpy(dq, qs.data(), qs.size(), hipMemcpyHostToDevice) != hipSuccess) return false;
        out.qs = dq;
        if (q5) {
            uint32_t * dh = dalloc<uint32_t>(dm, qh.size());
            if (!dh || hipMemcpy(dh, qh.data(), qh.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
            out.qh = dh;
        }
        if (one) {
            uint32_t * ds = dalloc<uint32_t>(dm, sc32.size());
            if (!ds || hipMemcpy(ds, sc32.data(), sc32.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
            out.sc = ds;
        } else {
            uint16_t * ds = dalloc<uint16_t>(dm, sc16.size());
            if (!ds || hipMemcpy(ds, sc16.data(), sc16.size() * 2, hipMemcpyHostToDevice) != hipSuccess) return false;
            out.sc = ds;
        }
        // the same blocks again as sequence-GEMM tile records (common.hpp qg_*); the head only
        // ever runs on one token
        if (!is_head) {
            const int wt = (int)t->type, R = qg_rows(wt);
            const size_t tiles = (M + R - 1) / R, rb = qg_w_bytes(wt);
            std::vector<uint8_t> gt(tiles * nb * rb, 0);
            for (size_t rt = 0; rt < tiles; rt++)
                for (size_t b = 0; b < nb; b++) {
                    uint8_t * rec = &gt[(rt * nb + b) * rb];
                    for (int r = 0; r < R && rt * R + r < M; r++) {
                        const size_t i = (rt * R + r) * nb + b;
                        int8_t * w8 = (int8_t *)rec;
                        for (int j = 0; j < 32; j++) {
                            int v;
                            if (wt == W_Q8_0) {
                                v = (int8_t)qs[i * 32 + j];
                            } else {
                                const uint8_t byte = qs[i * 16 + (j & 15)];
                                v = j < 16 ? (byte & 0xF) : (byte >> 4);
                                if (q5) v |= (int)((qh[i] >> j) & 1u) << 4;
                                if (wt == W_Q4_0) v -= 8;
                                if (wt == W_Q5_0) v -= 16;
                            }
                            w8[qg_w_off(r, j)] = (int8_t)v;
                        }
                        const float d = f16_to_f32(one ? (uint16_t)(sc32[i] & 0xFFFFu) : sc16[i]);
                        memcpy(rec + qg_w_d(wt) + r * 4, &d, 4);
                    }
                }
            uint8_t * dg = dalloc<uint8_t>(dm, gt.size());
            if (!dg || hipMemcpy(dg, gt.data(), gt.size(), hipMemcpyHostToDevice) != hipSuccess) return false;
            out.gt = dg;
            if (one) {  // the mins, block-major, for the m*s chain kernel
                const size_t MS = qm_stride((int)M);  // rows padded to k_qg_msum's 8-row loads
                std::vector<float> mt(nb * MS, 0.0f);
                for (size_t r = 0; r < M; r++)
                    for (size_t b = 0; b < nb; b++) mt[b * MS + r] = f16_to_f32((uint16_t)(sc32[r * nb + b] >> 16));
                float * dmt = dalloc<float>(dm, mt.size());
                if (!dmt || hipMemcpy(dmt, mt.data(), mt.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
                out.mt = dmt;
            }
        }
    }
    if (count_bytes) {
        const double bytes = (double)type_nbytes(t->type, t->nel());
        const double flops = 2.0 * (double)M * (double)K;
        if (is_head) {
            dm.head_weight_bytes += bytes;
            dm.head_flops += flops;
        } else {
            dm.layer_weight_bytes += bytes;
            dm.layer_flops += flops;
        }
    }
    if (out.K > dm.kmax) dm.kmax = out.K;
    return true;
}

bool upload_model(const ModelFile & mf, DeviceModel & dm, uint32_t layer_begin, uint32_t layer_end) {
    dm.n_vocab = mf.header.n_vocab;
    dm.n_embed = mf.header.n_embed;
    dm.n_layer = mf.header.n_layer;
    dm.layer_lo = std::min(layer_begin, dm.n_layer);
    dm.layer_hi = std::min(layer_end, dm.n_layer);
    if (dm.layer_lo >= dm.layer_hi) {
        fprintf(stderr, "rwkv: empty layer range [%u, %u)\n", layer_begin, layer_end);
        return false;
    }
    const bool first = dm.layer_lo == 0, last = dm.layer_hi == dm.n_layer;
    dm.major = mf.arch_major;
    dm.minor = mf.arch_minor;
    dm.H = mf.head_count;
    dm.S = mf.head_size;
    const size_t C = dm.n_embed;
    dm.state_len = dm.major >= 5 ? C * (2 + (size_t)dm.S) * dm.n_layer : C * 5 * dm.n_layer;
    if (C % 64) {
        fprintf(stderr, "rwkv: n_embed %zu must be a multiple of 64\n", C);
        return false;
    }
    auto T = [&](const std::string & n) { return mf.find(n); };
    // a pipeline stage holds only its layers (+ embedding on the first, head on the last)
    if (first && (!upload_mat(dm, T("emb.weight"), dm.emb, false, false) ||
                  !(dm.ln0_w = upload_vec(dm, T("blocks.0.ln0.weight"))) ||
                  !(dm.ln0_b = upload_vec(dm, T("blocks.0.ln0.bias")))))
        return false;
    if (last && (!upload_mat(dm, T("head.weight"), dm.head, true, true) ||
                 !(dm.lnout_w = upload_vec(dm, T("ln_out.weight"))) || !(dm.lnout_b = upload_vec(dm, T("ln_out.bias")))))
        return false;
    dm.layers.resize(dm.n_layer);
    for (uint32_t i = dm.layer_lo; i < dm.layer_hi; i++) {
        DLayer & L = dm.layers[i];
        const std::string p = "blocks." + std::to_string(i) + ".";
        auto V = [&](const char * n) { return upload_vec(dm, T(p + n)); };
        auto Mt = [&](const char * n, DMat & d) { return upload_mat(dm, T(p + n), d, true, false); };
        bool ok = (L.ln1_w = V("ln1.weight")) && (L.ln1_b = V("ln1.bias")) && (L.ln2_w = V("ln2.weight")) &&
                  (L.ln2_b = V("ln2.bias"));
        ok = ok && Mt("att.key.weight", L.att_k) && Mt("att.value.weight", L.att_v) &&
             Mt("att.receptance.weight", L.att_r) && Mt("att.output.weight", L.att_o) &&
             Mt("ffn.key.weight", L.ffn_k) && Mt("ffn.value.weight", L.ffn_v);
        if (!ok) return false;
        dm.F = L.ffn_k.M;
        if (dm.major != 7 && !Mt("ffn.receptance.weight", L.ffn_r)) return false;
        if (dm.major == 4 || dm.major == 5) {
            ok = (L.att_mix_k = V("att.time_mix_k")) && (L.att_mix_v = V("att.time_mix_v")) &&
                 (L.att_mix_r = V("att.time_mix_r")) && (L.ffn_mix_k = V("ffn.time_mix_k")) &&
                 (L.ffn_mix_r = V("ffn.time_mix_r"));
            if (!ok) return false;
        }
        if (dm.major == 4) {
            if (!(L.att_first = V("att.time_first")) || !(L.att_decay = V("att.time_decay"))) return false;
        }
        if (dm.major >= 5) {
            if (!(L.att_lnx_w = V("att.ln_x.weight")) || !(L.att_lnx_b = V("att.ln_x.bias"))) return false;
        }
        if (dm.major == 5) {
            // wkv6 operands u and w expanded to [C] (5.1 repeats per head, rwkv_graph.inc:256-273)
            const HostTensor * dec = T(p + "att.time_decay");
            const HostTensor * fu = dm.minor >= 2 ? T(p + "att.time_faaaa") : T(p + "att.time_first");
            std::vector<float> u(C), w(C);
            const float * dd = (const float *)dec->data.data();
            const float * ff = (const float *)fu->data.data();
            if (dec->type != W_F32 || fu->type != W_F32) return false;
            for (int64_t h = 0; h < dm.H; h++)
                for (int64_t j = 0; j < dm.S; j++) {
                    u[h * dm.S + j] = dm.minor >= 2 ? ff[h * dm.S + j] : ff[h];
                    w[h * dm.S + j] = dm.minor >= 2 ? dd[h * dm.S + j] : dd[h];
                }
            if (!(L.att_u = upload_host_floats(dm, u)) || !(L.att_w = upload_host_floats(dm, w))) return false;
            if (dm.minor >= 2) {
                if (!(L.att_mix_g = V("att.time_mix_g")) || !Mt("att.gate.weight", L.att_g)) return false;
            }
        }
        if (dm.major == 6) {
            ok = (L.maa_x = V("att.time_maa_x")) && (L.maa[0] = V("att.time_maa_w")) && (L.maa[1] = V("att.time_maa_k")) &&
                 (L.maa[2] = V("att.time_maa_v")) && (L.maa[3] = V("att.time_maa_r")) && (L.maa[4] = V("att.time_maa_g")) &&
                 (L.maa_w2 = V("att.time_maa_w2")) && (L.att_u = V("att.time_faaaa")) && (L.decay6 = V("att.time_decay")) &&
                 (L.ffn_maa_k = V("ffn.time_maa_k")) && (L.ffn_maa_r = V("ffn.time_maa_r"));
            ok = ok && Mt("att.time_maa_w1", L.maa_w1) && Mt("att.time_decay_w1", L.decay_w1) &&
                 Mt("att.time_decay_w2", L.decay_w2) && Mt("att.gate.weight", L.att_g);
            if (!ok) return false;
            dm.maa_D = (int)T(p + "att.time_maa_w2")->ne[0];
            {
                const HostTensor * w2 = T(p + "att.time_maa_w2");
                if (w2->type != W_F32) return false;
                const size_t D = w2->ne[0], Cc = w2->ne[1];
                const float * src = (const float *)w2->data.data();
                std::vector<float> t(5 * D * Cc);
                for (size_t n = 0; n < 5; n++)
                    for (size_t c = 0; c < Cc; c++)
                        for (size_t i = 0; i < D; i++) t[(n * D + i) * Cc + c] = src[(n * Cc + c) * D + i];
                if (!(L.maa_w2t = upload_host_floats(dm, t))) return false;
                dm.small_param_bytes -= (double)t.size() * 4;  // same bytes as maa_w2, counted once
            }
            if (L.maa_w1.M != 5 * dm.maa_D) {
                fprintf(stderr, "rwkv: unexpected time_maa_w1 shape\n");
                return false;
            }
        }
        if (dm.major == 7) {
            ok = (L.x_rwkvag = V("att.x_rwkvag")) && (L.w0 = V("att.w0")) && (L.a0 = V("att.a0")) &&
                 (L.k_k = V("att.k_k")) && (L.k_a = V("att.k_a")) && (L.r_k = V("att.r_k")) && (L.ffn_x_k = V("ffn.x_k"));
            ok = ok && Mt("att.w1", L.w1) && Mt("att.w2", L.w2) && Mt("att.a1", L.a1) && Mt("att.a2", L.a2) &&
                 Mt("att.g1", L.g1) && Mt("att.g2", L.g2);
            if (ok && i != 0) ok = (L.v0 = V("att.v0")) && Mt("att.v1", L.v1) && Mt("att.v2", L.v2);
            if (!ok) return false;
        }
    }
    if (dm.H && dm.S > 64) {
        fprintf(stderr, "rwkv: head size %lld > 64 unsupported\n", (long long)dm.S);
        return false;
    }
    return hipDeviceSynchronize() == hipSuccess;
}

void free_model(DeviceModel & dm) {
    for (void * p : dm.allocs) (void)hipFree(p);
    dm.allocs.clear();
}

// ------------------------------------------------------------------------- engine

__global__ void k_init_state(float * st, size_t n, int C, int v4) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = 0.0f;
    if (v4) {
        const size_t in_layer = i % (5 * (size_t)C);
        if (in_layer >= 4 * (size_t)C) v = -1e30f;  // rwkv_eval.inc:224-241
    }
    st[i] = v;
}

Engine::~Engine() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    release_device();
    stamp_dump();
    drop_graphs();
    drop_io_graphs();
    for (hipStream_t s : io_stream_)
        if (s) (void)hipStreamDestroy(s);
    for (hipEvent_t e : io_ev_) (void)hipEventDestroy(e);
    if (io_entry_ev_) (void)hipEventDestroy(io_entry_ev_);
    drop_batch_graphs();
    for (float * p : bstate_)
        if (p) (void)hipFree(p);
    if (blogits_) (void)hipFree(blogits_);
    if (gy_) (void)hipFree(gy_);
    if (part_) (void)hipFree(part_);
    if (m2_) (void)hipFree(m2_);
    if (wkvc_) (void)hipFree(wkvc_);
    for (void * p : ws_allocs_) (void)hipFree(p);
    if (htokens_) (void)hipHostFree(htokens_);
    if (herr_h_) (void)hipHostFree(herr_h_);
    collect_timing();
    for (hipEvent_t e : event_pool_) (void)hipEventDestroy(e);
    if (tok_event_) (void)hipEventDestroy(tok_event_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

bool Engine::init() {
    HIP_OK(hipSetDevice(m_->device));
    stamp_init();
    {
        int cus = 0;
        HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, m_->device));
        set_mv_device_cus(cus);
    }
    HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&tok_event_, hipEventDisableTiming));
    HIP_OK(hipEventRecord(tok_event_, stream_));
    for (int i = 0; i < 2; i++) {
        HIP_OK(hipMalloc(&dstate_[i], m_->state_len * sizeof(float) + 16));
        ws_allocs_.push_back(dstate_[i]);
    }
    HIP_OK(hipMalloc(&logits_, (size_t)m_->n_vocab * sizeof(float) + 16));
    ws_allocs_.push_back(logits_);
    // in-launch hand-off (k_v6_att_fused): granules zeroed once here and re-armed by their readers;
    // the timeout flag is a host-mapped word, so checking it costs the host one load after a sync
    HIP_OK(hipHostMalloc((void **)&herr_h_, 64, hipHostMallocMapped | hipHostMallocCoherent));
    *(volatile unsigned *)herr_h_ = 0;
    HIP_OK(hipHostGetDevicePointer((void **)&herr_d_, herr_h_, 0));
    {
        hgran_n_ = 6 * (size_t)m_->n_embed;  // k_v6_att_fused granules: 4 C + H D (D <= 128, H = C / 64)
        HIP_OK(hipMalloc(&hgran_, hgran_n_ * 8));
        ws_allocs_.push_back(hgran_);
        HIP_OK(hipMemset(hgran_, 0, hgran_n_ * 8));
        // the tagged hand-offs (fused Wo, fused channel mix): tagged per (layer, state parity)
        const size_t C = m_->n_embed, kg = (size_t)KG_STRIDE * ((size_t)std::max(m_->F, 32) / 32);
        tgran_n_ = C + kg + C + C;
        HIP_OK(hipMalloc(&ygran_, tgran_n_ * 8));
        ws_allocs_.push_back(ygran_);
        HIP_OK(hipMemset(ygran_, 0, tgran_n_ * 8));
        kgran_ = ygran_ + C;
        rgran_ = kgran_ + kg;
        xgran_ = rgran_ + C;
    }
    // Per-context switches read when the context is created (each arm tested):
    const char * io = getenv("RWKV_MI355X_STATE_PIPELINE");  // 0: host state copied whole
    io_pipeline_ = !(io && io[0] == '0');
    const char * ic = getenv("RWKV_MI355X_IO_CHUNK");  // layers per chunk graph (host-state decode)
    io_chunk_ = ic ? std::max(1, atoi(ic)) : 4;
    const char * sm = getenv("RWKV_MI355X_SPLIT_MAA");  // 1: v6 decode W1 and mix as two launches
    split_maa_ = sm && sm[0] == '1';
    const char * df = getenv("RWKV_MI355X_DECODE_FUSION");  // mask of Engine::FUSE_* (default all)
    fuse_ = df ? (unsigned)strtoul(df, nullptr, 0) & FUSE_ALL : FUSE_DEFAULT | (m_->major == 4 ? FUSE_FFNCO : 0u);
    const char * wc = getenv("RWKV_MI355X_WKV_CHUNK");  // 1: chunk-parallel wkv6 (not bit-exact)
    wkv_chunk_ = wc && wc[0] == '1';
    // the fused decode prologues hold LayerNorm inputs in registers up to n_embed 4096
    if (m_->n_embed > 4096 || m_->n_embed % 64) generic_decode_ = true;
    return ensure_workspace(1) && init_state(dstate_[0]);
}

void Engine::drop_graphs() {
    for (auto & pc : graphs_)
        for (auto & pl : pc)
            for (hipGraphExec_t & g : pl) {
                if (g) (void)hipGraphExecDestroy(g);
                g = nullptr;
            }
}

// Contexts of this process with decode work queued per device (a context counts once from its
// first decode launch until it synchronises its stream).  The co-resident v6 attention layout
// (mv_att6c.hip) is safe only while its launches cannot share the compute units with another
// context's waiting launches: a context picks it when the count is 1 (itself).  Two contexts that
// claim at once both see 2; a context that picks it keeps the count until its launches finished.
static std::atomic<int> g_dev_claims[64];

void Engine::claim_device() {
    if (claimed_) return;
    claimed_ = true;
    g_dev_claims[m_->device & 63].fetch_add(1);
}

void Engine::release_device() {
    if (!claimed_) return;
    claimed_ = false;
    g_dev_claims[m_->device & 63].fetch_sub(1);
}

bool Engine::choose_co() {
    claim_device();
    bool co = co_knob_ == 1 || (co_knob_ < 0 && co_ok_ && g_dev_claims[m_->device & 63].load() == 1);
    // the co-resident forms: the v6 attention launch (with its Wo) and the channel mix's
    const bool att6 = (fuse_ & FUSE_ATT6) && (fuse_ & FUSE_WO6), sigmaa = (fuse_ & FUSE_SIGMAA) && (fuse_ & FUSE_SIG);
    co = co && ((m_->major == 6 && (att6 || sigmaa)) || (fuse_ & FUSE_FFNCO));
    // (both layouts hand y to Wo as the same Q8-block granules under the same tags: a switch needs
    // no clearing)
    co_ = co;
    co_pending_ += co;
    return co;
}

bool Engine::ensure_workspace(int T) {
    if (T <= tcap_) return true;
    HIP_OK(hipStreamSynchronize(stream_));
    drop_graphs();
    drop_batch_graphs();
    drop_io_graphs();
    // keep state and logits, drop the rest; until every allocation below has succeeded the
    // workspace counts as absent (tcap_ = 0, pointers null), so a failed grow can never leave a
    // capacity that points at freed or missing buffers
    std::vector<void *> keep = {dstate_[0], dstate_[1], logits_, hgran_, ygran_};
    for (void * p : ws_allocs_) {
        bool k = false;
        for (void * q : keep) k |= (p == q);
        if (!k) (void)hipFree(p);
    }
    ws_allocs_ = keep;
    tcap_ = 0;
    float ** fbufs[] = {&x_, &xa_, &sx_, &r_, &k_, &v_, &g_, &w_, &y_, &a_, &nb_, &bb_, &vfirst_, &fr_, &lora_, &bonus_};
    for (float ** b : fbufs) *b = nullptr;
    for (auto & p : dsmall_) p = nullptr;
    dtokens_ = nullptr;
    for (auto & s : slots_) s = ActSlot{};
    HIP_OK(hipEventSynchronize(tok_event_));
    if (htokens_) {
        (void)hipHostFree(htokens_);
        htokens_ = nullptr;
    }
    int cap = 1;
    while (cap < T) cap *= 2;
    const size_t C = m_->n_embed, TC = (size_t)cap * C;
    bool ok = true;
    auto A = [&](size_t bytes) -> void * {
        void * p = nullptr;
        if (!ok || hipMalloc(&p, bytes + 64) != hipSuccess) {
            ok = false;
            return nullptr;
        }
        ws_allocs_.push_back(p);
        return p;
    };
    float *x = nullptr, *xa = nullptr, *sx = nullptr, *r = nullptr, *k = nullptr, *v = nullptr, *g = nullptr,
          *w = nullptr, *y = nullptr, *a = nullptr, *nb = nullptr, *bb = nullptr, *vf = nullptr, *fr = nullptr;
    float ** locals[] = {&x, &xa, &sx, &r, &k, &v, &g, &w, &y, &a, &nb, &bb, &vf, &fr};
    for (float ** b : locals) *b = (float *)A(TC * 4);
    const size_t kmax = std::max<size_t>((size_t)m_->kmax, C);
    float * lora = (float *)A((size_t)cap * kmax * 4);
    float * bonus = (float *)A((size_t)cap * std::max<int64_t>(1, m_->H) * 4);
    float * dsmall[4];
    for (auto & p : dsmall) p = (float *)A(kmax * 4);
    uint32_t * dtok = (uint32_t *)A((size_t)cap * 4);
    ActSlot slots[kSlots];
    for (auto & s : slots) {
        const size_t n = (size_t)cap * kmax, nbk = n / 32 + 1;
        s.q = (int8_t *)A(n);
        s.d = (float *)A(nbk * 4);
        s.s = (float *)A(nbk * 4);
        s.qsum = (int *)A(nbk * 4);
        s.h = (__half *)A(n * 2);
        s.f = (float *)A(n * 4);
        // sequence-GEMM token tiles: whole QG_TOK-token tiles, records of up to qg_a_bytes(true)
        const size_t ttiles = ((size_t)cap + QG_TOK - 1) / QG_TOK;
        s.tq = (uint8_t *)A(ttiles * (kmax / 32 + 1) * qg_a_bytes(true));
    }
    uint32_t * htok = nullptr;
    if (ok && hipHostMalloc((void **)&htok, (size_t)cap * 4, hipHostMallocDefault) != hipSuccess) {
        htok = nullptr;
        ok = false;
    }
    if (!ok) {
        (void)hipGetLastError();  // clear the sticky out-of-memory status: later launches check it
        fprintf(stderr, "rwkv: device workspace allocation for %d tokens failed\n", cap);
        return false;  // tcap_ stays 0: the next call retries the allocation
    }
    for (size_t i = 0; i < sizeof(locals) / sizeof(*locals); i++) *fbufs[i] = *locals[i];
    lora_ = lora;
    bonus_ = bonus;
    for (int i = 0; i < 4; i++) dsmall_[i] = dsmall[i];
    dtokens_ = dtok;
    for (int i = 0; i < kSlots; i++) slots_[i] = slots[i];
    htokens_ = htok;
    tcap_ = cap;
    return true;
}

bool Engine::init_state(float * st, size_t n) {
    if (!n) n = m_->state_len;
    RK_LAUNCH(k_init_state, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream_, st, n,
                       (int)m_->n_embed, m_->major == 4 ? 1 : 0);
    HIP_OK(hipGetLastError());
    return true;
}

ActBuf Engine::Aview(int slot, int K, int fmt) const {
    const ActSlot & s = slots_[slot];
    ActBuf a;
    a.fmt = fmt;
    a.K = K;
    a.f = s.f;
    a.h = s.h;
    a.q = s.q;
    a.d = s.d;
    a.s = s.s;
    a.qsum = s.qsum;
    a.tq = s.tq;
    a.tiled = tile_acts_ && (fmt == A_Q8_0 || fmt == A_Q8_1);
    return a;
}

ActBuf Engine::A(int slot, const DMat & W) const { return Aview(slot, W.K, act_fmt_for(W.type)); }

// Collects matmul entries and launches them grouped by weight type.
struct MMBatch {
    std::vector<MMEntry> e;
    void add(const DMat & W, const ActBuf & in, float * y, int ldy, int epi, const float * aux = nullptr,
             const float * bias = nullptr, const ActBuf * out = nullptr) {
        MMEntry m;
        memset(&m, 0, sizeof(m));
        m.W = W;
        m.in = in;
        m.y = y;
        m.ldy = ldy;
        m.aux = aux;
        m.bias = bias;
        m.epi = epi;
        if (out) {
            m.out = *out;
            m.emit = 1;
        }
        e.push_back(m);
    }
    bool run(Engine & eng, int T) {
        std::vector<bool> done(e.size(), false);
        for (size_t i = 0; i < e.size(); i++) {
            if (done[i]) continue;
            MMGroup g;
            memset(&g, 0, sizeof(g));
            g.T = T;
            const int type = e[i].W.type;
            for (size_t j = i; j < e.size() && g.n < MM_MAX_ENTRIES; j++) {
                if (!done[j] && e[j].W.type == type) {
                    g.e[g.n++] = e[j];
                    done[j] = true;
                }
            }
            if (!eng.mm_launch(g, type)) return false;
        }
        e.clear();
        return true;
    }
};

static double act_bytes(const ActBuf & a, double T) {
    const double K = a.K;
    switch (a.fmt) {
        case A_F32: return T * K * 4;
        case A_F16: return T * K * 2;
        case A_Q8_1: return T * K + T * K / 32 * 12;
        default: return T * K + T * K / 32 * 8;
    }
}

static double wbytes(const DMat & W) { return (double)type_nbytes((uint32_t)W.type, (uint64_t)W.M * W.K); }

void Engine::set_timing(bool on) {
    (void)hipStreamSynchronize(stream_);
    collect_timing();
    timing_ = on;
    if (on) stats_.clear();
}

// Split-K partial scratch of at least n floats (grows; captured batched graphs point at the old one)
bool Engine::ensure_part(size_t n) {
    if (n <= part_cap_) return true;
    HIP_OK(hipStreamSynchronize(stream_));
    drop_batch_graphs();
    if (part_) (void)hipFree(part_);
    part_ = nullptr;
    part_cap_ = 0;
    if (hipMalloc(&part_, n * 4 + 64) != hipSuccess) {
        part_ = nullptr;
        (void)hipGetLastError();
        return false;
    }
    part_cap_ = n;
    return true;
}

// Sequence matmuls on quantized weights go to the int8-MFMA GEMM; entries that only emit get
// a scratch y, and emission is a separate quantization pass (same bits as k_mm's epilogue).
bool Engine::mm_dispatch(MMGroup & g, int wtype) {
    // batched decode (bs_ > 0): the decode matvec over the contexts (k_mvb; k_mm for shapes it
    // does not cover -- the same bits); from batch_gemm_min_ contexts on, the quantized matmuls
    // take the int8-MFMA sequence GEMM on token tiles instead (tile_acts_; also the same bits)
    if (!wtype_quantized(wtype) && g.T >= 32) {
        // k_fmm may split the class tree of a small grid (the v7 LoRA first stage): partials, only
        // when launch_fmm_group's rule can split this group (below 2 workgroups per CU)
        size_t msum = 0;
        int blocks = 0;
        bool splittable = true;
        for (int i = 0; i < g.n; i++) {
            msum += g.e[i].W.M;
            blocks += (g.e[i].W.M + 63) / 64 * ((g.T + 63) / 64);
            splittable = splittable && g.e[i].W.K >= 512 && g.e[i].W.M % 32 == 0;
        }
        if (splittable && blocks < 2 * kQgCUs) {
            const size_t split = (size_t)blocks * 4 >= (size_t)2 * kQgCUs ? 4 : 8;
            if (!ensure_part(split * g.T * msum)) return false;
            g.part = part_;
            g.part_floats = part_cap_;
        }
    }
    if (bs_ && !(tile_acts_ && wtype_quantized(wtype))) {
        bool launched = false;
        // float weights (the F16 head, LoRA) over 16+ contexts: the f32-MFMA form, same bits
        if (!launch_fmm_group(stream_, g, wtype, &launched)) return false;
        if (launched) return true;
        if (!launch_mvb_group(stream_, g, wtype, &launched)) return false;
        if (launched) return true;
        return launch_mm_group(stream_, g, wtype);
    }
    if (g.T < 2 || !wtype_quantized(wtype) || use_mm_) return launch_mm_group(stream_, g, wtype);
    size_t need = 0;
    for (int i = 0; i < g.n; i++)
        if (!g.e[i].y) need += (size_t)g.T * g.e[i].W.M;
    if (need > gy_cap_) {
        HIP_OK(hipStreamSynchronize(stream_));
        drop_batch_graphs();  // captured batched steps point at the old scratch
        if (gy_) (void)hipFree(gy_);
        gy_ = nullptr;
        gy_cap_ = 0;
        if (hipMalloc(&gy_, need * 4 + 64) != hipSuccess) {
            gy_ = nullptr;
            (void)hipGetLastError();
            return false;
        }
        gy_cap_ = need;
    }
    // split-K partials (launch_qgemm splits groups with few tiles: small T or small M)
    {
        const int rows = qg_rows(wtype), tilesT = (g.T + QG_TOK - 1) / QG_TOK;
        size_t msum = 0, tiles = 0;
        for (int i = 0; i < g.n; i++) {
            msum += g.e[i].W.M;
            tiles += (size_t)(g.e[i].W.M + rows - 1) / rows * tilesT;
        }
        if (tiles < 1024) {
            if (!ensure_part((size_t)8 * g.T * msum)) return false;
            g.part = part_;
            g.part_floats = part_cap_;
        }
        if (qg_one(wtype)) {
            const size_t mneed = (size_t)g.T * msum;
            if (mneed > m2_cap_) {
                HIP_OK(hipStreamSynchronize(stream_));
                drop_batch_graphs();
                if (m2_) (void)hipFree(m2_);
                m2_ = nullptr;
                m2_cap_ = 0;
                if (hipMalloc(&m2_, mneed * 4 + 64) != hipSuccess) {
                    m2_ = nullptr;
                    (void)hipGetLastError();
                    return false;
                }
                m2_cap_ = mneed;
            }
            g.m2 = m2_;
            g.m2_floats = m2_cap_;
        }
    }
    size_t off = 0;
    for (int i = 0; i < g.n; i++) {
        MMEntry & e = g.e[i];
        if (!e.y) {
            e.y = gy_ + off;
            e.ldy = e.W.M;
            off += (size_t)g.T * e.W.M;
        }
    }
    if (!launch_qgemm(stream_, g, wtype)) return false;
    for (int i = 0; i < g.n; i++) {
        const MMEntry & e = g.e[i];
        if (e.emit && !e.fuse_emit && e.ldy == e.W.M && !launch_act_from_f32(stream_, e.y, g.T, e.W.M, e.out))
            return false;
        if (e.emit && e.ldy != e.W.M) {
            fprintf(stderr, "rwkv: emitting GEMM entry needs ldy == M\n");
            return false;
        }
    }
    return true;
}

bool Engine::mm_launch(MMGroup & g, int wtype) {
    if (!timing_) return mm_dispatch(g, wtype);
    bool emit = false;
    double bytes = 0, flops = 0;
    for (int i = 0; i < g.n; i++) {
        const MMEntry & e = g.e[i];
        emit |= e.emit != 0;
        bytes += (double)type_nbytes((uint32_t)e.W.type, (uint64_t)e.W.M * e.W.K) + act_bytes(e.in, g.T);
        if (e.y) bytes += (double)g.T * e.W.M * 4 * ((e.epi == EPI_ADD || e.epi == EPI_SIGMUL_ADD || e.epi == EPI_VMIX7) ? 2 : 1);
        if (e.emit) bytes += act_bytes(e.out, g.T);
        flops += 2.0 * e.W.M * e.W.K * g.T;
    }
    // kernel class = the template instantiation rocprofv3 reports: k_mm<WF, RPW, NT>
    const bool mfma = g.T >= 2 && wtype_quantized(wtype) && !use_mm_ && (!bs_ || tile_acts_);
    const std::string name = mfma ? "k_qgemm<" + std::to_string(wtype) + ">"
                           : bs_ ? "k_mvb<" + std::to_string(wtype) + ">"
                                  : "k_mm<" + std::to_string(wtype) + ", " + (emit ? "8" : "2") + ", " + (g.T == 1 ? "1" : "4") + ">";
    const int si = add_stat(name);
    hipEvent_t a, b;
    if (event_pool_.size() >= 2) {
        a = event_pool_.back();
        event_pool_.pop_back();
        b = event_pool_.back();
        event_pool_.pop_back();
    } else {
        HIP_OK(hipEventCreate(&a));
        HIP_OK(hipEventCreate(&b));
    }
    HIP_OK(hipEventRecord(a, stream_));
    const bool ok = mm_dispatch(g, wtype);
    HIP_OK(hipEventRecord(b, stream_));
    pending_.push_back(Pending{si, a, b, bytes, flops});
    return ok;
}

int Engine::add_stat(const std::string & name) {
    for (size_t i = 0; i < stats_.size(); i++)
        if (stats_[i].name == name) return (int)i;
    stats_.push_back(KernelStat{name});
    return (int)stats_.size() - 1;
}

void Engine::collect_timing() {
    for (auto & p : pending_) {
        float ms = 0;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            KernelStat & s = stats_[p.stat];
            s.total_ms += ms;
            s.total_bytes += p.bytes;
            s.total_flops += p.flops;
            s.launches++;
        }
        event_pool_.push_back(p.a);
        event_pool_.push_back(p.b);
    }
    pending_.clear();
}

const std::vector<KernelStat> & Engine::stats() {
    (void)hipStreamSynchronize(stream_);
    collect_timing();
    return stats_;
}

bool Engine::ffn(int l, int T, const float * si, float * so) {
    const DLayer & L = m_->layers[l];
    const int C = (int)m_->n_embed;
    LnMixArgs a;
    memset(&a, 0, sizeof(a));
    a.T = T;
    a.C = C;
    a.x = x_;
    a.carry_in = si;        // ffn_xx at layer offset 0
    a.carry_out = so;
    a.bs = bs_;
    a.lnw = L.ln2_w;
    a.lnb = L.ln2_b;
    MMBatch b;
    if (m_->major == 7) {
        // rwkv_graph.inc:533-543
        a.form = 1;
        a.n_out = 1;
        a.mu[0] = L.ffn_x_k;
        a.out[0] = A(0, L.ffn_k);
        if (!launch_ln_mix(stream_, a)) return false;
        ActBuf kin = A(1, L.ffn_v);
        b.add(L.ffn_k, A(0, L.ffn_k), nullptr, 0, EPI_RELU_SQ, nullptr, nullptr, &kin);
        if (!b.run(*this, T)) return false;
        b.add(L.ffn_v, kin, x_, C, EPI_ADD);
        return b.run(*this, T);
    }
    // v4/v5: rwkv_graph.inc:484-511 (form 0); v6: :513-531 (form 1)
    a.form = m_->major == 6 ? 1 : 0;
    a.n_out = 2;
    a.mu[0] = m_->major == 6 ? L.ffn_maa_k : L.ffn_mix_k;
    a.mu[1] = m_->major == 6 ? L.ffn_maa_r : L.ffn_mix_r;
    a.out[0] = A(0, L.ffn_k);
    a.out[1] = A(1, L.ffn_r);
    if (!launch_ln_mix(stream_, a)) return false;
    ActBuf kin = A(2, L.ffn_v);
    b.add(L.ffn_r, A(1, L.ffn_r), fr_, C, EPI_STORE);
    b.add(L.ffn_k, A(0, L.ffn_k), nullptr, 0, EPI_RELU_SQ, nullptr, nullptr, &kin);
    if (!b.run(*this, T)) return false;
    b.add(L.ffn_v, kin, x_, C, EPI_SIGMUL_ADD, fr_);
    return b.run(*this, T);
}

// Batched decode (bs_ > 0): the attention core of every context is the decode kernel itself (one
// workgroup per head and context, k_att6_dec / k_att7_dec); its output goes to Wo's input `o`
// (emitted by the kernel when heads are whole quantization blocks, else fp32 y_ converted).
template <class Att>
static void batch_att(Att & a, int T, size_t bs, float * y, const ActBuf & o, int S) {
    a.nb = T;
    a.bs = bs;
    a.y = y;
    a.yq.fmt = -1;
    if (S >= 32) a.yq = o;
}

bool Engine::layer_v4(int l, int T, const float * si, float * so) {
    const DLayer & L = m_->layers[l];
    const int C = (int)m_->n_embed;
    LnMixArgs a;
    memset(&a, 0, sizeof(a));
    a.T = T;
    a.C = C;
    a.x = x_;
    a.carry_in = si + C;
    a.carry_out = so + C;
    a.bs = bs_;
    a.lnw = L.ln1_w;
    a.lnb = L.ln1_b;
    a.form = 0;
    a.n_out = 3;
    a.mu[0] = L.att_mix_k;
    a.mu[1] = L.att_mix_v;
    a.mu[2] = L.att_mix_r;
    a.out[0] = A(0, L.att_k);
    a.out[1] = A(1, L.att_v);
    a.out[2] = A(2, L.att_r);
    if (!launch_ln_mix(stream_, a)) return false;
    MMBatch b;
    b.add(L.att_r, A(2, L.att_r), r_, C, EPI_SIGMOID);
    b.add(L.att_k, A(0, L.att_k), k_, C, EPI_STORE);
    b.add(L.att_v, A(1, L.att_v), v_, C, EPI_STORE);
    if (!b.run(*this, T)) return false;
    ActBuf o = A(3, L.att_o);
    if (!launch_wkv4(stream_, T, C, r_, k_, v_, L.att_first, L.att_decay, si, so, o, (int)bs_)) return false;
    b.add(L.att_o, o, x_, C, EPI_ADD);
    if (!b.run(*this, T)) return false;
    return ffn(l, T, si, so);
}

// The chunked WKV scratch (wkv_chunk.hip, wkv7_chunk.hip), grown on demand.
bool Engine::ensure_wkvc(size_t need) {
    if (need <= wkvc_cap_) return true;
    HIP_OK(hipStreamSynchronize(stream_));
    if (wkvc_) (void)hipFree(wkvc_);
    wkvc_ = nullptr;
    wkvc_cap_ = 0;
    if (hipMalloc(&wkvc_, need * 4 + 64) != hipSuccess) {
        wkvc_ = nullptr;
        (void)hipGetLastError();
        fprintf(stderr, "rwkv: chunked wkv scratch (%zu MB) allocation failed\n", need * 4 >> 20);
        return false;
    }
    wkvc_cap_ = need;
    return true;
}

// v5/v6 sequence wkv: the serial recurrence (k_wkv6_s64, bit-exact with decode), or behind the
// wkv_chunk_ switch the chunk-parallel form (RA / KB in the v7-only nb_ / bb_ buffers, free during a
// v5/v6 layer; the chunk matrices and states in wkvc_, grown on demand)
bool Engine::wkv6(int T, int H, int S, const float * u, const float * w, int wpt, const float * sin, float * sout) {
    if (wkv_chunk_ && wkv6_chunked_supported(T, S, (int)bs_)) {
        if (!ensure_wkvc(wkv6_chunked_scratch_floats(T, H))) return false;
        return launch_wkv6_chunked(stream_, T, H, k_, v_, r_, u, w, wpt, sin, sout, y_, nb_, bb_, wkvc_);
    }
    return launch_wkv6(stream_, T, H, S, k_, v_, r_, u, w, wpt, sin, sout, y_, (int)bs_);
}

bool Engine::layer_v5(int l, int T, const float * si, float * so) {
    const DLayer & L = m_->layers[l];
    const int C = (int)m_->n_embed, H = (int)m_->H, S = (int)m_->S;
    const bool v52 = m_->minor >= 2;
    LnMixArgs a;
    memset(&a, 0, sizeof(a));
    a.T = T;
    a.C = C;
    a.x = x_;
    a.carry_in = si + C;
    a.carry_out = so + C;
    a.bs = bs_;
    a.lnw = L.ln1_w;
    a.lnb = L.ln1_b;
    a.form = 0;
    a.n_out = v52 ? 4 : 3;
    a.mu[0] = L.att_mix_k;
    a.mu[1] = L.att_mix_v;
    a.mu[2] = L.att_mix_r;
    a.out[0] = A(0, L.att_k);
    a.out[1] = A(1, L.att_v);
    a.out[2] = A(2, L.att_r);
    if (v52) {
        a.mu[3] = L.att_mix_g;
        a.out[3] = A(3, L.att_g);
    }
    if (!launch_ln_mix(stream_, a)) return false;
    MMBatch b;
    b.add(L.att_r, A(2, L.att_r), r_, C, EPI_STORE);
    b.add(L.att_k, A(0, L.att_k), k_, C, EPI_STORE);
    b.add(L.att_v, A(1, L.att_v), v_, C, EPI_STORE);
    if (v52) b.add(L.att_g, A(3, L.att_g), g_, C, EPI_SILU);
    if (!b.run(*this, T)) return false;
    if (bs_) {
        Att6Dec d;
        memset(&d, 0, sizeof(d));
        d.H = H;
        d.S = S;
        d.r = r_;
        d.k = k_;
        d.v = v_;
        d.g = v52 ? g_ : nullptr;
        d.u = L.att_u;
        d.w = L.att_w;
        d.sin = si + 2 * C;
        d.sout = so + 2 * C;
        d.lnx_w = L.att_lnx_w;
        d.lnx_b = L.att_lnx_b;
        d.eps = 1e-5f;
        ActBuf o = A(4, L.att_o);
        batch_att(d, T, bs_, y_, o, S);
        if (!launch_att6_dec(stream_, d)) return false;
        if (S < 32 && !launch_act_from_f32(stream_, y_, T, C, o)) return false;
        b.add(L.att_o, o, x_, C, EPI_ADD);
        if (!b.run(*this, T)) return false;
        return ffn(l, T, si, so);
    }
    if (!wkv6(T, H, S, L.att_u, L.att_w, 0, si + 2 * C, so + 2 * C)) return false;
    ActBuf o = A(4, L.att_o);
    if (!launch_groupnorm(stream_, T, H, S, 1e-5f, y_, L.att_lnx_w, L.att_lnx_b, v52 ? 1 : 0, g_, nullptr, nullptr, o))
        return false;
    b.add(L.att_o, o, x_, C, EPI_ADD);
    if (!b.run(*this, T)) return false;
    return ffn(l, T, si, so);
}

bool Engine::layer_v6(int l, int T, const float * si, float * so) {
    const DLayer & L = m_->layers[l];
    const int C = (int)m_->n_embed, H = (int)m_->H, S = (int)m_->S, D = m_->maa_D;
    LnMixArgs a;
    memset(&a, 0, sizeof(a));
    a.T = T;
    a.C = C;
    a.x = x_;
    a.carry_in = si + C;
    a.carry_out = so + C;
    a.bs = bs_;
    a.lnw = L.ln1_w;
    a.lnb = L.ln1_b;
    a.form = 1;
    a.n_out = 1;
    a.mu[0] = L.maa_x;
    a.out[0] = A(0, L.maa_w1);
    a.out_xa = xa_;
    a.out_sx = sx_;
    if (!launch_ln_mix(stream_, a)) return false;
    MMBatch b;
    b.add(L.maa_w1, A(0, L.maa_w1), lora_, 5 * D, EPI_TANH);
    if (!b.run(*this, T)) return false;
    // order w, k, v, r, g (rwkv_graph.inc:336-346)
    ActBuf outs[5] = {A(1, L.decay_w1), A(2, L.att_k), A(3, L.att_v), A(4, L.att_r), A(5, L.att_g)};
    // batched decode: the decode kernel's per-(mix, channel) arithmetic over the contexts; from
    // batch_gemm_min_ contexts on (token-tile outputs) the sequence kernel's f32-MFMA form over the
    // contexts as tokens -- W2 read once per 64 contexts instead of once per context, same bits
    if ((bs_ && !tile_acts_) ? !launch_v6_mix5_dec(stream_, C, D, xa_, nullptr, lora_, L.maa_w2t, L.maa, outs, T, sx_)
                             : !launch_v6_mix5(stream_, T, C, D, lora_, L.maa_w2t, L.maa, xa_, sx_, outs))
        return false;
    ActBuf dl = A(6, L.decay_w2);
    // decay tail by threads (k_att6_dec's rows) when Wd2 is quantized; dl fp32 then reuses lora_
    // (consumed by mix5 above)
    const int DD = L.decay_w2.K;  // decay LoRA width (64 for the released checkpoints)
    const bool dseq = v6_decay_seq_supported(L.decay_w2.type, DD) && L.decay_w1.M == DD;
    if (bs_) {
        // decode's split: decay W1 (tanh) with r,k,v,g; the LoRA tail, wkv and GroupNorm per head
        b.add(L.att_r, outs[3], r_, C, EPI_STORE);
        b.add(L.att_k, outs[1], k_, C, EPI_STORE);
        b.add(L.att_v, outs[2], v_, C, EPI_STORE);
        b.add(L.att_g, outs[4], g_, C, EPI_SILU);
        b.add(L.decay_w1, outs[0], lora_, L.decay_w1.M, EPI_TANH);
        if (!b.run(*this, T)) return false;
        Att6Dec d;
        memset(&d, 0, sizeof(d));
        d.H = H;
        d.S = S;
        d.r = r_;
        d.k = k_;
        d.v = v_;
        d.g = g_;
        d.u = L.att_u;
        d.wd2 = L.decay_w2;
        d.dl = lora_;
        d.ldd = L.decay_w1.M;
        d.decay = L.decay6;
        d.sin = si + 2 * C;
        d.sout = so + 2 * C;
        d.lnx_w = L.att_lnx_w;
        d.lnx_b = L.att_lnx_b;
        d.eps = 64e-5f;
        ActBuf o = A(7, L.att_o);
        batch_att(d, T, bs_, y_, o, S);
        if (!launch_att6_dec(stream_, d)) return false;
        if (S < 32 && !launch_act_from_f32(stream_, y_, T, C, o)) return false;
        b.add(L.att_o, o, x_, C, EPI_ADD);
        if (!b.run(*this, T)) return false;
        return ffn(l, T, si, so);
    }
    b.add(L.att_r, outs[3], r_, C, EPI_STORE);
    b.add(L.att_k, outs[1], k_, C, EPI_STORE);
    b.add(L.att_v, outs[2], v_, C, EPI_STORE);
    b.add(L.att_g, outs[4], g_, C, EPI_SILU);
    if (dseq) b.add(L.decay_w1, outs[0], lora_, DD, EPI_TANH);
    else b.add(L.decay_w1, outs[0], nullptr, 0, EPI_TANH, nullptr, nullptr, &dl);
    if (!b.run(*this, T)) return false;
    if (dseq) {
        if (!launch_v6_decay_seq(stream_, T, C, L.decay_w2, lora_, L.decay6, w_)) return false;
    } else {
        b.add(L.decay_w2, dl, w_, C, EPI_DECAY6, nullptr, L.decay6);
        if (!b.run(*this, T)) return false;
    }
    if (!wkv6(T, H, S, L.att_u, w_, 1, si + 2 * C, so + 2 * C)) return false;
    ActBuf o = A(7, L.att_o);
    if (!launch_groupnorm(stream_, T, H, S, 64e-5f, y_, L.att_lnx_w, L.att_lnx_b, 1, g_, nullptr, nullptr, o)) return false;
    b.add(L.att_o, o, x_, C, EPI_ADD);
    if (!b.run(*this, T)) return false;
    return ffn(l, T, si, so);
}

bool Engine::layer_v7(int l, int T, const float * si, float * so) {
    const DLayer & L = m_->layers[l];
    const int C = (int)m_->n_embed, H = (int)m_->H, S = (int)m_->S;
    LnMixArgs a;
    memset(&a, 0, sizeof(a));
    a.T = T;
    a.C = C;
    a.x = x_;
    a.carry_in = si + C;
    a.carry_out = so + C;
    a.bs = bs_;
    a.lnw = L.ln1_w;
    a.lnb = L.ln1_b;
    a.form = 1;
    // order r, w, k, v, a, g (rwkv_graph.inc:404-413)
    const DMat * cons[6] = {&L.att_r, &L.w1, &L.att_k, &L.att_v, &L.a1, &L.g1};
    a.n_out = 6;
    for (int n = 0; n < 6; n++) {
        a.mu[n] = L.x_rwkvag + (size_t)n * C;
        a.out[n] = A(n, *cons[n]);
    }
    const bool vlora = l != 0;
    ActBuf xv1;
    if (vlora) {
        xv1 = A(9, L.v1);
        if (xv1.fmt == a.out[3].fmt) {
            xv1 = a.out[3];
            xv1.K = L.v1.K;
        } else {
            // second emission of xv in the LoRA's input format; mix kernels take <= 6 outputs,
            // so re-run the mix for this one vector
            LnMixArgs a2 = a;
            a2.n_out = 1;
            a2.mu[0] = a.mu[3];
            a2.out[0] = xv1;
            a2.carry_out = nullptr;
            if (!launch_ln_mix(stream_, a2)) return false;
        }
    }
    if (!launch_ln_mix(stream_, a)) return false;
    MMBatch b;
    ActBuf lw = A(6, L.w2), la = A(7, L.a2), lg = A(8, L.g2);
    b.add(L.att_r, a.out[0], r_, C, EPI_STORE);
    b.add(L.att_k, a.out[2], k_, C, EPI_STORE);
    b.add(L.att_v, a.out[3], v_, C, EPI_STORE);
    b.add(L.w1, a.out[1], nullptr, 0, EPI_TANH, nullptr, nullptr, &lw);
    b.add(L.a1, a.out[4], nullptr, 0, EPI_STORE, nullptr, nullptr, &la);
    b.add(L.g1, a.out[5], nullptr, 0, EPI_SIGMOID, nullptr, nullptr, &lg);
    ActBuf lvv;
    if (vlora) {
        lvv = A(10, L.v2);
        b.add(L.v1, xv1, nullptr, 0, EPI_STORE, nullptr, nullptr, &lvv);
    }
    if (!b.run(*this, T)) return false;
    if (l == 0) {
        HIP_OK(hipMemcpyAsync(vfirst_, v_, (size_t)T * C * 4, hipMemcpyDeviceToDevice, stream_));
    }
    b.add(L.w2, lw, w_, C, EPI_DECAY7, nullptr, L.w0);
    b.add(L.a2, la, a_, C, EPI_SIGMOID_BIAS, nullptr, L.a0);
    b.add(L.g2, lg, g_, C, EPI_STORE);
    if (vlora) b.add(L.v2, lvv, v_, C, EPI_VMIX7, vfirst_, L.v0);
    if (!b.run(*this, T)) return false;
    if (bs_) {
        Att7Dec d;
        memset(&d, 0, sizeof(d));
        d.H = H;
        d.S = S;
        d.r = r_;
        d.w = w_;
        d.k = k_;
        d.v = v_;
        d.a = a_;
        d.g = g_;
        d.k_k = L.k_k;
        d.k_a = L.k_a;
        d.r_k = L.r_k;
        d.sin = si + 2 * C;
        d.sout = so + 2 * C;
        d.lnx_w = L.att_lnx_w;
        d.lnx_b = L.att_lnx_b;
        ActBuf o = A(0, L.att_o);
        batch_att(d, T, bs_, y_, o, S);
        if (!launch_att7_dec(stream_, d)) return false;
        if (S < 32 && !launch_act_from_f32(stream_, y_, T, C, o)) return false;
        b.add(L.att_o, o, x_, C, EPI_ADD);
        if (!b.run(*this, T)) return false;
        return ffn(l, T, si, so);
    }
    if (!launch_v7_prep(stream_, T, H, S, k_, a_, r_, L.k_k, L.k_a, L.r_k, nb_, bb_, bonus_)) return false;
    // the serial recurrence (bit-exact with decode), or behind the wkv_chunk_ switch the chunk-parallel
    // form (wkv7_chunk.hip; scratch in wkvc_)
    if (wkv_chunk_ && wkv7_chunked_supported(T, S, (int)bs_)) {
        if (!ensure_wkvc(wkv7_chunked_scratch_floats(T, H))) return false;
        if (!launch_wkv7_chunked(stream_, T, H, r_, w_, k_, v_, nb_, bb_, si + 2 * C, so + 2 * C, y_, wkvc_)) return false;
    } else if (!launch_wkv7(stream_, T, H, S, r_, w_, k_, v_, nb_, bb_, si + 2 * C, so + 2 * C, y_, (int)bs_)) {
        return false;
    }
    ActBuf o = A(0, L.att_o);
    if (!launch_groupnorm(stream_, T, H, S, 64e-5f, y_, L.att_lnx_w, L.att_lnx_b, 2, g_, v_, bonus_, o)) return false;
    b.add(L.att_o, o, x_, C, EPI_ADD);
    if (!b.run(*this, T)) return false;
    return ffn(l, T, si, so);
}

bool Engine::forward(int T, const float * sin, float * sout, bool logits) {
    if (T == 1 && !generic_decode_) return forward_decode(sin, sout, logits);
    return forward_range(T, sin, sout, 0, m_->n_layer, logits);
}

// Layers [l0, l1) over T tokens; l0 == 0 embeds the tokens into x_, otherwise x_ (and, v7,
// vfirst_) already hold the stream entering l0.  Head on the last token when l1 == n_layer.
bool Engine::forward_range(int T, const float * sin, float * sout, uint32_t l0, uint32_t l1, bool logits) {
    const size_t C = m_->n_embed;
    last_decode_ = false;
    if (l0 == 0 && !launch_embed_ln(stream_, dtokens_, T, m_->emb, m_->ln0_w, m_->ln0_b, x_)) return false;
    const size_t per_layer = m_->major >= 5 ? C * (2 + (size_t)m_->S) : 5 * C;
    // layer matmuls run over all T tokens: Q8 activations go straight into GEMM tiles
    tile_acts_ = T >= 2 && !use_mm_ && (!bs_ || T >= batch_gemm_min_);
    for (uint32_t l = l0; l < l1; l++) {
        const float * si = sin + l * per_layer;
        float * so = sout + l * per_layer;
        bool ok = false;
        switch (m_->major) {
            case 4: ok = layer_v4((int)l, T, si, so); break;
            case 5: ok = layer_v5((int)l, T, si, so); break;
            case 6: ok = layer_v6((int)l, T, si, so); break;
            case 7: ok = layer_v7((int)l, T, si, so); break;
            default: break;
        }
        if (!ok) {
            tile_acts_ = false;
            return false;
        }
    }
    tile_acts_ = false;  // the head runs on the last token only (batched decode: on every context)
    if (logits && l1 == m_->n_layer) {
        // rwkv_graph.inc:704-708 / :850-854
        const int rows = bs_ ? T : 1;
        ActBuf hin = A(0, m_->head);
        if (!launch_ln_emit(stream_, (int)C, x_ + (size_t)(T - rows) * C, m_->lnout_w, m_->lnout_b, hin, rows))
            return false;
        MMBatch b;
        b.add(m_->head, hin, head_out_ ? head_out_ : logits_, (int)m_->n_vocab, EPI_STORE);
        if (!b.run(*this, rows)) return false;
    }
    return true;
}

bool Engine::mv(MVGroup & g, hipStream_t st) {
    if (timing_) {
        // the group's single launch is timed by its own dispatch events (RK_LAUNCH, g_klt)
        double bytes = 0, flops = 0;
        for (int i = 0; i < g.n; i++) {
            const MVEntry & e = g.e[i];
            bytes += (double)type_nbytes((uint32_t)e.W.type, (uint64_t)e.W.M * e.W.K);
            bytes += e.src == SRC_ACT ? act_bytes(e.act, 1) : (double)e.W.K * 4 * (e.src == SRC_LNMIX ? 5 : 1);
            bytes += (double)e.W.M * 4 * ((e.epi == EPI_ADD || e.epi == EPI_SIGMUL_ADD || e.epi == EPI_VMIX7) ? 2 : 1);
            flops += 2.0 * e.W.M * e.W.K;
        }
        kt_bytes_ = bytes;
        kt_flops_ = flops;
    }
    return launch_mv_group(st ? st : stream_, g);
}

// KLaunchTimer (common.hpp): while a decode step is timed, every RK_LAUNCH takes an event pair
// bound to its dispatch; the algorithmic bytes / flops set by the caller just before (kt_bytes_)
// go to the first launch after them.
bool Engine::begin(hipEvent_t * a, hipEvent_t * b) {
    if (event_pool_.size() < 2) {
        hipEvent_t x, y;
        if (hipEventCreate(&x) != hipSuccess) return false;
        if (hipEventCreate(&y) != hipSuccess) {
            (void)hipEventDestroy(x);
            return false;
        }
        event_pool_.push_back(x);
        event_pool_.push_back(y);
    }
    *a = event_pool_.back();
    event_pool_.pop_back();
    *b = event_pool_.back();
    event_pool_.pop_back();
    kt_a_ = *a;
    kt_b_ = *b;
    return true;
}

void Engine::end(const char * kernel) {
    // "(k_mva<WFIX, Rv, Uv>)" -> "k_mva"
    std::string n(kernel);
    while (!n.empty() && (n[0] == '(' || n[0] == ' ')) n.erase(0, 1);
    const size_t cut = n.find_first_of("<) ");
    if (cut != std::string::npos) n.resize(cut);
    pending_.push_back(Pending{add_stat(n), kt_a_, kt_b_, kt_bytes_, kt_flops_});
    kt_bytes_ = kt_flops_ = 0;
}

// Builder for decode matvec groups.
struct MV {
    MVGroup g;
    MV() { memset(&g, 0, sizeof(g)); }
    MVEntry & add(const DMat & W, float * y, int epi, const float * aux = nullptr, const float * bias = nullptr) {
        MVEntry & e = g.e[g.n++];
        e.W = W;
        e.y = y;
        e.epi = epi;
        e.aux = aux;
        e.bias = bias;
        return e;
    }
};

static void src_lnmix(MVEntry & e, const float * x, const float * carry, const float * lnw, const float * lnb,
                      const float * mu, int form, float * carry_out = nullptr) {
    e.src = SRC_LNMIX;
    e.x = x;
    e.carry = carry;
    e.lnw = lnw;
    e.lnb = lnb;
    e.mu = mu;
    e.form = form;
    e.carry_out = carry_out;
}

static void src_f32(MVEntry & e, const float * f) {
    e.src = SRC_F32;
    e.f = f;
}

// Single-token forward: the fused decode program (kernels_decode.hip).  Per layer:
//   v6: W1+LN (1) -> mix5 (1) -> r,k,v,g,Wd1 (1) -> decay tail+wkv+GN (1) -> Wo (1) -> FFN k,r+LN (1) -> FFN v (1)
//   v5: r,k,v,g+LN (1) -> wkv+GN (1) -> Wo (1) -> FFN (2)      v4: r,k,v+LN (1) -> wkv4 (1) -> Wo (1) -> FFN (2)
//   v7: r,k,v,LoRA-in+LN (1) -> LoRA-out (1) -> prep+wkv7+GN (1) -> Wo (1) -> FFN (2)
// Layers [l0, l1) (embedding when l0 == 0, head when l1 == n_layer and logits).
bool Engine::forward_decode(const float * sin, float * sout, bool logits, uint32_t l0, uint32_t l1) {
    const int C = (int)m_->n_embed, H = (int)m_->H, S = (int)m_->S;
    l1 = std::min(l1, m_->n_layer);
    // v6: layer 0's maa launch computes the embedding LayerNorm itself (k_v6_maa_dec4 EMB: the same
    // bits as k_embed_ln; one launch and one boundary less per token)
    MaaDec emaa;
    bool emb_in = false;
    if (l0 == 0 && l1 > 0 && m_->major == 6 && (fuse_ & FUSE_EMBMAA) && !split_maa_) {
        const DLayer & F = m_->layers[0];
        const ActBuf o0[5] = {A(1, F.decay_w1), A(2, F.att_k), A(3, F.att_v), A(4, F.att_r), A(5, F.att_g)};
        v6_maa_dec_args(emaa, C, m_->maa_D, F.maa_w1, x_, sin + C, sout + C, F.ln1_w, F.ln1_b, F.maa_x, F.maa_w2t,
                        F.maa, o0);
        emaa.tok = dtokens_;
        emaa.emb = m_->emb;
        emaa.ln0w = m_->ln0_w;
        emaa.ln0b = m_->ln0_b;
        emaa.xout = x_;
        emb_in = v6_maa_emb_supported(emaa);
    }
    // v4: the same inside layer 0's fused attention launch (with Wo fused: the Wo rows store x)
    bool emb4_in = false;
    if (l0 == 0 && l1 > 0 && m_->major == 4 && (fuse_ & FUSE_EMBMAA) && (fuse_ & FUSE_ATT4) && (fuse_ & FUSE_WO4)) {
        const DLayer & F = m_->layers[0];
        emb4_in = v4_att_fused_supported(C, F.att_r, F.att_k, F.att_v, A(0, F.att_o)) && F.att_o.type == F.att_r.type &&
                  C % 8 == 0 && (m_->emb.type == W_F16 || m_->emb.type == W_F32) && (int)m_->emb.K == C;
        emb_in = emb4_in;
    }
    if (l0 == 0 && !emb_in && !launch_embed_ln(stream_, dtokens_, 1, m_->emb, m_->ln0_w, m_->ln0_b, x_)) return false;
    v7_fused_lora_ = false;
    const size_t per_layer = m_->major >= 5 ? (size_t)C * (2 + (size_t)S) : 5 * (size_t)C;
    bool maa_done = false;  // this layer's maa ran in the previous layer's channel-mix launch (k_sig_maa)
    for (uint32_t l = l0; l < l1; l++) {
        const DLayer & L = m_->layers[l];
        const float * si = sin + l * per_layer;
        float * so = sout + l * per_layer;
        // Wo matvec: input emitted by the attention kernel in Wo's format when heads are
        // whole 32-blocks, else read as fp32 by its own prologue
        MV c_wo;
        auto att_out = [&](auto & a, MV & wo, const DMat & Wo) {
            MVEntry & e = wo.add(Wo, x_, EPI_ADD);
            a.yq.fmt = -1;
            a.y = y_;
            if (S >= 32) {
                a.yq = A(6, Wo);
                e.src = SRC_ACT;
                e.act = a.yq;
            } else {
                src_f32(e, y_);
            }
            return true;
        };
        // ---------------- time mixing ----------------
        if (m_->major == 4) {
            ActBuf o = A(0, L.att_o);
            if ((fuse_ & FUSE_ATT4) && v4_att_fused_supported(C, L.att_r, L.att_k, L.att_v, o)) {
                // LN + r, k, v rows + WKV-4 in one launch, 8 channels per workgroup (mv_att4f.hip)
                if (timing_) {
                    kt_bytes_ = 3 * wbytes(L.att_r) + 9.0 * C * 4 + 6.0 * C * 4 + C * 4.0 + act_bytes(o, 1);
                    kt_flops_ = 6.0 * C * C;
                }
                V4WoFused wf;
                memset(&wf, 0, sizeof(wf));
                const bool wo_in = (fuse_ & FUSE_WO4) && L.att_o.type == L.att_r.type && C % 8 == 0;
                if (wo_in && emb4_in && l == 0) {
                    wf.tok = dtokens_;
                    wf.emb = m_->emb;
                    wf.ln0w = m_->ln0_w;
                    wf.ln0b = m_->ln0_b;
                    if (timing_) kt_bytes_ += (double)C * (m_->emb.type == W_F16 ? 2 : 4) + 2.0 * C * 4;
                }
                if (wo_in) {
                    wf.wo = L.att_o;
                    wf.xres = x_;
                    wf.ygran = ygran_;
                    wf.ytag = (unsigned)(l + 1) | ((unsigned)(cur_ + 1) << 16);
                    wf.err = herr_d_;
                    wf.spin_max = spin_max_;
                    if (timing_) {
                        kt_bytes_ += wbytes(L.att_o) + 2.0 * C * 8 + 2.0 * C * 4;
                        kt_flops_ += 2.0 * C * C;
                    }
                }
                if (!launch_v4_att_fused(stream_, C, L.att_r, L.att_k, L.att_v, x_, si + C, so + C, L.ln1_w, L.ln1_b,
                                         L.att_mix_r, L.att_mix_k, L.att_mix_v, L.att_first, L.att_decay, si, so, o, y_,
                                         wo_in ? &wf : nullptr))
                    return false;
                if (wo_in) goto v4_att_done;
                {
                    // y fp32: Wo quantizes it in its own prologue (the same Q8 bits as the emission)
                    MV c;
                    src_f32(c.add(L.att_o, x_, EPI_ADD), y_);
                    if (!mv(c.g)) return false;
                    goto v4_att_done;
                }
            } else {
                MV b;
                src_lnmix(b.add(L.att_r, r_, EPI_SIGMOID), x_, si + C, L.ln1_w, L.ln1_b, L.att_mix_r, 0, so + C);
                src_lnmix(b.add(L.att_k, k_, EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, L.att_mix_k, 0);
                src_lnmix(b.add(L.att_v, v_, EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, L.att_mix_v, 0);
                if (!mv(b.g)) return false;
                if (!launch_wkv4(stream_, 1, C, r_, k_, v_, L.att_first, L.att_decay, si, so, o)) return false;
            }
            {
                MV c;
                MVEntry & e = c.add(L.att_o, x_, EPI_ADD);
                e.src = SRC_ACT;
                e.act = o;
                if (!mv(c.g)) return false;
            }
        v4_att_done:;
        } else if (m_->major == 5) {
            const bool v52 = m_->minor >= 2;
            MV b;
            src_lnmix(b.add(L.att_r, r_, EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, L.att_mix_r, 0, so + C);
            src_lnmix(b.add(L.att_k, k_, EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, L.att_mix_k, 0);
            src_lnmix(b.add(L.att_v, v_, EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, L.att_mix_v, 0);
            if (v52) src_lnmix(b.add(L.att_g, g_, EPI_SILU), x_, si + C, L.ln1_w, L.ln1_b, L.att_mix_g, 0);
            if (!mv(b.g)) return false;
            Att6Dec a;
            memset(&a, 0, sizeof(a));
            a.H = H;
            a.S = S;
            a.r = r_;
            a.k = k_;
            a.v = v_;
            a.g = v52 ? g_ : nullptr;
            a.u = L.att_u;
            a.w = L.att_w;
            a.sin = si + 2 * C;
            a.sout = so + 2 * C;
            a.lnx_w = L.att_lnx_w;
            a.lnx_b = L.att_lnx_b;
            a.eps = 1e-5f;
            if (!att_out(a, c_wo, L.att_o)) return false;
            if (!launch_att6_dec(stream_, a)) return false;
            if (!mv(c_wo.g)) return false;
        } else if (m_->major == 6) {
            const int D = m_->maa_D;
            ActBuf outs[5] = {A(1, L.decay_w1), A(2, L.att_k), A(3, L.att_v), A(4, L.att_r), A(5, L.att_g)};
            if (maa_done) {
                maa_done = false;
            } else if (emb_in && l == 0) {
                if (timing_) {
                    // + the embedding row, LN0 vectors and x written
                    kt_bytes_ = wbytes(L.maa_w1) + 5.0 * D * C * 4 + 11.0 * C * 4 + C * 4.0 + 5 * act_bytes(outs[0], 1) +
                                (double)C * (m_->emb.type == W_F16 ? 2 : 4) + 3.0 * C * 4;
                    kt_flops_ = 2.0 * L.maa_w1.M * L.maa_w1.K + 2.0 * 5 * D * C;
                }
                if (!launch_v6_maa_dec_emb(stream_, emaa)) return false;
            } else if (v6_maa_dec_supported(C, D, L.maa_w1.type) && !split_maa_) {
                // W1 rows + mix in one launch (mv_maa.hip)
                if (timing_) {
                    // W1, W2 (fp32), x / carry / LN / maa vectors in, carry and 5 Q8 mixes out
                    kt_bytes_ = wbytes(L.maa_w1) + 5.0 * D * C * 4 + 11.0 * C * 4 + C * 4.0 + 5 * act_bytes(outs[0], 1);
                    kt_flops_ = 2.0 * L.maa_w1.M * L.maa_w1.K + 2.0 * 5 * D * C;
                }
                if (!launch_v6_maa_dec(stream_, C, D, L.maa_w1, x_, si + C, so + C, L.ln1_w, L.ln1_b, L.maa_x,
                                       L.maa_w2t, L.maa, outs))
                    return false;
            } else {
                MV b;
                src_lnmix(b.add(L.maa_w1, lora_, EPI_TANH), x_, si + C, L.ln1_w, L.ln1_b, L.maa_x, 1, so + C);
                if (!mv(b.g)) return false;
                if (!launch_v6_mix5_dec(stream_, C, D, so + C, si + C, lora_, L.maa_w2t, L.maa, outs))
                    return false;
            }
            const int mats[5] = {3, 1, 2, 4, 0};  // r, k, v, g, w
            float * ys[5] = {r_, k_, v_, g_, dsmall_[0]};
            const DMat * Ws[5] = {&L.att_r, &L.att_k, &L.att_v, &L.att_g, &L.decay_w1};
            const int epis[5] = {EPI_STORE, EPI_STORE, EPI_STORE, EPI_SILU, EPI_TANH};
            Att6Dec a;
            memset(&a, 0, sizeof(a));
            a.H = H;
            a.S = S;
            a.r = r_;
            a.k = k_;
            a.v = v_;
            a.g = g_;
            a.u = L.att_u;
            a.w = nullptr;
            a.wd2 = L.decay_w2;
            a.dl = dsmall_[0];
            a.decay = L.decay6;
            a.sin = si + 2 * C;
            a.sout = so + 2 * C;
            a.lnx_w = L.att_lnx_w;
            a.lnx_b = L.att_lnx_b;
            a.eps = 64e-5f;
            if (!att_out(a, c_wo, L.att_o)) return false;
            // r, k, v, g, Wd1 rows and the per-head attention in one launch (mv_att6f.hip), else
            // the k_mva group + k_att6_dec pair (the same bits)
            Att6Fused f;
            memset(&f, 0, sizeof(f));
            f.H = H;
            f.C = C;
            f.D = L.decay_w1.M;
            for (int i = 0; i < 4; i++) {
                f.W[i] = *Ws[i];
                f.x[i] = outs[mats[i]];
            }
            f.wd1 = L.decay_w1;
            f.xw = outs[mats[4]];
            f.att = a;
            f.gran = hgran_;
            f.err = herr_d_;
            f.spin_max = spin_max_;
            f.skip_wg = dbg_skip_gran_;
            // Wo inside the same launch (the head outputs handed to the non-reducer workgroups as
            // granules tagged by layer and state parity); else Wo is its own k_mva launch below
            bool wo_in = false;
            if ((fuse_ & FUSE_WO6) && (fuse_ & FUSE_ATT6)) {
                f.wo = L.att_o;
                f.xres = x_;
                f.ygran = ygran_;
                f.ytag = (unsigned)(l + 1) | ((unsigned)(cur_ + 1) << 16);
                f.wo_rows = wo_rows_;
                f.wo_prepoll = wo_prepoll_;
                wo_in = v6_att_fused_supported(f);
                if (!wo_in) {
                    memset(&f.wo, 0, sizeof(f.wo));
                    f.xres = nullptr;
                    f.ygran = nullptr;
                }
            }
            if ((fuse_ & FUSE_ATT6) && v6_att_fused_supported(f)) {
                if (timing_) {
                    // r, k, v, g, Wd1, Wd2 weights, their 5 Q8 inputs, the head state in and out,
                    // u / decay / ln_x vectors, r / k / v / g / dl written (sc1) and read back, Wo's input out
                    kt_bytes_ = 4 * wbytes(L.att_r) + wbytes(L.decay_w1) + wbytes(L.decay_w2) + 5 * act_bytes(outs[0], 1) +
                                2.0 * H * S * S * 4 + 4.0 * C * 4 + 2.0 * (4.0 * C + f.D) * 4 + act_bytes(a.yq, 1);
                    kt_flops_ = 2.0 * (4.0 * C + f.D) * C + 2.0 * C * f.D;
                    if (wo_in) {
                        // Wo weights, the y granules (Q8 blocks) written and gathered, x read and written
                        kt_bytes_ += wbytes(L.att_o) + 2.0 * KG_STRIDE * (C / 32) * 8 + 2.0 * C * 4 - act_bytes(a.yq, 1);
                        kt_flops_ += 2.0 * C * C;
                    }
                }
                // the co-resident layout when this context has the device to itself (choose_co)
                if (co_ && v6_att_co_supported(f) ? !launch_v6_att_co(stream_, f) : !launch_v6_att_fused(stream_, f))
                    return false;
            } else {
                MV c;
                for (int i = 0; i < 5; i++) {
                    MVEntry & e = c.add(*Ws[i], ys[i], epis[i]);
                    e.src = SRC_ACT;
                    e.act = outs[mats[i]];
                }
                if (!mv(c.g)) return false;
                if (!launch_att6_dec(stream_, a)) return false;
            }
            if (!wo_in && !mv(c_wo.g)) return false;
        } else {
            // v7, order r, w, k, v, a, g of x_rwkvag (rwkv_graph.inc:404-413)
            MV b;
            const float * mu = L.x_rwkvag;
            src_lnmix(b.add(L.att_r, r_, EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, mu, 1, so + C);
            src_lnmix(b.add(L.att_k, k_, EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, mu + 2 * (size_t)C, 1);
            src_lnmix(b.add(L.att_v, v_, EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, mu + 3 * (size_t)C, 1);
            // the LoRA first stages (F16 in the released files) as their own launch when their type
            // differs from r,k,v: one weight type per launch keeps the fixed-type kernels (fewer
            // registers, no per-entry type switch, no padded units)
            MV lb;
            MV & bl = L.w1.type == L.att_r.type ? b : lb;
            src_lnmix(bl.add(L.w1, dsmall_[0], EPI_TANH), x_, si + C, L.ln1_w, L.ln1_b, mu + 1 * (size_t)C, 1);
            src_lnmix(bl.add(L.a1, dsmall_[1], EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, mu + 4 * (size_t)C, 1);
            src_lnmix(bl.add(L.g1, dsmall_[2], EPI_SIGMOID), x_, si + C, L.ln1_w, L.ln1_b, mu + 5 * (size_t)C, 1);
            if (l != 0) src_lnmix(bl.add(L.v1, dsmall_[3], EPI_STORE), x_, si + C, L.ln1_w, L.ln1_b, mu + 3 * (size_t)C, 1);
            if (!mv(b.g)) return false;
            if (lb.g.n && !mv(lb.g)) return false;
            if (l == 0) HIP_OK(hipMemcpyAsync(vfirst_, v_, (size_t)C * 4, hipMemcpyDeviceToDevice, stream_));
            Att7Dec a;
            memset(&a, 0, sizeof(a));
            a.H = H;
            a.S = S;
            a.r = r_;
            a.w = w_;
            a.k = k_;
            a.v = v_;
            a.a = a_;
            a.g = g_;
            a.k_k = L.k_k;
            a.k_a = L.k_a;
            a.r_k = L.r_k;
            a.sin = si + 2 * C;
            a.sout = so + 2 * C;
            a.lnx_w = L.att_lnx_w;
            a.lnx_b = L.att_lnx_b;
            if (!att_out(a, c_wo, L.att_o)) return false;
            // LoRA second stages + attention in one launch (mv_att7f.hip), else the LoRA-out matvec
            // group + k_att7_dec (the same bits)
            Att7Lora f;
            memset(&f, 0, sizeof(f));
            f.att = a;
            f.W2[0] = L.w2;
            f.W2[1] = L.a2;
            f.W2[2] = L.g2;
            f.W2[3] = L.v2;
            for (int i = 0; i < 4; i++) f.lin[i] = dsmall_[i];
            f.bias[0] = L.w0;
            f.bias[1] = L.a0;
            f.bias[2] = nullptr;
            f.bias[3] = L.v0;
            f.vfirst = vfirst_;
            f.has_v = l != 0;
            if ((fuse_ & FUSE_ATT7) && att7_lora_supported(f)) {
                if (timing_) {
                    double lb = wbytes(L.w2) + wbytes(L.a2) + wbytes(L.g2) + (l ? wbytes(L.v2) : 0.0);
                    kt_bytes_ = lb + 2.0 * H * S * S * 4 + 12.0 * C * 4 + act_bytes(a.yq, 1);
                    kt_flops_ = 2.0 * (L.w2.K + L.a2.K + L.g2.K + (l ? L.v2.K : 0)) * C;
                }
                if (!launch_att7_lora(stream_, f)) return false;
                v7_fused_lora_ = true;  // w, a, g and the mixed v never leave the launch (debug_copy)
            } else {
                MV c;
                src_f32(c.add(L.w2, w_, EPI_DECAY7, nullptr, L.w0), dsmall_[0]);
                src_f32(c.add(L.a2, a_, EPI_SIGMOID_BIAS, nullptr, L.a0), dsmall_[1]);
                src_f32(c.add(L.g2, g_, EPI_STORE), dsmall_[2]);
                if (l != 0) src_f32(c.add(L.v2, v_, EPI_VMIX7, vfirst_, L.v0), dsmall_[3]);
                if (!mv(c.g)) return false;
                if (!launch_att7_dec(stream_, a)) return false;
            }
            if (!mv(c_wo.g)) return false;
        }
        // ---------------- channel mixing ----------------
        if (m_->major == 7) {
            ActBuf kin = A(0, L.ffn_v);
            const bool ffco7 = co_ && (fuse_ & FUSE_FFNCO);
            if ((fuse_ & FUSE_FFN) || ffco7) {
                FfnFused ff;
                memset(&ff, 0, sizeof(ff));
                ff.co = ffco7;
                MVEntry & fk = ff.e[0];
                fk.W = L.ffn_k;
                fk.epi = EPI_RELU_SQ;
                src_lnmix(fk, x_, si, L.ln2_w, L.ln2_b, L.ffn_x_k, 1, so);
                fk.emit = 1;
                fk.act_out = kin;
                ff.wv = L.ffn_v;
                ff.x = x_;
                ff.kg = kgran_;
                ff.tag = (unsigned)(l + 1) | ((unsigned)(cur_ + 1) << 16);
                ff.err = herr_d_;
                ff.spin_max = spin_max_;
                ff.wdelay = ffn_wdelay_ >= 0 ? ffn_wdelay_ : (int)std::min(2000.0, wbytes(L.ffn_k) / 4e4);
                ff.prepoll = ffn_prepoll_;
                if (ff.co && !ffn_fused_supported(ff, 1, false)) ff.co = 0;  // the ordered form, if on
                if ((ff.co || (fuse_ & FUSE_FFN)) && ffn_fused_supported(ff, 1, false)) {
                    if (timing_) {
                        kt_bytes_ = wbytes(L.ffn_k) + wbytes(L.ffn_v) + 5.0 * C * 4 + 2.0 * C * 4 +
                                    (double)L.ffn_k.M / 32 * KG_STRIDE * 8 * 2;
                        kt_flops_ = 2.0 * ((double)L.ffn_k.M * L.ffn_k.K + (double)L.ffn_v.M * L.ffn_v.K);
                    }
                    if (!launch_ffn_fused(stream_, ff, 1, false)) return false;
                    continue;
                }
            }
            MV b;
            MVEntry & ek = b.add(L.ffn_k, nullptr, EPI_RELU_SQ);
            src_lnmix(ek, x_, si, L.ln2_w, L.ln2_b, L.ffn_x_k, 1, so);
            ek.emit = 1;
            ek.act_out = kin;
            if (!mv(b.g)) return false;
            MV c;
            MVEntry & ev = c.add(L.ffn_v, x_, EPI_ADD);
            ev.src = SRC_ACT;
            ev.act = kin;
            if (!mv(c.g)) return false;
        } else {
            const int form = m_->major == 6 ? 1 : 0;
            const float * muk = m_->major == 6 ? L.ffn_maa_k : L.ffn_mix_k;
            const float * mur = m_->major == 6 ? L.ffn_maa_r : L.ffn_mix_r;
            MV b;
            ActBuf kin = A(0, L.ffn_v);
            MVEntry & ek = b.add(L.ffn_k, nullptr, EPI_RELU_SQ);
            src_lnmix(ek, x_, si, L.ln2_w, L.ln2_b, muk, form, so);
            ek.emit = 1;
            ek.act_out = kin;
            // the receptance rows go with the value rows (k_mvsig) when the key launch can emit
            // their input: one launch of 224 workgroups for the key instead of 288 for key +
            // receptance (more workgroups than CUs), and fr_ never leaves the wave
            MVEntry sv, sr;
            memset(&sv, 0, sizeof(sv));
            memset(&sr, 0, sizeof(sr));
            sv.W = L.ffn_v;
            sv.src = SRC_ACT;
            sv.act = kin;
            sv.y = x_;
            sv.epi = EPI_SIGMUL_ADD;
            sr.W = L.ffn_r;
            sr.src = SRC_ACT;
            sr.act = A(7, L.ffn_r);
            sr.epi = EPI_STORE;
            // the whole channel mix in one launch (mv_ffnf.hpp), else the key group + k_mvsig
            const bool ffco = co_ && (fuse_ & FUSE_FFNCO);
            if ((fuse_ & FUSE_FFN) || ffco) {
                FfnFused ff;
                memset(&ff, 0, sizeof(ff));
                ff.co = ffco;
                MVEntry & fk = ff.e[0];
                fk.W = L.ffn_k;
                fk.epi = EPI_RELU_SQ;
                src_lnmix(fk, x_, si, L.ln2_w, L.ln2_b, muk, form, so);
                fk.emit = 1;
                fk.act_out = kin;
                MVEntry & fr = ff.e[1];
                fr.W = L.ffn_r;
                fr.epi = EPI_STORE;
                src_lnmix(fr, x_, si, L.ln2_w, L.ln2_b, mur, form);
                ff.wv = L.ffn_v;
                ff.x = x_;
                ff.kg = kgran_;
                ff.rg = rgran_;
                ff.tag = (unsigned)(l + 1) | ((unsigned)(cur_ + 1) << 16);
                ff.err = herr_d_;
                ff.spin_max = spin_max_;
                ff.wdelay = ffn_wdelay_ >= 0 ? ffn_wdelay_ : (int)std::min(2000.0, (wbytes(L.ffn_k) + wbytes(L.ffn_r)) / 4e4);
                ff.prepoll = ffn_prepoll_;
                if (ff.co && !ffn_fused_supported(ff, form, true)) ff.co = 0;  // the ordered form, if on
                if ((ff.co || (fuse_ & FUSE_FFN)) && ffn_fused_supported(ff, form, true)) {
                    if (timing_) {
                        kt_bytes_ = wbytes(L.ffn_k) + wbytes(L.ffn_r) + wbytes(L.ffn_v) + 5.0 * C * 4 + 2.0 * C * 4 +
                                    (double)L.ffn_k.M / 32 * KG_STRIDE * 8 * 2 + 2.0 * C * 8 + C * 4.0;
                        kt_flops_ = 2.0 * ((double)L.ffn_k.M * L.ffn_k.K + (double)L.ffn_r.M * L.ffn_r.K +
                                           (double)L.ffn_v.M * L.ffn_v.K);
                    }
                    if (!launch_ffn_fused(stream_, ff, form, true)) return false;
                    continue;
                }
            }
            const bool sig = (fuse_ & FUSE_SIG) && L.ffn_r.type == L.ffn_k.type && mv_sigmul_supported(sv, sr);
            if (sig) {
                ek.mu2 = mur;
                ek.act2_out = sr.act;
            } else {
                src_lnmix(b.add(L.ffn_r, fr_, EPI_STORE), x_, si, L.ln2_w, L.ln2_b, mur, form);
            }
            if (!mv(b.g)) return false;
            // co-resident: the next layer's maa in this launch (mv_sigmaa.hip), its x from granules
            bool sm_in = false;
            if (sig && co_ && (fuse_ & FUSE_SIGMAA) && m_->major == 6 && l + 1 < l1 && !split_maa_) {
                const DLayer & N = m_->layers[l + 1];
                const float * si1 = sin + (l + 1) * per_layer;
                float * so1 = sout + (l + 1) * per_layer;
                const ActBuf outs1[5] = {A(1, N.decay_w1), A(2, N.att_k), A(3, N.att_v), A(4, N.att_r), A(5, N.att_g)};
                SigMaa sm;
                memset(&sm, 0, sizeof(sm));
                mv_fill_hot(sv, sm.hv);
                mv_fill_hot(sr, sm.hr);
                sm.wtype = L.ffn_v.type;
                v6_maa_dec_args(sm.maa, C, m_->maa_D, N.maa_w1, x_, si1 + C, so1 + C, N.ln1_w, N.ln1_b, N.maa_x,
                                N.maa_w2t, N.maa, outs1);
                sm.nm = 5 * (C / 64);
                sm.xg = xgran_;
                sm.xtag = (unsigned)(l + 1) | ((unsigned)(cur_ + 1) << 16);
                sm.err = herr_d_;
                sm.spin_max = spin_max_;
                if (sig_maa_supported(sm)) {
                    if (timing_) {
                        // + the maa's W1, W2 (fp32), LayerNorm vectors, carry and mixes; x granules out / in
                        kt_bytes_ = wbytes(L.ffn_v) + wbytes(L.ffn_r) + act_bytes(kin, 1) + act_bytes(sr.act, 1) +
                                    2.0 * C * 4 + wbytes(N.maa_w1) + 5.0 * m_->maa_D * C * 4 + 11.0 * C * 4 +
                                    5 * act_bytes(outs1[0], 1) + 2.0 * C * 8;
                        kt_flops_ = 2.0 * ((double)L.ffn_v.M * L.ffn_v.K + (double)L.ffn_r.M * L.ffn_r.K) +
                                    2.0 * N.maa_w1.M * N.maa_w1.K + 2.0 * 5 * m_->maa_D * C;
                    }
                    if (!launch_sig_maa(stream_, sm)) return false;
                    sm_in = maa_done = true;
                }
            }
            if (sm_in) {
            } else if (sig) {
                if (timing_) {
                    kt_bytes_ = wbytes(L.ffn_v) + wbytes(L.ffn_r) + act_bytes(kin, 1) + act_bytes(sr.act, 1) + 2.0 * C * 4;
                    kt_flops_ = 2.0 * ((double)L.ffn_v.M * L.ffn_v.K + (double)L.ffn_r.M * L.ffn_r.K);
                }
                if (!launch_mv_sigmul(stream_, sv, sr)) return false;
            } else {
                MV c;
                MVEntry & ev = c.add(L.ffn_v, x_, EPI_SIGMUL_ADD, fr_);
                ev.src = SRC_ACT;
                ev.act = kin;
                if (!mv(c.g)) return false;
            }
        }
    }
    if (logits && l1 == m_->n_layer) {
        MV h;
        src_lnmix(h.add(m_->head, logits_, EPI_STORE), x_, nullptr, m_->lnout_w, m_->lnout_b, nullptr, 2);
        if (!mv(h.g)) return false;
    }
    return true;
}

// Runs T tokens from dstate_[cur_] (ping-pong), chunked by the workspace capacity.
bool Engine::run_tokens(const uint32_t * tokens, size_t T, bool want_logits) {
    // a failed call restores the ping-pong parity it started with, so the next state upload
    // (every rwkv_eval with state_in, rwkv_mi355x_state_upload) lands where the next step reads;
    // the device state's contents after a failure are unspecified (re-upload it)
    const int cur0 = cur_;
    if (!run_tokens_impl(tokens, T, want_logits)) {
        (void)hipStreamSynchronize(stream_);
        // the call's tagged Wo-input granules must not satisfy a replay of the same parity
        (void)hipMemsetAsync(ygran_, 0, tgran_n_ * 8, stream_);
        (void)hipStreamSynchronize(stream_);
        release_device();
        cur_ = cur0;
        return false;
    }
    return true;
}

bool Engine::run_tokens_impl(const uint32_t * tokens, size_t T, bool want_logits) {
    const size_t kChunkMax = 1024;
    size_t done = 0;
    while (done < T) {
        const size_t n = std::min(T - done, kChunkMax);
        const bool last = done + n == T;
        if (!ensure_workspace((int)n)) return false;
        if (n == 1) {
            // one token: a CP write packet in stream order (no blit kernel, no pinned buffer)
            HIP_OK(hipStreamWriteValue32(stream_, dtokens_, tokens[done], 0));
        } else {
            // the pinned token buffer may still feed the previous (async) call's copy
            HIP_OK(hipEventSynchronize(tok_event_));
            memcpy(htokens_, tokens + done, n * 4);
            HIP_OK(hipMemcpyAsync(dtokens_, htokens_, n * 4, hipMemcpyHostToDevice, stream_));
            HIP_OK(hipEventRecord(tok_event_, stream_));
        }
        const bool lg = last && want_logits;
        last_decode_ = n == 1 && !generic_decode_;
        const bool co = last_decode_ ? choose_co() : (co_ = false);
        if (timing_) {
            // eager launches; a decode step's kernels each carry a dispatch-bound event pair
            // (RK_LAUNCH through g_klt), the sequence path's matmul groups an event pair around
            // the group (mm_launch)
            if (n == 1) g_klt = this;
            const bool ok = forward((int)n, dstate_[cur_], dstate_[cur_ ^ 1], lg);
            g_klt = nullptr;
            if (!ok) return false;
        } else if (n == 1 && use_graphs_) {
            hipGraphExec_t & ge = graphs_[co][cur_][lg ? 1 : 0];
            if (!ge) {
                hipGraph_t g = nullptr;
                HIP_OK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
                const bool ok = forward(1, dstate_[cur_], dstate_[cur_ ^ 1], lg);
                HIP_OK(hipStreamEndCapture(stream_, &g));
                if (!ok) {
                    (void)hipGraphDestroy(g);
                    return false;
                }
                HIP_OK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                (void)hipGraphDestroy(g);
            }
            HIP_OK(hipGraphLaunch(ge, stream_));
        } else {
            if (!forward((int)n, dstate_[cur_], dstate_[cur_ ^ 1], lg)) return false;
        }
        // The fused decode's Wo granules are tagged (layer, state parity) and never cleared by their
        // readers.  A step that did not run the fused decode flips the parity without writing them,
        // so the next decode would run at the parity of the decode before this step and could take
        // a value that step left (one-layer engines: the same layer tag).  Clear them in stream order.
        if (n > 1 || generic_decode_) {
            HIP_OK(hipMemsetAsync(ygran_, 0, tgran_n_ * 8, stream_));
        }
        // tokens buffer is reused by the next chunk: wait before overwriting the pinned copy
        if (!last) HIP_OK(hipStreamSynchronize(stream_));
        cur_ ^= 1;
        done += n;
    }
    return true;
}

bool Engine::state_upload(const float * state) {
    if (state) {
        HIP_OK(hipMemcpyAsync(dstate_[cur_], state, m_->state_len * 4, hipMemcpyHostToDevice, stream_));
        io_h2d_ += m_->state_len * 4.0;
        return true;
    }
    return init_state(dstate_[cur_]);
}

bool Engine::state_download(float * state) {
    HIP_OK(hipMemcpyAsync(state, dstate_[cur_], m_->state_len * 4, hipMemcpyDeviceToHost, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
    io_d2h_ += m_->state_len * 4.0;
    return handoff_check();
}

// The host layout is per layer contiguous (rwkv_graph.inc:545-606), so layers [l0, l1) are one
// range of the device-resident state: only that range crosses PCIe.
bool Engine::state_upload_layers(const float * slice, uint32_t l0, uint32_t l1) {
    const size_t per = layer_state_len(), off = (size_t)l0 * per, n = (size_t)(l1 - l0) * per;
    if (slice) {
        HIP_OK(hipMemcpyAsync(dstate_[cur_] + off, slice, n * 4, hipMemcpyHostToDevice, stream_));
        io_h2d_ += n * 4.0;
        return true;
    }
    return init_state(dstate_[cur_] + off, n);
}

bool Engine::state_download_layers(float * slice, uint32_t l0, uint32_t l1) {
    const size_t per = layer_state_len(), off = (size_t)l0 * per, n = (size_t)(l1 - l0) * per;
    HIP_OK(hipMemcpyAsync(slice, dstate_[cur_] + off, n * 4, hipMemcpyDeviceToHost, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
    io_d2h_ += n * 4.0;
    return handoff_check();
}

bool Engine::sync() {
    HIP_OK(hipStreamSynchronize(stream_));
    return handoff_check();
}

// k_v6_att_fused's reducer gives up after spin_max_ sweep passes and sets the host-mapped flag
// (mv_att6f.hip).  Every call that synchronises the stream reads it: a set flag fails that call
// (the reference's error convention: false + RWKV_ERROR_CTX, rwkv_error_handling.inc:1-54).  A
// producer that arrives after the timeout leaves its granule tagged, which the next launch would
// read as its own value, so every granule is cleared before the flag is re-armed.
bool Engine::handoff_check() {
    // called after the stream has drained: nothing of this context is queued any more
    release_device();
    const bool co_seen = co_pending_ > 0;
    co_pending_ = 0;
    if (*(volatile unsigned *)herr_h_ == 0) return true;
    (void)hipStreamSynchronize(stream_);
    (void)hipMemsetAsync(hgran_, 0, hgran_n_ * 8, stream_);
    (void)hipMemsetAsync(ygran_, 0, tgran_n_ * 8, stream_);
    (void)hipStreamSynchronize(stream_);
    *(volatile unsigned *)herr_h_ = 0;
    if (co_seen && co_knob_ < 0) {
        // the co-resident layout lost its co-residency (another process's launches on the device):
        // this context uses the ordered layout from now on; a synchronous one-token call re-runs
        co_ok_ = false;
        co_retry_ = true;
        fprintf(stderr, "rwkv: in-launch hand-off timed out in the co-resident attention layout; using the ordered layout\n");
    } else {
        fprintf(stderr, "rwkv: in-launch hand-off timed out: the evaluation's results are invalid\n");
    }
    return false;
}

bool Engine::debug_set(const char * name, long long value) {
    if (!name) return false;
    const std::string n(name);
    // "delay_us": a kernel that holds the context's stream for value us, enqueued now (no sync) --
    // the timing pass puts one ahead of each eager decode step, so the host queues the step's
    // launches before the GPU reaches them and they run back to back, as in a graph replay (and as
    // under a profiler, whose slower launches would otherwise leave the GPU idle between kernels)
    if (n == "delay_us") return value > 0 && value <= 100000 && launch_delay(stream_, (int)value);
    if (n == "skip_granule") dbg_skip_gran_ = (int)value;
    else if (n == "spin_max") spin_max_ = value > 0 ? (unsigned)std::min<long long>(value, 0xffffffffLL) : (1u << 20);
    else if (n == "wkv_chunk") wkv_chunk_ = value != 0;
    else if (n == "generic_decode") generic_decode_ = value != 0 || m_->n_embed > 4096;
    else if (n == "graphs") use_graphs_ = value != 0;
    else if (n == "co_mode" && value >= -1 && value <= 1) co_knob_ = (int)value;
    else if (n == "decode_fusion")  // -1: the default for this model
        fuse_ = value < 0 ? FUSE_DEFAULT | (m_->major == 4 ? FUSE_FFNCO : 0u) : (unsigned)value & FUSE_ALL;
    else if (n == "wo_rows" && (value == 4 || value == 8)) wo_rows_ = (int)value;
    else if (n == "wo_prepoll") wo_prepoll_ = value != 0;
    else if (n == "ffn_wdelay" && value >= -1 && value <= 10000) ffn_wdelay_ = (int)value;
    else if (n == "ffn_prepoll") ffn_prepoll_ = value != 0;
    else return false;
    // the decode graphs captured the old values; a decode program without the fused Wo flips the
    // state parity without writing the Wo granules (see run_tokens_impl): clear them
    (void)hipStreamSynchronize(stream_);
    drop_graphs();
    drop_io_graphs();
    (void)hipMemsetAsync(ygran_, 0, tgran_n_ * 8, stream_);
    (void)hipStreamSynchronize(stream_);
    return true;
}

// ---------------------------------------------------------------- ABI decode with host state
// rwkv_eval's contract hands the whole recurrent state over as host buffers on every call
// (rwkv_eval.inc:2-22): 13 MB each way for v6-1B6, ~0.5 ms of PCIe against a 0.82 ms decode.
// The decode runs as io_chunk_-layer graphs instead of one, so the copies of one chunk's state
// slice overlap the other chunks' kernels: the host uploads chunk c+1 (copy stream 0) while the
// GPU runs chunk c, and downloads chunk c-1 (copy stream 1) while the GPU runs chunk c.  This
// works for ordinary pageable buffers too: a pageable hipMemcpyAsync holds the HOST until its
// bytes are staged, but the chunk graphs are already queued, so the GPU keeps computing.  The
// bytes moved and every result are exactly those of the one-graph path.
// Both caller state buffers page-locked (registered with / allocated by the HIP runtime)?  NULL
// buffers count as page-locked (no copy).
static bool host_pinned(const void * p) {
    if (!p) return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

bool Engine::pinned_io(const float * state_in, const float * state_out) {
    return host_pinned(state_in) && host_pinned(state_out);
}

bool Engine::eval_host_chunked(uint32_t token, const float * state_in, float * state_out, float * logits_out) {
    const uint32_t NL = m_->n_layer, K = (uint32_t)io_chunk_, NC = (NL + K - 1) / K;
    const size_t C = m_->n_embed, per_layer = m_->major >= 5 ? C * (2 + (size_t)m_->S) : 5 * C;
    if (!ensure_workspace(1)) return false;
    if (!io_stream_[0]) {
        // copy streams (high-priority queues and CU-masked download queues measured no better)
        HIP_OK(hipStreamCreateWithFlags(&io_stream_[0], hipStreamNonBlocking));
        HIP_OK(hipStreamCreateWithFlags(&io_stream_[1], hipStreamNonBlocking));
        HIP_OK(hipEventCreateWithFlags(&io_entry_ev_, hipEventDisableTiming));
    }
    // the copy streams start behind everything already queued on stream_ (an earlier
    // rwkv_mi355x_eval_device(sync = false) may still be writing dstate_[cur_], the upload target)
    HIP_OK(hipEventRecord(io_entry_ev_, stream_));
    for (auto & st : io_stream_) HIP_OK(hipStreamWaitEvent(st, io_entry_ev_, 0));
    if (io_ev_.size() < 2 * (size_t)NC) {
        for (hipEvent_t e : io_ev_) (void)hipEventDestroy(e);
        io_ev_.assign(2 * NC, nullptr);
        for (auto & e : io_ev_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    const bool lg = logits_out != nullptr;
    const bool co = choose_co();
    std::vector<hipGraphExec_t> & gs = io_graphs_[co][cur_][lg ? 1 : 0];
    if (gs.size() != NC) {
        for (hipGraphExec_t g : gs)
            if (g) (void)hipGraphExecDestroy(g);
        gs.assign(NC, nullptr);
    }
    float * din = dstate_[cur_], * dout = dstate_[cur_ ^ 1];
    for (uint32_t c = 0; c < NC; c++) {
        if (gs[c]) continue;
        hipGraph_t g = nullptr;
        HIP_OK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
        const bool ok = forward_decode(din, dout, lg, c * K, (c + 1) * K);
        HIP_OK(hipStreamEndCapture(stream_, &g));
        if (!ok) {
            (void)hipGraphDestroy(g);
            return false;
        }
        HIP_OK(hipGraphInstantiate(&gs[c], g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
    }
    auto slice = [&](uint32_t c, size_t & off, size_t & bytes) {
        const uint32_t l0 = c * K, l1 = std::min(NL, l0 + K);
        off = l0 * per_layer;
        bytes = (l1 - l0) * per_layer * 4;
    };
    hipEvent_t * in_ev = io_ev_.data(), * done_ev = io_ev_.data() + NC;
    size_t off, bytes;
    HIP_OK(hipStreamWriteValue32(stream_, dtokens_, token, 0));
    last_decode_ = true;
    if (!state_in && !init_state(din)) return false;
    auto upload = [&](uint32_t c) -> bool {
        slice(c, off, bytes);
        HIP_OK(hipMemcpyAsync(din + off, state_in + off, bytes, hipMemcpyHostToDevice, io_stream_[0]));
        HIP_OK(hipEventRecord(in_ev[c], io_stream_[0]));
        io_h2d_ += (double)bytes;
        return true;
    };
    auto download = [&](uint32_t c) -> bool {
        slice(c, off, bytes);
        HIP_OK(hipStreamWaitEvent(io_stream_[1], done_ev[c], 0));
        HIP_OK(hipMemcpyAsync(state_out + off, dout + off, bytes, hipMemcpyDeviceToHost, io_stream_[1]));
        io_d2h_ += (double)bytes;
        return true;
    };
    auto launch = [&](uint32_t c) -> bool {
        if (state_in) HIP_OK(hipStreamWaitEvent(stream_, in_ev[c], 0));
        HIP_OK(hipGraphLaunch(gs[c], stream_));
        HIP_OK(hipEventRecord(done_ev[c], stream_));
        return true;
    };
    // Page-locked caller buffers: every copy call returns at once, so all uploads are queued first
    // (they only read din, which no chunk graph writes), then the graphs, then the downloads.  A
    // rocprofv3 memory-copy trace of the interleaved order showed each upload starting only when
    // the previous chunk's kernels ended: the download call issued between them held the host
    // until its chunk had finished.  Pageable buffers: a copy call returns once the runtime has
    // staged the bytes, so the interleaved order keeps the GPU fed; downloads lag two chunks.
    if (pinned_io(state_in, state_out)) {
        for (uint32_t c = 0; state_in && c < NC; c++)
            if (!upload(c)) return false;
        for (uint32_t c = 0; c < NC; c++)
            if (!launch(c)) return false;
        for (uint32_t c = 0; state_out && c < NC; c++)
            if (!download(c)) return false;
    } else {
        if (state_in && !upload(0)) return false;
        for (uint32_t c = 0; c < NC; c++) {
            if (!launch(c)) return false;
            if (state_in && c + 1 < NC && !upload(c + 1)) return false;
            if (state_out && c >= 2 && !download(c - 2)) return false;
        }
        for (uint32_t c = NC >= 2 ? NC - 2 : 0; state_out && c < NC; c++)
            if (!download(c)) return false;
    }
    if (logits_out)
        HIP_OK(hipMemcpyAsync(logits_out, logits_, (size_t)m_->n_vocab * 4, hipMemcpyDeviceToHost, stream_));
    HIP_OK(hipStreamSynchronize(io_stream_[1]));
    HIP_OK(hipStreamSynchronize(io_stream_[0]));
    HIP_OK(hipStreamSynchronize(stream_));
    if (!handoff_check()) return false;
    cur_ ^= 1;
    return true;
}

void Engine::drop_io_graphs() {
    for (auto & pc : io_graphs_)
        for (auto & p : pc)
            for (auto & v : p) {
                for (hipGraphExec_t g : v)
                    if (g) (void)hipGraphExecDestroy(g);
                v.clear();
            }
}

bool Engine::eval(const uint32_t * tokens, size_t T, const float * state_in, float * state_out, float * logits_out) {
    co_retry_ = false;
    const int pend0 = co_pending_;
    if (eval_once(tokens, T, state_in, state_out, logits_out)) return true;
    // a co-resident layout timeout in this call's own launches (none of an earlier asynchronous
    // call was pending): the inputs are untouched (host state_in, or the device state this call
    // started from), so the call runs again, in the ordered layout
    if (!co_retry_ || pend0 > 0) return false;
    co_retry_ = false;
    return eval_once(tokens, T, state_in, state_out, logits_out);
}

bool Engine::eval_once(const uint32_t * tokens, size_t T, const float * state_in, float * state_out, float * logits_out) {
    HIP_OK(hipSetDevice(m_->device));
    // one token with host state: chunked decode, copies overlapped (needs graphs; timing and the
    // generic decode path keep the whole-state copies)
    if (T == 1 && io_pipeline_ && use_graphs_ && !timing_ && !generic_decode_ && (state_in || state_out)) {
        const int cur0 = cur_;
        if (eval_host_chunked(tokens[0], state_in, state_out, logits_out)) return true;
        (void)hipStreamSynchronize(stream_);
        cur_ = cur0;
        return false;
    }
    if (!state_upload(state_in)) return false;
    const int cur0 = cur_;
    if (!run_tokens(tokens, T, logits_out != nullptr)) return false;
    if (logits_out)
        HIP_OK(hipMemcpyAsync(logits_out, logits_, (size_t)m_->n_vocab * 4, hipMemcpyDeviceToHost, stream_));
    if (state_out) {
        HIP_OK(hipMemcpyAsync(state_out, dstate_[cur_], m_->state_len * 4, hipMemcpyDeviceToHost, stream_));
        io_d2h_ += m_->state_len * 4.0;
    }
    HIP_OK(hipStreamSynchronize(stream_));
    if (!handoff_check()) {
        cur_ = cur0;
        return false;
    }
    return true;
}

// One layer-pipeline stage step on the device-resident state: x_io / vfirst_io
// are device buffers [T][C] on this engine's device carrying the residual stream (and v7's
// layer-0 values) between stages.  Synchronous: on return x_io holds this stage's output.
bool Engine::eval_layers(const uint32_t * tokens, size_t T, uint32_t l0, uint32_t l1, float * x_io, float * vfirst_io,
                         bool want_logits, float * logits_out, bool sync) {
    HIP_OK(hipSetDevice(m_->device));
    co_ = false;  // pipeline stages: the ordered layouts only
    if (!ensure_workspace((int)T)) return false;
    const size_t bytes = T * (size_t)m_->n_embed * 4;
    if (l0 == 0) {
        HIP_OK(hipEventSynchronize(tok_event_));
        memcpy(htokens_, tokens, T * 4);
        HIP_OK(hipMemcpyAsync(dtokens_, htokens_, T * 4, hipMemcpyHostToDevice, stream_));
        HIP_OK(hipEventRecord(tok_event_, stream_));
    } else {
        HIP_OK(hipMemcpyAsync(x_, x_io, bytes, hipMemcpyDeviceToDevice, stream_));
        if (m_->major == 7) HIP_OK(hipMemcpyAsync(vfirst_, vfirst_io, bytes, hipMemcpyDeviceToDevice, stream_));
    }
    const bool lg = (want_logits || logits_out) && l1 == m_->n_layer;
    if (!forward_range((int)T, dstate_[cur_], dstate_[cur_ ^ 1], l0, l1, lg)) return false;
    // only this range's slices were written: copy them back instead of flipping the ping-pong
    // pair, so later calls on other ranges still read a complete current state
    const size_t C = m_->n_embed, per_layer = m_->major >= 5 ? C * (2 + (size_t)m_->S) : 5 * C;
    HIP_OK(hipMemcpyAsync(dstate_[cur_] + l0 * per_layer, dstate_[cur_ ^ 1] + l0 * per_layer,
                          (size_t)(l1 - l0) * per_layer * 4, hipMemcpyDeviceToDevice, stream_));
    if (x_io) HIP_OK(hipMemcpyAsync(x_io, x_, bytes, hipMemcpyDeviceToDevice, stream_));
    if (vfirst_io && m_->major == 7) HIP_OK(hipMemcpyAsync(vfirst_io, vfirst_, bytes, hipMemcpyDeviceToDevice, stream_));
    if (lg && logits_out)
        HIP_OK(hipMemcpyAsync(logits_out, logits_, (size_t)m_->n_vocab * 4, hipMemcpyDeviceToHost, stream_));
    if (sync) {
        HIP_OK(hipStreamSynchronize(stream_));
        return handoff_check();
    }
    return true;  // async: the caller orders on stream() (pipeline.py) and synchronises (sync())
}

// Names: x xa sx r k v g w y a nb bb vfirst fr lora bonus logits, slot<i>.<q|d|s|qsum|h|f>.
// Returns -1 for an unknown name, a buffer that is not allocated, or more bytes than it holds.
long long Engine::debug_copy(const char * name, void * out, size_t bytes) {
    if (!name || !out) return -1;
    const std::string n(name);
    const void * src = nullptr;
    size_t cap_bytes = 0;
    const size_t cap = (size_t)tcap_, C = m_->n_embed;
    const size_t kmax = std::max<size_t>((size_t)m_->kmax, C);
    const std::pair<const char *, float *> fb[] = {{"x", x_}, {"xa", xa_}, {"sx", sx_}, {"r", r_}, {"k", k_},
        {"v", v_}, {"g", g_}, {"w", w_}, {"y", y_}, {"a", a_}, {"nb", nb_}, {"bb", bb_}, {"vfirst", vfirst_},
        {"fr", fr_}};
    for (const auto & p : fb)
        if (n == p.first) src = p.second, cap_bytes = cap * C * 4;
    // the fused v7 decode (k_att7_lora) keeps w, a, g and the mixed v in LDS: those buffers hold
    // another evaluation's values, so they are refused rather than returned stale
    if (last_decode_ && v7_fused_lora_ && (n == "w" || n == "a" || n == "g" || n == "v")) return -1;
    if (n == "lora") src = lora_, cap_bytes = cap * kmax * 4;
    if (n == "bonus") src = bonus_, cap_bytes = cap * (size_t)std::max<int64_t>(1, m_->H) * 4;
    if (n == "logits") src = logits_, cap_bytes = (size_t)m_->n_vocab * 4;
    if (n == "granules") src = hgran_, cap_bytes = 6 * C * 8;  // k_v6_att_fused hand-off granules
    if (!src && n.rfind("slot", 0) == 0) {
        const size_t dot = n.find('.');
        const int i = atoi(n.c_str() + 4);
        if (dot == std::string::npos || i < 0 || i >= kSlots) return -1;
        const std::string f = n.substr(dot + 1);
        const ActSlot & s = slots_[i];
        const size_t el = cap * kmax, nbk = el / 32 + 1;
        if (f == "q") src = s.q, cap_bytes = el;
        else if (f == "d") src = s.d, cap_bytes = nbk * 4;
        else if (f == "s") src = s.s, cap_bytes = nbk * 4;
        else if (f == "qsum") src = s.qsum, cap_bytes = nbk * 4;
        else if (f == "h") src = s.h, cap_bytes = el * 2;
        else if (f == "f") src = s.f, cap_bytes = el * 4;
    }
    if (!src || bytes > cap_bytes) return -1;
    if (hipStreamSynchronize(stream_) != hipSuccess || hipMemcpy(out, src, bytes, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return (long long)bytes;
}

// ---------------------------------------------------------------- batched decode
// B independent contexts of this model advance one token each in one pass: the layer matmuls
// run the decode matvec kernel (k_mm) over the B activation rows, so every weight byte is read
// once per step for all B contexts, and each context's arithmetic is exactly its single-token
// decode (same lane/block association, same kernels' per-token math); token shift and the wkv
// recurrences take context t's state at t * state_len (LnMixArgs::bs, launch_wkv* bs).
// states: [B][state_len] contiguous.  dev: pointers are device memory (else host).
bool Engine::eval_batch(const uint32_t * tokens, size_t B, const float * state_in, float * state_out,
                        float * logits_out, bool dev) {
    HIP_OK(hipSetDevice(m_->device));
    co_ = false;  // batched decode: the ordered layouts only
    if (B == 0) return true;
    if (B > (size_t)kBatchMax) {
        fprintf(stderr, "rwkv: batched decode takes at most %d contexts (got %zu)\n", kBatchMax, B);
        return false;
    }
    if (!ensure_workspace((int)B)) return false;
    const size_t n = m_->state_len, V = m_->n_vocab;
    if (B > bcap_) {
        HIP_OK(hipStreamSynchronize(stream_));
        drop_batch_graphs();
        for (float *& p : bstate_) {
            if (p) (void)hipFree(p);
            p = nullptr;
        }
        if (blogits_) (void)hipFree(blogits_);
        blogits_ = nullptr;
        bcap_ = 0;
        size_t cap = 1;
        while (cap < B) cap *= 2;
        bool ok = true;
        for (float *& p : bstate_) ok = ok && hipMalloc(&p, cap * n * 4 + 64) == hipSuccess;
        ok = ok && hipMalloc(&blogits_, cap * V * 4 + 64) == hipSuccess;
        if (!ok) {
            (void)hipGetLastError();
            for (float *& p : bstate_) {
                if (p) (void)hipFree(p);
                p = nullptr;
            }
            if (blogits_) (void)hipFree(blogits_);
            blogits_ = nullptr;
            fprintf(stderr, "rwkv: batched decode state allocation for %zu contexts failed\n", B);
            return false;
        }
        bcap_ = cap;
    }
    // tokens: pinned copy in stream order (the previous call's copy may still read it)
    HIP_OK(hipEventSynchronize(tok_event_));
    memcpy(htokens_, tokens, B * 4);
    HIP_OK(hipMemcpyAsync(dtokens_, htokens_, B * 4, hipMemcpyHostToDevice, stream_));
    HIP_OK(hipEventRecord(tok_event_, stream_));
    // input states: device pointer as given, else staged into bstate_[0] (NULL = fresh states)
    const float * sin = state_in;
    if (!state_in) {
        RK_LAUNCH(k_init_state, dim3((unsigned)((B * n + 255) / 256)), dim3(256), 0, stream_, bstate_[0],
                           B * n, (int)m_->n_embed, m_->major == 4 ? 1 : 0);
        HIP_OK(hipGetLastError());
        sin = bstate_[0];
    } else if (!dev) {
        HIP_OK(hipMemcpyAsync(bstate_[0], state_in, B * n * 4, hipMemcpyHostToDevice, stream_));
        sin = bstate_[0];
    }
    float * sout = (dev && state_out) ? state_out : bstate_[1];
    float * lout = (dev && logits_out) ? logits_out : blogits_;
    const bool lg = logits_out != nullptr;
    bool ok;
    if (use_graphs_ && !timing_) {
        // one graph per (B, state pointers, logits pointer): a decode loop alternating two state
        // buffers replays two graphs
        hipGraphExec_t ge = nullptr;
        for (const BatchGraph & g : bgraphs_)
            if (g.B == B && g.sin == sin && g.sout == sout && g.lout == (lg ? lout : nullptr)) ge = g.ge;
        if (!ge) {
            // first step with these buffers: run it eagerly (lazy GEMM scratch allocations happen
            // here, outside any capture), then capture the graph the next steps replay
            bs_ = n;
            head_out_ = lout;
            ok = forward_range((int)B, sin, sout, 0, m_->n_layer, lg);
            bs_ = 0;
            head_out_ = nullptr;
            if (!ok) {
                (void)hipStreamSynchronize(stream_);
                return false;
            }
            if (bgraphs_.size() >= 8) drop_batch_graphs();
            hipGraph_t g = nullptr;
            HIP_OK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
            bs_ = n;
            head_out_ = lout;
            ok = forward_range((int)B, sin, sout, 0, m_->n_layer, lg);
            bs_ = 0;
            head_out_ = nullptr;
            HIP_OK(hipStreamEndCapture(stream_, &g));
            if (!ok) {
                (void)hipGraphDestroy(g);
                return false;
            }
            HIP_OK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            (void)hipGraphDestroy(g);
            bgraphs_.push_back(BatchGraph{B, sin, sout, lg ? lout : nullptr, ge});
        } else {
            HIP_OK(hipGraphLaunch(ge, stream_));
        }
        ok = true;
    } else {
        bs_ = n;
        head_out_ = lout;
        ok = forward_range((int)B, sin, sout, 0, m_->n_layer, lg);
        bs_ = 0;
        head_out_ = nullptr;
    }
    if (!ok) {
        (void)hipStreamSynchronize(stream_);
        return false;
    }
    if (!dev) {
        if (logits_out) HIP_OK(hipMemcpyAsync(logits_out, lout, B * V * 4, hipMemcpyDeviceToHost, stream_));
        if (state_out) HIP_OK(hipMemcpyAsync(state_out, sout, B * n * 4, hipMemcpyDeviceToHost, stream_));
        HIP_OK(hipStreamSynchronize(stream_));
        return handoff_check();
    }
    return true;
}

void Engine::drop_batch_graphs() {
    for (BatchGraph & g : bgraphs_) (void)hipGraphExecDestroy(g.ge);
    bgraphs_.clear();
}

bool Engine::eval_device(const uint32_t * tokens, size_t T, bool want_logits, float * logits_out, bool sync_after) {
    HIP_OK(hipSetDevice(m_->device));
    const int cur0 = cur_, pend0 = co_pending_;
    co_retry_ = false;
    for (int attempt = 0;; attempt++) {
        if (!run_tokens(tokens, T, want_logits || logits_out != nullptr)) return false;
        if (logits_out)
            HIP_OK(hipMemcpyAsync(logits_out, logits_, (size_t)m_->n_vocab * 4, hipMemcpyDeviceToHost, stream_));
        if (!(sync_after || logits_out)) return true;
        HIP_OK(hipStreamSynchronize(stream_));
        if (handoff_check()) return true;
        // a co-resident layout timeout in this one-token call (an earlier asynchronous call's
        // timeout cannot be re-run: its state has moved on): run the token again from the state it
        // started from, in the ordered layout
        if (!co_retry_ || pend0 > 0 || attempt > 0 || T != 1 || cur_ != (cur0 ^ 1)) return false;
        co_retry_ = false;
        cur_ = cur0;
    }
}

}  // namespace rwkvmi
