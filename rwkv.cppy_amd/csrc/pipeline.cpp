// pipeline.cpp -- the layer pipeline behind the C ABI (reference placement by layer
// range, rwkv_model_loading.inc:128-142).
//
// One process drives P stage engines, stage s owning the contiguous layers [l0_s, l1_s) and their
// state slice on its own GPU (all stages on one GPU is valid too: the tests run that way).  A
// sequence is cut into chunks along T; chunk c runs through stage 0, its residual stream x
// [T_c][C] fp32 (plus v7's layer-0 values v_first) goes to stage s+1 by a peer copy over xGMI
// (hipMemcpyPeerAsync on the producing stage's stream), and stage s+1 starts it after an event.
// Every stage takes its chunks in order -- the order the recurrence needs -- so the result is
// bit-identical to one rwkv_eval_sequence; different stages work on different chunks at once.
// Two staging buffers per stage alternate between chunks; a producer overwrites buffer b only
// after the consumer has read chunk c-2 from it (event).  The host enqueues everything without
// waiting except where the ABI hands results back (state slices, logits).
#include "pipeline.hpp"

#include <stdio.h>

#include <algorithm>

namespace rwkvmi {

LayerPipeline::~LayerPipeline() {
    for (Stage & s : st_) {
        (void)hipSetDevice(s.device);
        if (s.eng) (void)hipStreamSynchronize(s.eng->stream());
        for (int b = 0; b < 2; b++) {
            if (s.xb[b]) (void)hipFree(s.xb[b]);
            if (s.vb[b]) (void)hipFree(s.vb[b]);
            if (s.ready[b]) (void)hipEventDestroy(s.ready[b]);
            if (s.consumed[b]) (void)hipEventDestroy(s.consumed[b]);
        }
    }
}

bool LayerPipeline::init(const std::vector<StageSpec> & specs, size_t n_embed, bool v7) {
    C_ = n_embed;
    v7_ = v7;
    for (const StageSpec & sp : specs) {
        Stage s;
        s.eng = sp.eng;
        s.device = sp.device;
        s.l0 = sp.l0;
        s.l1 = sp.l1;
        st_.push_back(s);
    }
    for (Stage & s : st_) {
        HIP_OK(hipSetDevice(s.device));
        for (int b = 0; b < 2; b++) {
            HIP_OK(hipEventCreateWithFlags(&s.ready[b], hipEventDisableTiming));
            HIP_OK(hipEventCreateWithFlags(&s.consumed[b], hipEventDisableTiming));
        }
    }
    // The hop between adjacent stages on different GPUs is a peer copy issued on the producer's
    // stream: with peer access enabled both ways it is one DMA over xGMI; without it the runtime
    // would stage it through host memory, so a pair without peer access fails the init.
    for (size_t i = 0; i + 1 < st_.size(); i++) {
        const int a = st_[i].device, b = st_[i + 1].device;
        if (a == b) continue;
        int ab = 0, ba = 0;
        HIP_OK(hipDeviceCanAccessPeer(&ab, a, b));
        HIP_OK(hipDeviceCanAccessPeer(&ba, b, a));
        if (!ab || !ba) {
            fprintf(stderr, "rwkv: layer pipeline: GPUs %d and %d have no peer access (stages %zu, %zu)\n", a, b, i,
                    i + 1);
            return false;
        }
        for (int k = 0; k < 2; k++) {
            HIP_OK(hipSetDevice(k ? b : a));
            const hipError_t e = hipDeviceEnablePeerAccess(k ? a : b, 0);
            if (e == hipErrorPeerAccessAlreadyEnabled) {
                (void)hipGetLastError();
            } else if (e != hipSuccess) {
                fprintf(stderr, "rwkv: layer pipeline: enabling peer access %d -> %d failed: %s\n", k ? b : a, k ? a : b,
                        hipGetErrorString(e));
                return false;
            }
        }
        peer_pairs_++;
    }
    return true;
}

// Drains every stage stream (after an error: no copy or kernel of this call may still touch the
// staging buffers when the next call reuses or frees them).
void LayerPipeline::drain() {
    for (Stage & s : st_) {
        (void)hipSetDevice(s.device);
        (void)hipStreamSynchronize(s.eng->stream());
    }
}

bool LayerPipeline::ensure_buffers(size_t chunk) {
    if (chunk <= cap_) return true;
    for (Stage & s : st_) {
        HIP_OK(hipSetDevice(s.device));
        HIP_OK(hipStreamSynchronize(s.eng->stream()));
        for (int b = 0; b < 2; b++) {
            if (s.xb[b]) (void)hipFree(s.xb[b]);
            if (s.vb[b]) (void)hipFree(s.vb[b]);
            s.xb[b] = s.vb[b] = nullptr;
        }
    }
    cap_ = 0;
    for (Stage & s : st_) {
        HIP_OK(hipSetDevice(s.device));
        for (int b = 0; b < 2; b++) {
            HIP_OK(hipMalloc(&s.xb[b], chunk * C_ * 4 + 64));
            if (v7_) HIP_OK(hipMalloc(&s.vb[b], chunk * C_ * 4 + 64));
        }
    }
    cap_ = chunk;
    return true;
}

size_t LayerPipeline::pick_chunk(size_t T) const {
    // every stage call should keep its GEMMs on >= 256-token tiles; below that the MFMA GEMM is
    // mostly fixed cost (64-token chunks were the worst shape)
    const size_t P = st_.size();
    size_t c = (T + 2 * P - 1) / (2 * P);
    c = (c + 63) / 64 * 64;
    return std::min(T, std::max<size_t>(c, 256));
}

bool LayerPipeline::eval(const uint32_t * tokens, size_t T, const float * state_in, float * state_out,
                         float * logits_out, size_t layer_len, size_t chunk) {
    if (st_.empty() || T == 0) return false;
    if (!chunk) chunk = pick_chunk(T);
    chunk = std::min(chunk, T);
    if (!ensure_buffers(chunk)) return false;
    if (!eval_impl(tokens, T, state_in, state_out, logits_out, layer_len, chunk)) {
        drain();
        // a failure may have been an in-launch hand-off timeout: clear every stage's flag
        for (Stage & s : st_) {
            (void)hipSetDevice(s.device);
            (void)s.eng->handoff_check();
        }
        return false;
    }
    return true;
}

bool LayerPipeline::eval_impl(const uint32_t * tokens, size_t T, const float * state_in, float * state_out,
                              float * logits_out, size_t layer_len, size_t chunk) {
    const size_t P = st_.size();
    // state in: each stage uploads its own slice (NULL = fresh)
    for (Stage & s : st_) {
        HIP_OK(hipSetDevice(s.device));
        if (!s.eng->state_upload_layers(state_in ? state_in + (size_t)s.l0 * layer_len : nullptr, s.l0, s.l1))
            return false;
    }
    const size_t nc = (T + chunk - 1) / chunk;
    for (size_t c = 0; c < nc; c++) {
        const size_t a = c * chunk, n = std::min(chunk, T - a);
        const int b = (int)(c & 1);
        for (size_t i = 0; i < P; i++) {
            Stage & s = st_[i];
            HIP_OK(hipSetDevice(s.device));
            hipStream_t sst = s.eng->stream();
            if (i > 0) HIP_OK(hipStreamWaitEvent(sst, st_[i - 1].ready[b], 0));  // chunk c's input landed
            const bool last = i + 1 == P && c + 1 == nc;
            if (!s.eng->eval_layers(tokens + a, n, s.l0, s.l1, s.xb[b], v7_ ? s.vb[b] : nullptr, last && logits_out,
                                    last ? logits_out : nullptr, false))
                return false;
            if (i + 1 < P) {
                Stage & d = st_[i + 1];
                // the next stage's buffer b is free once it is done with chunk c - 2
                if (c >= 2) HIP_OK(hipStreamWaitEvent(sst, d.consumed[b], 0));
                HIP_OK(hipMemcpyPeerAsync(d.xb[b], d.device, s.xb[b], s.device, n * C_ * 4, sst));
                if (v7_) HIP_OK(hipMemcpyPeerAsync(d.vb[b], d.device, s.vb[b], s.device, n * C_ * 4, sst));
                HIP_OK(hipEventRecord(s.ready[b], sst));
            }
            // this stage is done with its buffer b (read, written and forwarded)
            HIP_OK(hipEventRecord(s.consumed[b], sst));
        }
    }
    // state out: each stage's slice (synchronous per stage); otherwise wait for every stage.  Both
    // read each stage's hand-off flag (Engine::handoff_check).
    bool ok = true;
    for (Stage & s : st_) {
        HIP_OK(hipSetDevice(s.device));
        if (state_out) ok = s.eng->state_download_layers(state_out + (size_t)s.l0 * layer_len, s.l0, s.l1) && ok;
        else ok = s.eng->sync() && ok;
    }
    return ok;
}

}  // namespace rwkvmi
