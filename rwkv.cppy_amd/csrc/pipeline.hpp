// pipeline.hpp -- layer pipeline over several stage engines in one process (pipeline.cpp).
#pragma once

#include <vector>

#include "engine.hpp"

namespace rwkvmi {

class LayerPipeline {
  public:
    struct StageSpec {
        Engine * eng;  // owns layers [l0, l1) on `device`
        int device;
        uint32_t l0, l1;
    };
    LayerPipeline() = default;
    ~LayerPipeline();
    bool init(const std::vector<StageSpec> & stages, size_t n_embed, bool v7);
    // rwkv_eval_sequence semantics over the stages: host tokens / state / logits (NULL allowed as in
    // the ABI); chunk = 0 picks max(256, T / 2P) rounded to 64 tokens
    bool eval(const uint32_t * tokens, size_t T, const float * state_in, float * state_out, float * logits_out,
              size_t layer_len, size_t chunk = 0);
    size_t stages() const { return st_.size(); }
    size_t pick_chunk(size_t T) const;
    int peer_pairs() const { return peer_pairs_; }  // adjacent stage pairs on different GPUs (peer access on)

  private:
    struct Stage {
        Engine * eng = nullptr;
        int device = 0;
        uint32_t l0 = 0, l1 = 0;
        float * xb[2] = {nullptr, nullptr};  // x of a chunk entering / leaving this stage
        float * vb[2] = {nullptr, nullptr};  // v7 v_first
        hipEvent_t ready[2] = {nullptr, nullptr};     // chunk forwarded to the next stage
        hipEvent_t consumed[2] = {nullptr, nullptr};  // this stage is done with buffer b
    };
    bool ensure_buffers(size_t chunk);
    bool eval_impl(const uint32_t * tokens, size_t T, const float * state_in, float * state_out, float * logits_out,
                   size_t layer_len, size_t chunk);
    void drain();
    int peer_pairs_ = 0;
    std::vector<Stage> st_;
    size_t C_ = 0, cap_ = 0;
    bool v7_ = false;
};

}  // namespace rwkvmi
