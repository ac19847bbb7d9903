/*
 * rwkv_mi355x.h -- ADDITIVE extensions of librwkv.so (nothing in rwkv.h changes).
 *
 * The reference ABI hands the recurrent state over as host float buffers on every call
 * (rwkv_eval.inc:2-22).  For RWKV-v6-1B6 that is 13 MB each way per token, more than the
 * weights' HBM time, so these entry points let a caller keep the state resident in HBM.
 * They are the path bench.py measures as "device-resident"; ABI-level rates are reported
 * beside them.
 */
#ifndef RWKV_MI355X_H
#define RWKV_MI355X_H

#include "rwkv.h"

#if defined(__cplusplus)
extern "C" {
#endif

/* Copies a host state into the context's device-resident state (NULL => fresh state). */
RWKV_API bool rwkv_mi355x_state_upload(struct rwkv_context * ctx, const float * state);
/* Copies the device-resident state out to host memory. */
RWKV_API bool rwkv_mi355x_state_download(struct rwkv_context * ctx, float * state);

/* The state of layers [layer_begin, layer_end) only: `slice` holds those layers in the host layout
 * (rwkv_mi355x_layer_state_len(ctx) floats per layer, layer_begin's first), so a pipeline stage or a
 * caller that owns part of the layers moves just its part over PCIe.  Upload with slice == NULL
 * resets those layers to the fresh state.  Layer ranges outside [0, n_layer) fail with
 * RWKV_ERROR_ARGS. */
RWKV_API size_t rwkv_mi355x_layer_state_len(const struct rwkv_context * ctx);
RWKV_API bool rwkv_mi355x_state_upload_layers(struct rwkv_context * ctx, const float * slice, uint32_t layer_begin,
                                              uint32_t layer_end);
RWKV_API bool rwkv_mi355x_state_download_layers(struct rwkv_context * ctx, float * slice, uint32_t layer_begin,
                                                uint32_t layer_end);
/* State bytes this context has moved so far: out[0] host->device, out[1] device->host (the state
 * entry points above and rwkv_eval's host state buffers). */
RWKV_API void rwkv_mi355x_state_io_bytes(const struct rwkv_context * ctx, double out[2]);

/* rwkv_clone_context onto GPU `device` (reference clone semantics, rwkv.h:93-99, rwkv.cpp:123-139:
 * a new context with a fresh state sharing the parent's model).  The model is uploaded once per
 * GPU -- the first clone on a GPU re-reads the parent's file (same layer range), later clones and
 * their parent-device siblings share that copy -- so a server runs one replica per GPU of a node
 * from one process.  device == the parent's GPU is rwkv_clone_context.  A device outside
 * [0, device count) fails with RWKV_ERROR_ARGS (on the parent's error flags) and returns NULL. */
RWKV_API struct rwkv_context * rwkv_mi355x_clone_context_on(struct rwkv_context * ctx, uint32_t n_threads,
                                                            int device);
/* The GPU a context evaluates on (-1 for NULL). */
RWKV_API int rwkv_mi355x_context_device(const struct rwkv_context * ctx);

/* rwkv_eval_sequence semantics on the device-resident state: tokens host array, T >= 1.
 * compute_logits: run the head on the last token (logits stay in HBM); logits_out (host, may be
 * NULL) additionally receives them.  No state crosses PCIe.  sync=false returns after
 * enqueueing (the caller later calls rwkv_mi355x_sync). */
RWKV_API bool rwkv_mi355x_eval_device(struct rwkv_context * ctx, const uint32_t * tokens, size_t T,
                                      bool compute_logits, float * logits_out, bool sync);
RWKV_API bool rwkv_mi355x_sync(struct rwkv_context * ctx);

/* Debugging aid: copies `bytes` of the named workspace buffer of the last evaluation to host `out`
 * (names: x xa sx r k v g w y a nb bb vfirst fr lora bonus logits, slot<i>.<q|d|s|qsum|h|f>).
 * Returns the bytes copied, or -1 (unknown name / copy failure).  Not part of rwkv.h. */
RWKV_API long long rwkv_mi355x_debug_buffer(struct rwkv_context * ctx, const char * name, void * out, size_t bytes);
/* Test hooks (not part of rwkv.h): "skip_granule" = index of a k_v6_att_fused producer workgroup that
 * publishes nothing (-1: off), so the in-launch hand-off times out and the next synchronising call
 * fails with RWKV_ERROR_CTX; "spin_max" = the hand-off sweep bound in passes (<= 0: the default
 * 2^20).  Returns false for an unknown name or a NULL context. */
RWKV_API bool rwkv_mi355x_debug_set(struct rwkv_context * ctx, const char * name, long long value);

/* One stage of the layer pipeline (the reference has no such entry point -- it is
 * the unit the multi-GPU sequence evaluation is built from, rwkv.cppy_amd/python/rwkv_cpp/pipeline.py).
 * Runs layers [layer_begin, layer_end) over T tokens on the device-resident state; only those
 * layers' state slices change.  x_dev / vfirst_dev: device buffers [T][n_embed] fp32 on the
 * context's GPU with the residual stream (and, v7 only, the layer-0 values v_first) entering
 * layer_begin; on return they hold the ones leaving layer_end - 1.  layer_begin == 0 embeds
 * `tokens` instead of reading x_dev (which may then be NULL).  When layer_end == n_layer and
 * compute_logits, the head runs on the last token (logits_out host, may be NULL).  Synchronous.
 * The same tensors, chunked along T, give results bit-identical to rwkv_eval_sequence. */
RWKV_API bool rwkv_mi355x_eval_layers(struct rwkv_context * ctx, const uint32_t * tokens, size_t T,
                                      uint32_t layer_begin, uint32_t layer_end, float * x_dev, float * vfirst_dev,
                                      bool compute_logits, float * logits_out);

/* The same stage, enqueued on the context's stream (rwkv_mi355x_stream) without waiting for it:
 * the caller orders its own work (e.g. an RCCL send of x_dev) on that stream.  Logits, when
 * computed, stay on the device (rwkv_mi355x_logits_device). */
RWKV_API bool rwkv_mi355x_eval_layers_async(struct rwkv_context * ctx, const uint32_t * tokens, size_t T,
                                            uint32_t layer_begin, uint32_t layer_end, float * x_dev, float * vfirst_dev,
                                            bool compute_logits);
/* The context's device logits buffer [n_vocab] (NULL for a NULL context).  It holds valid logits
 * only after an evaluation that computed them: on the context holding the head (the last stage)
 * with compute_logits / a logits request; otherwise its contents are stale. */
RWKV_API float * rwkv_mi355x_logits_device(struct rwkv_context * ctx);

/* A pipeline stage's context: only layers [layer_begin, layer_end) are uploaded (plus the
 * embedding when layer_begin == 0 and the head when layer_end == n_layer), so a stage's HBM holds
 * ~1/P of the weights (reference placement by layer range: rwkv_model_loading.inc:128-142).  The
 * state keeps the full layout.  Whole-model calls (rwkv_eval, ...) fail with
 * RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED on such a context; rwkv_mi355x_eval_layers accepts
 * ranges inside [layer_begin, layer_end). */
RWKV_API struct rwkv_context * rwkv_mi355x_init_from_file_layers(const char * path, uint32_t n_threads,
                                                                 uint32_t layer_begin, uint32_t layer_end);

/* The layer pipeline behind the reference entry points: n_stages stage contexts in
 * this process, stage i on GPU devices[i] (NULL: i modulo the device count) holding the contiguous
 * layers [i*L/P .. (i+1)*L/P) (earlier stages take the extra layers; the embedding on stage 0, the
 * head on the last).  rwkv_eval / rwkv_eval_sequence[_in_chunks] on the returned context (stage 0)
 * run every stage: the sequence is cut into chunks of >= 256 tokens, chunk c's residual stream
 * (and v7's v_first) crosses from stage s to s+1 by a peer copy over xGMI while stage s starts
 * chunk c+1; results are bit-identical to a single-GPU context.  rwkv_clone_context clones the
 * pipeline (same stages and GPUs, weights shared).  The same context is what rwkv_init_from_file
 * returns when RWKV_MI355X_PIPELINE=P (P >= 2) is set (devices: RWKV_MI355X_PIPELINE_DEVICES, a
 * comma list).  Adjacent stages on different GPUs get peer access enabled at init (a GPU pair
 * without it fails the init).  rwkv_eval_sequence_in_chunks passes chunk_size to the pipeline as
 * its chunk (the results do not depend on it).  rwkv_mi355x_state_upload / _download / sync act on
 * every stage; the other device-resident entry points (eval_device, eval_batch*, stream,
 * device_state, clone_context_on) refuse a pipeline context with RWKV_ERROR_UNSUPPORTED. */
RWKV_API struct rwkv_context * rwkv_mi355x_init_pipeline(const char * path, uint32_t n_threads, int n_stages,
                                                         const int * devices);
/* Stages of a context: P for a pipeline context, 1 otherwise (0 for NULL). */
RWKV_API int rwkv_mi355x_pipeline_stages(const struct rwkv_context * ctx);
/* Adjacent stage pairs of a pipeline context that sit on different GPUs (their hop is a peer copy
 * over xGMI, peer access enabled at init); 0 when every stage shares one GPU or for a non-pipeline. */
RWKV_API int rwkv_mi355x_pipeline_peer_pairs(const struct rwkv_context * ctx);

/* Batched decode (multi-context serving): n_contexts independent sequences of this
 * model advance ONE token each in one pass -- the rwkv_eval of each context, with every weight byte
 * read once per step for all of them (the reference runs clones side by side instead:
 * rwkv_clone_context, rwkv.h:93-99, rwkv.cpp:123-139).  Results are bit-identical to
 * rwkv_eval(ctx, tokens[i], state_in + i * state_len, ...) for every i.
 * tokens: host [n_contexts]; state_in / state_out: [n_contexts][state_len] (state_in NULL = fresh
 * states, state_out NULL = not returned); logits_out: [n_contexts][logits_len] or NULL.
 * n_contexts <= 256.  Host buffers; synchronous. */
RWKV_API bool rwkv_mi355x_eval_batch(struct rwkv_context * ctx, const uint32_t * tokens, size_t n_contexts,
                                     const float * state_in, float * state_out, float * logits_out);
/* The same with state_in / state_out / logits_out in device memory of the context's GPU (no PCIe
 * traffic; state_in != state_out; NULL state_out / logits_out: kept in library buffers).
 * Enqueued on the context's stream (rwkv_mi355x_stream); returns without waiting. */
RWKV_API bool rwkv_mi355x_eval_batch_device(struct rwkv_context * ctx, const uint32_t * tokens, size_t n_contexts,
                                            const float * state_in, float * state_out, float * logits_out);

/* The context's HIP stream (hipStream_t), so callers can time kernels with events on it. */
RWKV_API void * rwkv_mi355x_stream(struct rwkv_context * ctx);

/* Device pointer of the current device-resident state (state_len floats). */
RWKV_API float * rwkv_mi355x_device_state(struct rwkv_context * ctx);

/* Per-token algorithmic HBM bytes of one decode step (weights read + state read/written),
 * counted from the original block sizes (Q4_0 18 B / 32 weights ...), see DESIGN.md. */
RWKV_API double rwkv_mi355x_decode_bytes(const struct rwkv_context * ctx, bool with_logits);

/* Algorithmic bytes of the model's weight matrices only (all layers, + head if asked). */
RWKV_API double rwkv_mi355x_weight_bytes(const struct rwkv_context * ctx, bool with_head);

/* 2*M*K summed over every matmul of one token (head included if asked). */
RWKV_API double rwkv_mi355x_matmul_flops_per_token(const struct rwkv_context * ctx, bool with_head);

/* Architecture info: out[0..3] = arch_major, arch_minor, head_count, head_size. */
RWKV_API void rwkv_mi355x_arch(const struct rwkv_context * ctx, int64_t out[4]);

/* Writes a synthetic rwkv.cpp model file with the exact tensor shapes of a real checkpoint,
 * seeded random weights (N(0, 1/sqrt(fan_in)) for matrices), quantized with this library's
 * quantizer.  arch: 4, 5 (v5.2), 6, 7.  fmt: "FP32" "FP16" "Q4_0" "Q4_1" "Q5_0" "Q5_1" "Q8_0".
 * ffn = 0 picks the architecture's default FFN width; head_size 64 for v5+; lora dims of
 * the real checkpoints.  Used by bench.py (no checkpoints are downloadable). */
RWKV_API bool rwkv_mi355x_write_synthetic_model(const char * path, int arch, uint32_t n_vocab,
                                                uint32_t n_embed, uint32_t n_layer, uint32_t ffn,
                                                const char * fmt, uint64_t seed);

/* Kernel timing: while on, every matmul launch on the context stream is bracketed by hipEvents
 * (decode runs eagerly, not from the captured graph) and accumulated per kernel class -- the
 * template instantiation name rocprofv3 reports, e.g. "k_mm<2, 2, 1>" (weight type, rows per
 * wave, columns per pass).  Turning it on clears the counters. */
RWKV_API void rwkv_mi355x_set_kernel_timing(struct rwkv_context * ctx, bool on);
/* Reads counter `index`; returns the number of kernel classes (call with index -1 to count).
 * total_bytes: algorithmic bytes (weights at original block sizes + activations in/out). */
RWKV_API int rwkv_mi355x_kernel_stats(struct rwkv_context * ctx, int index, char * name, size_t name_len,
                                      long long * launches, double * total_ms, double * total_bytes,
                                      double * total_flops);

/* ---- kernel self-tests (used by tests/ for per-kernel parity; not on the eval path) ----
 * Runs the library's activation quantizer (the emit stage every producer kernel uses) on
 * x [T][K] (host) for the activation format of weight type `wtype` (rwkv file type id) and
 * returns the int8 codes, fp16-rounded scales d and (Q8_1) s, as fp32.  q/d/s may be NULL. */
RWKV_API bool rwkv_mi355x_selftest_quantize_act(int wtype, const float * x, int T, int K, int8_t * q, float * d,
                                                float * s);
/* Runs the decode/sequence matmul kernel on W (ggml block bytes of type wtype, ne=[K, M],
 * host) and x [T][K] (host): y [T][M] = W x with the library's activation quantization. */
RWKV_API bool rwkv_mi355x_selftest_matmul(int wtype, const void * W, int K, int M, const float * x, int T, float * y);

// Self-test of the sequence GEMM: the same product as rwkv_mi355x_selftest_matmul computed by
// the int8-MFMA kernel (quantized weight types only; T >= 2).
RWKV_API bool rwkv_mi355x_selftest_gemm(int wtype, const void * W, int K, int M, const float * x, int T, float * y);
/* The same with the GEMM's split-K form forced: split 1 = one workgroup per tile, 4 / 8 = the class
 * tree in that many subtrees on as many workgroups plus the combine kernel (same bits). */
RWKV_API bool rwkv_mi355x_selftest_gemm_split(int wtype, const void * W, int K, int M, const float * x, int T,
                                              float * y, int split);

/* WKV-6 (v5 / v6 time mixing, head size 64) over T tokens of one context on host operands:
 * chunked = 0 runs the serial kernel (bit-exact with decode), 1 the chunk-parallel form
 * (RWKV_MI355X_WKV_CHUNK; re-associated sums).  k, v, r: [T][H*64]; w: [T][H*64] (w_per_token = 1,
 * v6) or [H*64] (v5); u: [H*64]; state_in / state_out: [H][64 key][64 value]; y: [T][H*64]. */
RWKV_API bool rwkv_mi355x_selftest_wkv6(int T, int H, int chunked, int w_per_token, const float * k, const float * v,
                                       const float * r, const float * u, const float * w, const float * state_in,
                                       float * state_out, float * y);

/* WKV-7 (v7 time mixing, head size 64) over T tokens of one context on host operands: chunked = 0 the
 * serial kernel (bit-exact with decode), 1 the chunk-parallel form (RWKV_MI355X_WKV_CHUNK; re-associated
 * sums).  r, w, k, v, a, b: [T][H*64] (a, b: the transition's rank-one factors, -kk and kk * a in
 * rwkv_operators_wkv_v7.inc:37-107); state_in / state_out: [H][64 value][64 key]; y: [T][H*64]. */
RWKV_API bool rwkv_mi355x_selftest_wkv7(int T, int H, int chunked, const float * r, const float * w, const float * k,
                                       const float * v, const float * a, const float * b, const float * state_in,
                                       float * state_out, float * y);

#if defined(__cplusplus)
}
#endif

#endif
