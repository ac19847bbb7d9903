/*
 * oracle.h -- CPU restatement of the rwkv.cpp eval path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker for the MI355X path.  Only tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it.
 * The product library (librwkv.so) never links or calls it.
 *
 * Pinning: see oracle.c header and DESIGN.md section "Oracle".
 */
#ifndef RWKV_ORACLE_H
#define RWKV_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* rwkv.cpp file-format type ids (rwkv_file_format.inc:5-24). */
enum oracle_type {
    OT_FP32 = 0, OT_FP16 = 1, OT_Q4_0 = 2, OT_Q4_1 = 3,
    OT_Q5_0 = 7, OT_Q5_1 = 8, OT_Q8_0 = 9, OT_Q8_1 = 10
};

typedef struct oracle_model oracle_model;

/* Loads an rwkv.cpp model file.  Returns NULL on error (message on stderr). */
oracle_model * oracle_load(const char * path);
void oracle_free(oracle_model * m);

/* out[0..7] = n_vocab, n_embed, n_layer, arch_major, arch_minor, head_count, head_size, state_len */
void oracle_info(const oracle_model * m, int64_t out[8]);

/* rwkv_init_state semantics (rwkv_eval.inc:224-241). */
void oracle_init_state(const oracle_model * m, float * state);

/* rwkv_eval_sequence semantics for T >= 1 (rwkv_eval.inc:38-155):
 * state_in NULL => fresh state; state_out / logits_out NULL => skipped.
 * state_in may alias state_out.  Returns 0 on success. */
int oracle_eval(const oracle_model * m, const uint32_t * tokens, size_t T,
                const float * state_in, float * state_out, float * logits_out);

/* Layers [l0, l1) only (a layer-pipeline stage): x_io / vfirst_io [T][C] carry the residual
 * stream (and v7's layer-0 values) in and out; l0 == 0 embeds the tokens instead.  Only the
 * state slices of those layers change; logits when l1 == n_layer.  Returns 0 on success. */
int oracle_eval_layers(const oracle_model * m, const uint32_t * tokens, size_t T, uint32_t l0, uint32_t l1,
                       float * x_io, float * vfirst_io, const float * state_in, float * state_out,
                       float * logits_out);

/* rwkv_quantize_model_file semantics (rwkv_quantize.inc:16-171).  0 on success. */
int oracle_quantize_file(const char * in_path, const char * out_path, const char * format);

/* 0: ggml-mirror numerics (default).  Bits 1, 2, 4: re-associated reductions (noise-floor
 * probes).  Bit 8 (ORACLE_VARIANT_GPU): the MI355X kernels' association and their exp/tanh, which
 * the GPU path reproduces bit for bit (oracle.c "GPU-association variant"). */
#define ORACLE_VARIANT_GPU 8
void oracle_set_variant(int v);

/* The kernels' exp / tanh restated (device_common.hpp rk_expf / rk_tanhf). */
float oracle_gpu_expf(float x);
float oracle_gpu_tanhf(float x);

/* Number of OpenMP threads used by the matmuls (<=0: library default). */
void oracle_set_threads(int n);
int  oracle_get_threads(void);

/* ---- primitives, exported for kernel-level parity tests ---- */
/* Bytes per 32-element block of a type (34 for Q8_0, 36 for Q8_1, ...); 0 for FP32/FP16. */
size_t oracle_block_bytes(int type);
/* File quantizer (ggml quantize_row_*_ref restatement): k floats -> k/32 blocks. */
void oracle_quantize_row(int type, const float * x, void * dst, int64_t k);
/* Activation quantizer used inside the quantized matmul: Q8_0 or Q8_1. */
void oracle_quantize_act(int type, const float * x, void * dst, int64_t k);
/* Dequantize one row of k elements of any supported weight type into fp32. */
void oracle_dequantize_row(int type, const void * src, float * dst, int64_t k);
/* y[t*M + m] = sum_k W[m,k] * x[t*K + k] with ggml CPU matmul numerics. */
void oracle_matmul(int wtype, const void * W, int64_t K, int64_t M,
                   const float * x, int64_t T, float * y);
uint16_t oracle_f32_to_f16(float f);
float    oracle_f16_to_f32(uint16_t h);

#ifdef __cplusplus
}
#endif

#endif
