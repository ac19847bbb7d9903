// common.hpp -- shared types for the MI355X (gfx950) RWKV eval engine.
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//   * quantized weights are repacked at load time into structure-of-arrays:
//       qs  [M][nb][16]   (Q4_0/Q4_1/Q5_0/Q5_1: 16 nibble bytes per 32-block;
//                          low nibble of byte j = element j, high = element j+16 --
//                          the ggml block order, rwkv_graph.inc's mul_mat operand)
//       qs  [M][nb][32]   (Q8_0 int8)
//       qh  [M][nb] u32   (Q5_*: bit j = 5th bit of element j)
//       sc  [M][nb] u16   (_0 formats: fp16 d)  /  u32 (_1 formats: fp16 d | fp16 m << 16)
//     so every lane load is a 16-byte aligned dwordx4 and the algorithmic bytes per block
//     stay 18/20/22/24/34 (ggml block sizes).
//   * F16 / F32 matrices stay row-major [M][K].
//   * activations feeding a matmul are produced directly in the consumer's input format
//     (ActBuf): fp32, fp16, or Q8 blocks (int8 [T][K] + fp32 d/s + int qsum [T][K/32]),
//     mirroring ggml's src1 conversion (vec_dot_type) in rwkv_graph.inc's ggml_mul_mat calls.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stddef.h>

namespace rwkvmi {

// rwkv.cpp file type ids (reference rwkv_file_format.inc:5-24)
enum WType : int { W_F32 = 0, W_F16 = 1, W_Q4_0 = 2, W_Q4_1 = 3, W_Q5_0 = 7, W_Q5_1 = 8, W_Q8_0 = 9 };

// activation formats (ggml vec_dot_type of the consuming weight type)
enum AFmt : int { A_F32 = 0, A_F16 = 1, A_Q8_0 = 2, A_Q8_1 = 3 };

__host__ __device__ inline int act_fmt_for(int wtype) {
    switch (wtype) {
        case W_F32: return A_F32;
        case W_F16: return A_F16;
        case W_Q4_1:
        case W_Q5_1: return A_Q8_1;
        default: return A_Q8_0;
    }
}

inline bool wtype_quantized(int t) { return t == W_Q4_0 || t == W_Q4_1 || t == W_Q5_0 || t == W_Q5_1 || t == W_Q8_0; }

// Activation buffer: T rows of K elements in one format.
struct ActBuf {
    int fmt;
    int K;
    float * f;       // [T][K]       A_F32
    __half * h;      // [T][K]       A_F16
    int8_t * q;      // [T][K]       A_Q8_*
    float * d;       // [T][K/32]    fp16-rounded block scale, stored as fp32
    float * s;       // [T][K/32]    A_Q8_1: fp16-rounded d*sum(q)
    int * qsum;      // [T][K/32]    sum(q) (exact, used for the -8/-16 offset of _0 formats)
    // Sequence-GEMM layout (tiled != 0): Q8 blocks are written as token-tile records into tq
    // instead of q/d/s/qsum (qg_* below); only the int8-MFMA GEMM reads it.
    uint8_t * tq = nullptr;
    int tiled = 0;
};

// --------------------------------------------------------------------------- sequence-GEMM tiles
// Records the int8-MFMA GEMM (qgemm.hip) copies global->LDS as whole, contiguous pieces:
//   weights     per (row tile of qg_rows rows, block b), ordered [row tile][b]:
//                 [rows x 32 int8 (the block's integer weights, offset applied: q-8 / q-16 for
//                  _0, q for _1, 5th bit merged)][rows x f32 d] (the fp16 scales widened exactly,
//                  so the GEMM epilogue needs no conversion); the _1 formats' mins m go to DMat::mt
//                  ([block][row] f32), read by the m*s chain kernel (qgemm.hip k_qg_msum)
//   activations per (QG_TOK-token tile, block b), ordered [token tile][b]:
//                 [2 halves x QG_TOK tokens x 16 B int8][QG_TOK x f32 d][Q8_1: QG_TOK x f32 s]
constexpr int QG_TOK = 64;
// Row r's 32 int8 weights sit at byte r * 32 of the weight record with their two 16-byte halves
// swapped when bit 3 of r is set: the GEMM's 8-byte fragment reads (lane = row r16 of a 16-row
// tile, 8-byte piece h) then hit 32 distinct LDS banks per 32-lane group instead of rows r and
// r + 8 sharing banks (2-way conflicts on every read, 49% of LDS cycles in the PMC profile).
__host__ __device__ constexpr int qg_w_off(int r, int byte) { return r * 32 + (byte ^ (((r >> 3) & 1) << 4)); }
__host__ __device__ constexpr bool qg_one(int wt) { return wt == W_Q4_1 || wt == W_Q5_1; }
__host__ __device__ constexpr int qg_rows(int) { return 64; }
__host__ __device__ constexpr int qg_w_d(int wt) { return qg_rows(wt) * 32; }
__host__ __device__ constexpr int qg_w_bytes(int wt) { return qg_w_d(wt) + qg_rows(wt) * 4; }
// DMat::mt row stride (rows padded with zeros to a multiple of 16, k_qg_msum's row tiles)
__host__ __device__ constexpr int qm_stride(int M) { return (M + 15) / 16 * 16; }
constexpr int QG_A_D = 2 * QG_TOK * 16;
constexpr int QG_A_S = QG_A_D + QG_TOK * 4;
__host__ __device__ constexpr int qg_a_bytes(bool one) { return QG_A_S + (one ? QG_TOK * 4 : 0); }

// Device weight matrix, ggml ne=[K, M] (M output rows of K elements).
struct DMat {
    int type;
    int M, K;
    const uint8_t * qs;     // quantized nibbles / int8, or raw F16/F32 rows
    const uint32_t * qh;    // Q5 high bits
    const void * sc;        // u16 d  or u32 (d | m<<16)
    const uint8_t * gt;     // the same blocks as sequence-GEMM tile records (qg_w_*), quantized types
    const float * mt;       // _1 formats with tile records: the mins m as f32, [K / 32][qm_stride(M)]
};

enum Epi : int {
    EPI_STORE = 0,       // y = acc
    EPI_SIGMOID = 1,     // y = sigmoid(acc)
    EPI_TANH = 2,        // y = tanh(acc)
    EPI_SILU = 3,        // y = silu(acc)
    EPI_RELU_SQ = 4,     // y = relu(acc)^2
    EPI_ADD = 5,         // y = y + acc                    (residual)
    EPI_SIGMUL_ADD = 6,  // y = y + sigmoid(aux) * acc     (FFN v4-v6: x += r * (Wv k))
    EPI_DECAY6 = 7,      // y = exp(-exp(acc + bias))      (rwkv_graph.inc:365-367)
    EPI_DECAY7 = 8,      // y = exp(sigmoid(acc + bias) * -0.606531)  (rwkv_graph.inc:425-430)
    EPI_SIGMOID_BIAS = 9,// y = sigmoid(acc + bias)        (rwkv_graph.inc:417-423)
    EPI_VMIX7 = 10,      // y = y + (aux - y) * sigmoid(acc + bias)  (rwkv_graph.inc:443-452)
};

struct MMEntry {
    DMat W;
    ActBuf in;          // input activations [T][K]
    float * y;          // fp32 output [T][ldy] (may be null when only emitting)
    int ldy;
    const float * aux;  // [T][ldy]
    const float * bias; // [M]
    ActBuf out;         // optional: emit post-epilogue values as the next matmul's input
    int emit;
    int epi;
    int block0;         // first workgroup of this entry
    int fuse_emit;      // qgemm: the epilogue emits `out` (Q8_0 tiles) itself; y is not written
    size_t poff;        // qgemm split-K: this entry's partials at part + poff ([S][T][M])
    int cblock0;        // qgemm split-K: first workgroup of this entry in the combine launch
    size_t moff;        // qgemm _1 formats: this entry's m*s totals at m2 + moff ([M][T])
};

constexpr int MM_MAX_ENTRIES = 8;

struct MMGroup {
    MMEntry e[MM_MAX_ENTRIES];
    int n;
    int T;
    float * part;        // split-K partials (qgemm.hip): up to 8 x T x sum(M) floats
    size_t part_floats;
    float * m2;          // qgemm _1 formats: the m*s chain totals, [M][T] per entry (k_qg_msum)
    size_t m2_floats;
    int split;           // qgemm split-K: 0 = by tile count, 1 = never, 4 / 8 = forced
    int fmm;             // float weights: 0 = f32-MFMA form from T = 32, 1 = from T = 16
};

// Per-launch kernel timing (bench roofline).  While a context times its kernels (Engine::set_timing),
// g_klt points at its timer and RK_LAUNCH launches through hipExtLaunchKernelGGL with a start /
// stop event pair: the runtime binds both to the dispatch itself, so their elapsed time is the
// kernel's own execution span -- the begin/end timestamps rocprofv3's kernel trace reports --
// not the gaps between launches.  Otherwise RK_LAUNCH is hipLaunchKernelGGL.
struct KLaunchTimer {
    virtual ~KLaunchTimer() {}
    virtual bool begin(hipEvent_t * a, hipEvent_t * b) = 0;
    virtual void end(const char * kernel) = 0;
};
extern thread_local KLaunchTimer * g_klt;

#define RK_LAUNCH(kern, grid, block, lds, st, ...)                                                  \
    do {                                                                                            \
        hipEvent_t rk_a_ = nullptr, rk_b_ = nullptr;                                                \
        if (::rwkvmi::g_klt && ::rwkvmi::g_klt->begin(&rk_a_, &rk_b_)) {                            \
            hipExtLaunchKernelGGL(kern, grid, block, lds, st, rk_a_, rk_b_, 0u, __VA_ARGS__);       \
            ::rwkvmi::g_klt->end(#kern);                                                            \
        } else {                                                                                    \
            hipLaunchKernelGGL(kern, grid, block, lds, st, __VA_ARGS__);                            \
        }                                                                                           \
    } while (0)

#define HIP_OK(x)                                                                             \
    do {                                                                                      \
        hipError_t _e = (x);                                                                  \
        if (_e != hipSuccess) {                                                               \
            fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(_e), __FILE__, \
                    __LINE__, #x);                                                            \
            return false;                                                                     \
        }                                                                                     \
    } while (0)

}  // namespace rwkvmi
