/*
 * oracle.c -- CPU restatement of the rwkv.cpp eval path.
 *
 * TEST INFRASTRUCTURE, NOT PRODUCT.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline).  librwkv.so never links it.
 *
 * What it restates (reference = /root/reference, cogpy/rwkv.cppy):
 *   - file format + loader      rwkv_file_format.inc:100-316, rwkv_model_loading.inc:128-419
 *   - per-version layer math    rwkv_graph.inc:56-543 (v4 :84-197, v5 :199-292, v6 :294-385,
 *                               v7 :387-482, FFN :484-543), serial/sequence graphs :611-866
 *   - custom operators          rwkv_operators.inc:5-97 (max, l2norm, layer_norm),
 *                               rwkv_operators_wkv_v7.inc:37-107 (wkv7)
 *   - eval drivers / state      rwkv_eval.inc:1-241
 *   - quantizer driver          rwkv_quantize.inc:1-171
 * and the third-party ggml arithmetic those call (ggml is an EMPTY submodule in the
 * reference, .gitmodules:1-4, branch master, commit unknown), restated from ggml's
 * published CPU algorithms:
 *   - ggml_norm (double accumulation), ggml_rwkv_wkv6, ggml_get_rows (F16 upcast)
 *   - ggml_mul_mat CPU numerics: src1 quantized per 32-block to Q8_0 (Q4_0/Q5_0/Q8_0
 *     weights) or Q8_1 (Q4_1/Q5_1 weights) with fp16 scales, id = 127/amax,
 *     round-half-even; integer block dots; F16 weights take fp16-rounded activations.
 *   - quantize_row_{q4_0,q4_1,q5_0,q5_1,q8_0}_ref for the file quantizer.
 *
 * Pinning (tests/test_oracle_pinning.py): FP32 tiny models vs the reference's
 * tests/expected-logits-*.bin (max |dlogit| ~3e-6); quantizer byte-exact vs the
 * reference's tests/tiny-rwkv-*-to-Q*.bin; quantized signed sums vs the reference's
 * constants in tests/test_tiny_rwkv.c:131-227 / test_quantization_format_compatibility.c.
 *
 * Built with -ffp-contract=off so results do not depend on compiler FMA contraction.
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <sys/stat.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#ifdef __AVX2__
#include <immintrin.h>
#endif

#define QK 32
#define ORACLE_MAX_TENSORS 16384

/* test infrastructure: an allocation failure aborts loudly instead of returning a half-computed result */
static void oracle_need(int ok, const char * what) {
    if (!ok) {
        fprintf(stderr, "oracle: out of memory (%s)\n", what);
        abort();
    }
}

/* ------------------------------------------------------------------ fp16 */

uint16_t oracle_f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t exp = (x >> 23) & 0xffu;
    uint32_t mant = x & 0x7fffffu;
    if (exp == 0xff) {
        return (uint16_t)(sign | 0x7c00u | (mant ? (0x200u | (mant >> 13)) : 0u));
    }
    int e = (int)exp - 127 + 15;
    if (e >= 0x1f) {
        return (uint16_t)(sign | 0x7c00u);
    }
    if (e <= 0) {
        if (e < -10) {
            return (uint16_t)sign;
        }
        mant |= 0x800000u;
        int shift = 14 - e;
        uint32_t h = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) {
            h++;
        }
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (mant >> 13);
    uint32_t rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) {
        h++;
    }
    return (uint16_t)(sign | h);
}

float oracle_f16_to_f32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t exp = ((uint32_t)h >> 10) & 0x1fu;
    uint32_t mant = (uint32_t)h & 0x3ffu;
    uint32_t x;
    if (exp == 0) {
        if (mant == 0) {
            x = sign;
        } else {
            int e = -1;
            do {
                e++;
                mant <<= 1;
            } while (!(mant & 0x400u));
            mant &= 0x3ffu;
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
        }
    } else if (exp == 0x1f) {
        x = sign | 0x7f800000u | (mant << 13);
    } else {
        x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

static inline float h2f(const uint8_t * p) {
    uint16_t h;
    memcpy(&h, p, 2);
    return oracle_f16_to_f32(h);
}

static inline void f2h(uint8_t * p, float f) {
    uint16_t h = oracle_f32_to_f16(f);
    memcpy(p, &h, 2);
}

/* ------------------------------------------------------------------ types */

size_t oracle_block_bytes(int type) {
    switch (type) {
        case OT_Q4_0: return 18;
        case OT_Q4_1: return 20;
        case OT_Q5_0: return 22;
        case OT_Q5_1: return 24;
        case OT_Q8_0: return 34;
        case OT_Q8_1: return 36;
        default: return 0;
    }
}

static int type_supported(uint32_t t) {
    return t == OT_FP32 || t == OT_FP16 || t == OT_Q4_0 || t == OT_Q4_1 ||
           t == OT_Q5_0 || t == OT_Q5_1 || t == OT_Q8_0;
}

static int type_quantized(uint32_t t) {
    return t == OT_Q4_0 || t == OT_Q4_1 || t == OT_Q5_0 || t == OT_Q5_1 || t == OT_Q8_0;
}

/* rwkv_utilities.inc:1-4: type_size * ne0 * ne1 * ne2 / block_size */
static size_t tensor_nbytes(uint32_t type, uint64_t n) {
    if (type == OT_FP32) return (size_t)n * 4;
    if (type == OT_FP16) return (size_t)n * 2;
    return (size_t)(n / QK) * oracle_block_bytes((int)type);
}

/* --------------------------------------------------------- file quantizers */
/* Restatement of ggml quantize_row_*_ref (called via ggml_quantize_chunk from
 * rwkv_quantize.inc:149). */

static void q4_0_row(const float * x, uint8_t * y, int64_t k) {
    for (int64_t i = 0; i < k / QK; i++) {
        const float * xb = x + i * QK;
        uint8_t * b = y + i * 18;
        float amax = 0.0f, max = 0.0f;
        for (int j = 0; j < QK; j++) {
            if (amax < fabsf(xb[j])) {
                amax = fabsf(xb[j]);
                max = xb[j];
            }
        }
        const float d = max / -8;
        const float id = d ? 1.0f / d : 0.0f;
        f2h(b, d);
        for (int j = 0; j < QK / 2; j++) {
            const float x0 = xb[j] * id;
            const float x1 = xb[QK / 2 + j] * id;
            int i0 = (int8_t)(x0 + 8.5f);
            int i1 = (int8_t)(x1 + 8.5f);
            uint8_t xi0 = (uint8_t)(i0 < 15 ? i0 : 15);
            uint8_t xi1 = (uint8_t)(i1 < 15 ? i1 : 15);
            b[2 + j] = (uint8_t)(xi0 | (xi1 << 4));
        }
    }
}

static void q4_1_row(const float * x, uint8_t * y, int64_t k) {
    for (int64_t i = 0; i < k / QK; i++) {
        const float * xb = x + i * QK;
        uint8_t * b = y + i * 20;
        float min = FLT_MAX, max = -FLT_MAX;
        for (int j = 0; j < QK; j++) {
            if (xb[j] < min) min = xb[j];
            if (xb[j] > max) max = xb[j];
        }
        const float d = (max - min) / ((1 << 4) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        f2h(b, d);
        f2h(b + 2, min);
        for (int j = 0; j < QK / 2; j++) {
            const float x0 = (xb[j] - min) * id;
            const float x1 = (xb[QK / 2 + j] - min) * id;
            int i0 = (int8_t)(x0 + 0.5f);
            int i1 = (int8_t)(x1 + 0.5f);
            uint8_t xi0 = (uint8_t)(i0 < 15 ? i0 : 15);
            uint8_t xi1 = (uint8_t)(i1 < 15 ? i1 : 15);
            b[4 + j] = (uint8_t)(xi0 | (xi1 << 4));
        }
    }
}

static void q5_0_row(const float * x, uint8_t * y, int64_t k) {
    for (int64_t i = 0; i < k / QK; i++) {
        const float * xb = x + i * QK;
        uint8_t * b = y + i * 22;
        float amax = 0.0f, max = 0.0f;
        for (int j = 0; j < QK; j++) {
            if (amax < fabsf(xb[j])) {
                amax = fabsf(xb[j]);
                max = xb[j];
            }
        }
        const float d = max / -16;
        const float id = d ? 1.0f / d : 0.0f;
        f2h(b, d);
        uint32_t qh = 0;
        for (int j = 0; j < QK / 2; j++) {
            const float x0 = xb[j] * id;
            const float x1 = xb[QK / 2 + j] * id;
            int i0 = (int8_t)(x0 + 16.5f);
            int i1 = (int8_t)(x1 + 16.5f);
            uint8_t xi0 = (uint8_t)(i0 < 31 ? i0 : 31);
            uint8_t xi1 = (uint8_t)(i1 < 31 ? i1 : 31);
            b[6 + j] = (uint8_t)((xi0 & 0x0f) | ((xi1 & 0x0f) << 4));
            qh |= ((uint32_t)(xi0 & 0x10u) >> 4) << (j + 0);
            qh |= ((uint32_t)(xi1 & 0x10u) >> 4) << (j + QK / 2);
        }
        memcpy(b + 2, &qh, 4);
    }
}

static void q5_1_row(const float * x, uint8_t * y, int64_t k) {
    for (int64_t i = 0; i < k / QK; i++) {
        const float * xb = x + i * QK;
        uint8_t * b = y + i * 24;
        float min = FLT_MAX, max = -FLT_MAX;
        for (int j = 0; j < QK; j++) {
            if (xb[j] < min) min = xb[j];
            if (xb[j] > max) max = xb[j];
        }
        const float d = (max - min) / ((1 << 5) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        f2h(b, d);
        f2h(b + 2, min);
        uint32_t qh = 0;
        for (int j = 0; j < QK / 2; j++) {
            const float x0 = (xb[j] - min) * id;
            const float x1 = (xb[QK / 2 + j] - min) * id;
            uint8_t xi0 = (uint8_t)(x0 + 0.5f);
            uint8_t xi1 = (uint8_t)(x1 + 0.5f);
            b[8 + j] = (uint8_t)((xi0 & 0x0f) | ((xi1 & 0x0f) << 4));
            qh |= ((uint32_t)(xi0 & 0x10u) >> 4) << (j + 0);
            qh |= ((uint32_t)(xi1 & 0x10u) >> 4) << (j + QK / 2);
        }
        memcpy(b + 4, &qh, 4);
    }
}

static void q8_0_row(const float * x, uint8_t * y, int64_t k) {
    for (int64_t i = 0; i < k / QK; i++) {
        const float * xb = x + i * QK;
        uint8_t * b = y + i * 34;
        float amax = 0.0f;
        for (int j = 0; j < QK; j++) {
            float a = fabsf(xb[j]);
            amax = amax > a ? amax : a;
        }
        const float d = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        f2h(b, d);
        for (int j = 0; j < QK; j++) {
            b[2 + j] = (uint8_t)(int8_t)roundf(xb[j] * id);
        }
    }
}

void oracle_quantize_row(int type, const float * x, void * dst, int64_t k) {
    uint8_t * y = (uint8_t *)dst;
    switch (type) {
        case OT_Q4_0: q4_0_row(x, y, k); break;
        case OT_Q4_1: q4_1_row(x, y, k); break;
        case OT_Q5_0: q5_0_row(x, y, k); break;
        case OT_Q5_1: q5_1_row(x, y, k); break;
        case OT_Q8_0: q8_0_row(x, y, k); break;
        default: break;
    }
}

/* ------------------------------------------------- activation quantization */
/* The quantizer ggml's CPU mul_mat applies to src1 (vec_dot_type of the weight
 * type): x86 SIMD form -- d = amax/127, id = 127/amax, q = round-half-even(x*id),
 * fp16 d; Q8_1 additionally s = fp16(d * sum(q)).  (SURVEY.md Appendix B.) */
void oracle_quantize_act(int type, const float * x, void * dst, int64_t k) {
    uint8_t * y = (uint8_t *)dst;
    const int bb = (type == OT_Q8_1) ? 36 : 34;
    const int qoff = (type == OT_Q8_1) ? 4 : 2;
    for (int64_t i = 0; i < k / QK; i++) {
        const float * xb = x + i * QK;
        uint8_t * b = y + i * bb;
        float amax = 0.0f;
        for (int j = 0; j < QK; j++) {
            float a = fabsf(xb[j]);
            amax = amax > a ? amax : a;
        }
        const float d = amax / 127.f;
        const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
        f2h(b, d);
        int sum = 0;
        for (int j = 0; j < QK; j++) {
            int q = (int)rintf(xb[j] * id);
            b[qoff + j] = (uint8_t)(int8_t)q;
            sum += q;
        }
        if (type == OT_Q8_1) {
            f2h(b + 2, d * (float)sum);
        }
    }
}

/* ------------------------------------------------------- dequantization */

void oracle_dequantize_row(int type, const void * src, float * dst, int64_t k) {
    const uint8_t * s = (const uint8_t *)src;
    if (type == OT_FP32) {
        memcpy(dst, s, (size_t)k * 4);
        return;
    }
    if (type == OT_FP16) {
        for (int64_t i = 0; i < k; i++) dst[i] = h2f(s + 2 * i);
        return;
    }
    for (int64_t i = 0; i < k / QK; i++) {
        float * o = dst + i * QK;
        switch (type) {
            case OT_Q4_0: {
                const uint8_t * b = s + i * 18;
                float d = h2f(b);
                for (int j = 0; j < 16; j++) {
                    o[j] = (float)((b[2 + j] & 0x0f) - 8) * d;
                    o[j + 16] = (float)((b[2 + j] >> 4) - 8) * d;
                }
            } break;
            case OT_Q4_1: {
                const uint8_t * b = s + i * 20;
                float d = h2f(b), m = h2f(b + 2);
                for (int j = 0; j < 16; j++) {
                    o[j] = (float)(b[4 + j] & 0x0f) * d + m;
                    o[j + 16] = (float)(b[4 + j] >> 4) * d + m;
                }
            } break;
            case OT_Q5_0: {
                const uint8_t * b = s + i * 22;
                float d = h2f(b);
                uint32_t qh;
                memcpy(&qh, b + 2, 4);
                for (int j = 0; j < 16; j++) {
                    int x0 = (b[6 + j] & 0x0f) | (int)(((qh >> j) << 4) & 0x10);
                    int x1 = (b[6 + j] >> 4) | (int)((qh >> (j + 12)) & 0x10);
                    o[j] = (float)(x0 - 16) * d;
                    o[j + 16] = (float)(x1 - 16) * d;
                }
            } break;
            case OT_Q5_1: {
                const uint8_t * b = s + i * 24;
                float d = h2f(b), m = h2f(b + 2);
                uint32_t qh;
                memcpy(&qh, b + 4, 4);
                for (int j = 0; j < 16; j++) {
                    int x0 = (b[8 + j] & 0x0f) | (int)(((qh >> j) << 4) & 0x10);
                    int x1 = (b[8 + j] >> 4) | (int)((qh >> (j + 12)) & 0x10);
                    o[j] = (float)x0 * d + m;
                    o[j + 16] = (float)x1 * d + m;
                }
            } break;
            case OT_Q8_0: {
                const uint8_t * b = s + i * 34;
                float d = h2f(b);
                for (int j = 0; j < 32; j++) o[j] = (float)(int8_t)b[2 + j] * d;
            } break;
            default: break;
        }
    }
}

/* Integer weight values of one block (offset applied for _0 formats). */
static inline void block_ints(int type, const uint8_t * b, int * w, float * d, float * m) {
    *m = 0.0f;
    *d = 0.0f;
    switch (type) {
        case OT_Q4_0:
            *d = h2f(b);
            for (int j = 0; j < 16; j++) {
                w[j] = (b[2 + j] & 0x0f) - 8;
                w[j + 16] = (b[2 + j] >> 4) - 8;
            }
            break;
        case OT_Q4_1:
            *d = h2f(b);
            *m = h2f(b + 2);
            for (int j = 0; j < 16; j++) {
                w[j] = b[4 + j] & 0x0f;
                w[j + 16] = b[4 + j] >> 4;
            }
            break;
        case OT_Q5_0: {
            *d = h2f(b);
            uint32_t qh;
            memcpy(&qh, b + 2, 4);
            for (int j = 0; j < 16; j++) {
                w[j] = ((b[6 + j] & 0x0f) | (int)(((qh >> j) << 4) & 0x10)) - 16;
                w[j + 16] = ((b[6 + j] >> 4) | (int)((qh >> (j + 12)) & 0x10)) - 16;
            }
        } break;
        case OT_Q5_1: {
            *d = h2f(b);
            *m = h2f(b + 2);
            uint32_t qh;
            memcpy(&qh, b + 4, 4);
            for (int j = 0; j < 16; j++) {
                w[j] = (b[8 + j] & 0x0f) | (int)(((qh >> j) << 4) & 0x10);
                w[j + 16] = (b[8 + j] >> 4) | (int)((qh >> (j + 12)) & 0x10);
            }
        } break;
        case OT_Q8_0:
            *d = h2f(b);
            for (int j = 0; j < 32; j++) w[j] = (int8_t)b[2 + j];
            break;
        default:
            break;
    }
}

/* ------------------------------------------------------------------ matmul */

static int g_threads = 0;
/* Variant bits re-associate the reductions -- equally valid restatements used only to
 * measure how strongly a model amplifies last-bit differences (the "noise floor" the GPU
 * comparison is judged against).  Variant 0 is the ggml-x86 mirror.
 *   1: reverse summation order   2: ggml's scalar quantized dot (no fma, m*s inline)
 *   4: fp32 instead of fp64 accumulators in the F32/F16 dots and norms */
static int g_variant = 0;

void oracle_set_variant(int v) { g_variant = v; }

void oracle_set_threads(int n) { g_threads = n; }

int oracle_get_threads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---------------------------------------------------- GPU-association variant
 * Variant bit 8 (ORACLE_VARIANT_GPU) evaluates the same ggml semantics in the association the
 * MI355X kernels use, so the GPU path can be held BIT-EXACT to a CPU restatement.
 * Every op below is an IEEE-exact primitive (add, mul, fma, correctly rounded div/sqrt, rint,
 * ldexp), evaluated in the order the kernels evaluate it:
 *   - matmul: output (row, token) is a 64-lane wave; lane l owns the 16-byte units l, l+64, ...
 *     (a quantized 32-block; 8 F16 or 4 F32 elements) and chains them in ascending order
 *     (quantized: acc = fma(d_w*d_x, sumi, acc), _1 formats: acc2 += m_w*s_x; F16/F32: one fma
 *     per element); the 64 lane partials are folded by wave_sum63's perfect binary tree over
 *     adjacent lanes; _1 formats add the folded acc2, others add +0.0.
 *   - LayerNorm (ggml_norm, fp64 sums): 512-element chunks, lane l owning the chunk's elements
 *     8l..8l+7 as an fp64 pairwise tree, the same 64-lane tree per chunk, chunks in order.
 *   - GroupNorm statistics fold in wave_sum63's tree (adjacent lanes first); the other per-head
 *     sums (wkv7 row sums, l2norm, v7 bonus) fold with the xor butterfly of __shfl_xor (stride
 *     S/2 first); wkv6 y sums over keys split in
 *     G = min(256/S, S) groups of S/G keys (head size 64: four 4-key runs (p0+p1)+(p2+p3)),
 *     groups folded as a stride-halving tree.
 *   - exp / tanh: the kernels' own polynomial implementations (device_common.hpp rk_expf /
 *     rk_tanhf), restated below with the same constants and operation order. */
#define OV_GPU 8

static float gpu_expf(float x) {
    if (x != x) return x;
    if (x > 0x1.62e43p+6f) return INFINITY;
    if (x < -0x1.9fe36ap+6f) return 0.0f;
    const float n = rintf(x * 0x1.715476p+0f);
    float r = fmaf(n, -0x1.62e43p-1f, x);
    r = fmaf(n, 0x1.05c61p-29f, r);
    float q = 0x1.687c22p-10f;
    q = fmaf(q, r, 0x1.123b8ep-7f);
    q = fmaf(q, r, 0x1.555b58p-5f);
    q = fmaf(q, r, 0x1.55548ep-3f);
    q = fmaf(q, r, 0x1.fffff8p-2f);
    const float r2 = r * r;
    const float p = fmaf(r2, q, r) + 1.0f;
    return ldexpf(p, (int)n);
}

static float gpu_tanhf(float x) {
    const float ax = fabsf(x);
    if (ax < 0.625f) {
        const float x2 = x * x;
        float p = -0x1.7507acp-8f;
        p = fmaf(p, x2, 0x1.51f0f0p-6f);
        p = fmaf(p, x2, -0x1.b83322p-5f);
        p = fmaf(p, x2, 0x1.1106d6p-3f);
        p = fmaf(p, x2, -0x1.555532p-2f);
        return fmaf(x * x2, p, x);
    }
    const float t = ax > 9.0f ? 1.0f : 1.0f - 2.0f / (gpu_expf(ax + ax) + 1.0f);
    return copysignf(t, x);
}

static inline float o_exp(float x) { return (g_variant & OV_GPU) ? gpu_expf(x) : expf(x); }
static inline float o_tanh(float x) { return (g_variant & OV_GPU) ? gpu_tanhf(x) : tanhf(x); }

float oracle_gpu_expf(float x) { return gpu_expf(x); }
float oracle_gpu_tanhf(float x) { return gpu_tanhf(x); }

/* wave_sum63 (device_common.hpp): perfect binary tree over adjacent lanes, n a power of two */
static float tree_f(float * a, int n) {
    for (; n > 1; n >>= 1)
        for (int i = 0; i < n / 2; i++) a[i] = a[2 * i] + a[2 * i + 1];
    return a[0];
}
static double tree_d(double * a, int n) {
    for (; n > 1; n >>= 1)
        for (int i = 0; i < n / 2; i++) a[i] = a[2 * i] + a[2 * i + 1];
    return a[0];
}
/* group_sum (__shfl_xor butterfly, stride n/2 first): every lane ends with this value */
static float bfly_f(float * a, int n) {
    for (; n > 1; n >>= 1)
        for (int i = 0; i < n / 2; i++) a[i] = a[i] + a[i + n / 2];
    return a[0];
}

/* ggml_norm statistics in the kernels' chunk association (device_common.hpp ln_stats_wave and the
 * decode prologues): 512-element chunks; lane l of a chunk owns elements 8l..8l+7, summed as the
 * fp64 pairwise tree ((e0+e1)+(e2+e3))+((e4+e5)+(e6+e7)); the 64 lane sums fold by wave_sum63's
 * tree; chunk sums are added in ascending order; elements past n count as zeros. */
static double ln_tree8(const float * v) {
    const double a = ((double)v[0] + (double)v[1]) + ((double)v[2] + (double)v[3]);
    const double b = ((double)v[4] + (double)v[5]) + ((double)v[6] + (double)v[7]);
    return a + b;
}
/* The device's one-pass LayerNorm statistics (device_common.hpp ln_chunk_sums / ln_finish): per
 * 512-element chunk, lane l's 8 elements and their exact fp64 squares summed as pairwise trees,
 * the 64 lanes folded by wave_sum63's tree, chunks added in order; mean = S1/n,
 * var = max(S2/n - mean^2, 0) in fp64, each rounded to f32 once.  ggml_norm's second pass sums
 * fp32-rounded (x - mean)^2 instead: the same quantity up to those roundings (variant 0). */
static double ln_tree8_sq(const float v[8]) {
    double q[8];
    for (int j = 0; j < 8; j++) q[j] = (double)v[j] * (double)v[j];
    const double a = (q[0] + q[1]) + (q[2] + q[3]);
    const double b = (q[4] + q[5]) + (q[6] + q[7]);
    return a + b;
}
static void ln_stats_gpu(const float * x, int64_t n, float eps, float * mean_out, float * scale_out) {
    double lanes[64], lanes2[64];
    const int64_t nc = (n + 511) / 512;
    double s = 0.0, q = 0.0;
    for (int64_t c = 0; c < nc; c++) {
        for (int l = 0; l < 64; l++) {
            float v[8];
            for (int j = 0; j < 8; j++) {
                const int64_t k = c * 512 + 8 * l + j;
                v[j] = k < n ? x[k] : 0.0f;
            }
            lanes[l] = ln_tree8(v);
            lanes2[l] = ln_tree8_sq(v);
        }
        s += tree_d(lanes, 64);
        q += tree_d(lanes2, 64);
    }
    const double md = s / (double)n;
    double vd = q / (double)n - md * md;
    vd = vd > 0.0 ? vd : 0.0;
    *mean_out = (float)md;
    *scale_out = 1.0f / sqrtf((float)vd + eps);
}

/* Exact integer dot of 32 int8 pairs (|w| <= 128, |x| <= 127: the Q8 activation quantizer's
 * range), AVX2 form of ggml's x86 sign/maddubs trick; the plain loop elsewhere. */
static inline int dot32_i8(const int8_t * w, const int8_t * x) {
#ifdef __AVX2__
    const __m256i vw = _mm256_loadu_si256((const __m256i *)w), vx = _mm256_loadu_si256((const __m256i *)x);
    const __m256i p16 = _mm256_maddubs_epi16(_mm256_sign_epi8(vw, vw), _mm256_sign_epi8(vx, vw));
    const __m256i p32 = _mm256_madd_epi16(p16, _mm256_set1_epi16(1));
    __m128i s = _mm_add_epi32(_mm256_castsi256_si128(p32), _mm256_extracti128_si256(p32, 1));
    s = _mm_add_epi32(s, _mm_shuffle_epi32(s, 0x4E));
    s = _mm_add_epi32(s, _mm_shuffle_epi32(s, 0xB1));
    return _mm_cvtsi128_si32(s);
#else
    int sumi = 0;
    for (int j = 0; j < 32; j++) sumi += (int)w[j] * (int)x[j];
    return sumi;
#endif
}

/* quantized matmul in the kernels' association; weights unpacked once per row */
static void matmul_gpu(int wtype, const uint8_t * W, int64_t K, int64_t M, const float * x, int64_t T, float * y) {
    const int nthr = oracle_get_threads();
    (void)nthr;
    if (wtype == OT_FP32 || wtype == OT_FP16) {
        const int per = wtype == OT_FP32 ? 4 : 8;   /* elements per 16-byte unit */
        float * xr = (float *)malloc((size_t)(T * K) * sizeof(float));
        for (int64_t i = 0; i < T * K; i++)
            xr[i] = wtype == OT_FP16 ? oracle_f16_to_f32(oracle_f32_to_f16(x[i])) : x[i];
#pragma omp parallel num_threads(nthr)
        {
            float * wr = (float *)malloc((size_t)K * sizeof(float));
#pragma omp for schedule(static)
            for (int64_t m = 0; m < M; m++) {
                if (wtype == OT_FP32) memcpy(wr, W + (size_t)m * K * 4, (size_t)K * 4);
                else for (int64_t k = 0; k < K; k++) wr[k] = h2f(W + ((size_t)m * K + k) * 2);
                for (int64_t t = 0; t < T; t++) {
                    const float * xt = xr + t * K;
                    float acc[64];
                    for (int l = 0; l < 64; l++) acc[l] = 0.0f;
                    for (int64_t c = 0; c * per < K; c++) {  /* unit c -> lane c % 64, ascending */
                        float a = acc[c & 63];
                        for (int e = 0; e < per; e++) a = fmaf(wr[c * per + e], xt[c * per + e], a);
                        acc[c & 63] = a;
                    }
                    y[t * M + m] = tree_f(acc, 64) + 0.0f;
                }
            }
            free(wr);
        }
        free(xr);
        return;
    }
    const int atype = (wtype == OT_Q4_1 || wtype == OT_Q5_1) ? OT_Q8_1 : OT_Q8_0;
    const int one = atype == OT_Q8_1;
    const int abb = one ? 36 : 34, aqo = one ? 4 : 2;
    const int64_t nb = K / QK;
    const size_t wbb = oracle_block_bytes(wtype);
    uint8_t * xq = (uint8_t *)malloc((size_t)(T * nb * abb));
    /* activations unpacked: int8 values, d, s per block */
    int8_t * xi = (int8_t *)malloc((size_t)(T * K));
    float * xd = (float *)malloc((size_t)(T * nb) * sizeof(float));
    float * xs = (float *)malloc((size_t)(T * nb) * sizeof(float));
    oracle_need(xq && xi && xd && xs, "matmul_gpu activations");
    for (int64_t t = 0; t < T; t++) oracle_quantize_act(atype, x + t * K, xq + t * nb * abb, K);
    for (int64_t t = 0; t < T; t++)
        for (int64_t b = 0; b < nb; b++) {
            const uint8_t * xb = xq + (t * nb + b) * abb;
            memcpy(xi + t * K + b * 32, xb + aqo, 32);
            xd[t * nb + b] = h2f(xb);
            xs[t * nb + b] = one ? h2f(xb + 2) : 0.0f;
        }
    /* weights unpacked once (int8 values, d, m per block), then (token tile x row tile) tasks so
     * the activation tile stays in cache across the rows -- the same arithmetic per output */
    int8_t * wi8 = (int8_t *)malloc((size_t)(M * K));
    float * dw = (float *)malloc((size_t)(M * nb) * sizeof(float));
    float * mw = (float *)malloc((size_t)(M * nb) * sizeof(float));
    oracle_need(wi8 && dw && mw, "matmul_gpu weights");
#pragma omp parallel for schedule(static) num_threads(nthr)
    for (int64_t m = 0; m < M; m++) {
        int wi[32];
        const uint8_t * wrow = W + (size_t)m * nb * wbb;
        for (int64_t b = 0; b < nb; b++) {
            block_ints(wtype, wrow + b * wbb, wi, &dw[m * nb + b], &mw[m * nb + b]);
            for (int j = 0; j < 32; j++) wi8[m * K + b * 32 + j] = (int8_t)wi[j];
        }
    }
    const int64_t TT = 32, MT = 32, ntt = (T + TT - 1) / TT, nmt = (M + MT - 1) / MT;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthr)
    for (int64_t task = 0; task < ntt * nmt; task++) {
        const int64_t t0 = (task / nmt) * TT, m0 = (task % nmt) * MT;
        for (int64_t m = m0; m < m0 + MT && m < M; m++) {
            const int8_t * wr = wi8 + m * K;
            const float * dr = dw + m * nb, * mr = mw + m * nb;
            for (int64_t t = t0; t < t0 + TT && t < T; t++) {
                float acc[64], acc2[64];
                for (int l = 0; l < 64; l++) acc[l] = acc2[l] = 0.0f;
                const int8_t * xt = xi + t * K;
                for (int64_t b = 0; b < nb; b++) {  /* block b -> lane b % 64, ascending */
                    const int sumi = dot32_i8(wr + b * 32, xt + b * 32);
                    acc[b & 63] = fmaf(dr[b] * xd[t * nb + b], (float)sumi, acc[b & 63]);
                    if (one) acc2[b & 63] += mr[b] * xs[t * nb + b];
                }
                const float s = tree_f(acc, 64);
                y[t * M + m] = one ? s + tree_f(acc2, 64) : s + 0.0f;
            }
        }
    }
    free(wi8);
    free(dw);
    free(mw);
    free(xq);
    free(xi);
    free(xd);
    free(xs);
}

/* ggml_mul_mat(W, x) with W ne=[K, M] (row m = K contiguous elements). */
void oracle_matmul(int wtype, const void * Wv, int64_t K, int64_t M,
                   const float * x, int64_t T, float * y) {
    const uint8_t * W = (const uint8_t *)Wv;
    if (g_variant & OV_GPU) {
        matmul_gpu(wtype, W, K, M, x, T, y);
        return;
    }
    const int nthr = oracle_get_threads();
    (void)nthr;
    if (wtype == OT_FP32) {
#pragma omp parallel for schedule(static) num_threads(nthr)
        for (int64_t m = 0; m < M; m++) {
            const float * w = (const float *)(W + (size_t)m * K * 4);
            for (int64_t t = 0; t < T; t++) {
                const float * xt = x + t * K;
                double acc = 0.0;
                float fa = 0.0f;
                for (int64_t kk = 0; kk < K; kk++) {
                    const int64_t k = (g_variant & 1) ? K - 1 - kk : kk;
                    if (g_variant & 4) fa += w[k] * xt[k]; else acc += (double)(w[k] * xt[k]);
                }
                if (g_variant & 4) acc = fa;
                y[t * M + m] = (float)acc;
            }
        }
        return;
    }
    if (wtype == OT_FP16) {
        /* vec_dot_type F16: activations rounded to fp16; fp16*fp16 products are exact in fp32. */
        float * xh = (float *)malloc((size_t)(T * K) * sizeof(float));
        for (int64_t i = 0; i < T * K; i++) xh[i] = oracle_f16_to_f32(oracle_f32_to_f16(x[i]));
#pragma omp parallel for schedule(static) num_threads(nthr)
        for (int64_t m = 0; m < M; m++) {
            const uint8_t * w = W + (size_t)m * K * 2;
            for (int64_t t = 0; t < T; t++) {
                const float * xt = xh + t * K;
                double acc = 0.0;
                float fa = 0.0f;
                for (int64_t kk = 0; kk < K; kk++) {
                    const int64_t k = (g_variant & 1) ? K - 1 - kk : kk;
                    if (g_variant & 4) fa += h2f(w + 2 * k) * xt[k]; else acc += (double)(h2f(w + 2 * k) * xt[k]);
                }
                if (g_variant & 4) acc = fa;
                y[t * M + m] = (float)acc;
            }
        }
        free(xh);
        return;
    }
    /* quantized weights: Q8_0 activations for _0 formats, Q8_1 for _1 formats */
    const int atype = (wtype == OT_Q4_1 || wtype == OT_Q5_1) ? OT_Q8_1 : OT_Q8_0;
    const int abb = atype == OT_Q8_1 ? 36 : 34;
    const int aqo = atype == OT_Q8_1 ? 4 : 2;
    const int64_t nb = K / QK;
    const size_t wbb = oracle_block_bytes(wtype);
    uint8_t * xq = (uint8_t *)malloc((size_t)(T * nb * abb));
    for (int64_t t = 0; t < T; t++) oracle_quantize_act(atype, x + t * K, xq + t * nb * abb, K);
#pragma omp parallel for schedule(static) num_threads(nthr)
    for (int64_t m = 0; m < M; m++) {
        const uint8_t * wrow = W + (size_t)m * nb * wbb;
        int wi[32];
        for (int64_t t = 0; t < T; t++) {
            const uint8_t * xr = xq + t * nb * abb;
            /* ggml x86 vec_dot_q*_q8_*: acc = fma(d_w*d_x, sumi, acc) in fp32; the
             * m_w*s_x terms of the _1 formats are summed separately and added last. */
            float acc = 0.0f, summs = 0.0f;
            for (int64_t bi = 0; bi < nb; bi++) {
                const int64_t b = (g_variant & 1) ? nb - 1 - bi : bi;
                float dw, mw;
                block_ints(wtype, wrow + b * wbb, wi, &dw, &mw);
                const uint8_t * xb = xr + b * abb;
                int sumi = 0;
                for (int j = 0; j < 32; j++) sumi += wi[j] * (int8_t)xb[aqo + j];
                const float dx = h2f(xb);
                if (g_variant & 2) {
                    /* ggml scalar form: sumf += sumi*dx*dy (+ m*s inline) */
                    acc += (float)sumi * dw * dx;
                    if (atype == OT_Q8_1) acc += mw * h2f(xb + 2);
                    continue;
                }
                acc = fmaf(dw * dx, (float)sumi, acc);
                if (atype == OT_Q8_1) summs += mw * h2f(xb + 2);
            }
            y[t * M + m] = acc + summs;
        }
    }
    free(xq);
}

/* ------------------------------------------------------------------- model */

typedef struct {
    char * name;
    uint32_t type;
    uint32_t ndim;
    uint32_t ne[3];
    uint64_t nel;
    uint8_t * data;
} otensor;

typedef struct {
    /* elementwise vectors (fp32 copies) */
    float *ln1_w, *ln1_b, *ln2_w, *ln2_b;
    float *att_mix_k, *att_mix_v, *att_mix_r, *att_mix_g;
    float *att_first, *att_decay, *att_faaaa, *att_lnx_w, *att_lnx_b;
    float *maa_x, *maa[5];               /* v6: w k v r g */
    float *maa_w2;                       /* v6: [5][C][32] */
    float *x_rwkvag;                     /* v7: [6][C] */
    float *w0, *a0, *v0, *k_k, *k_a, *r_k;
    float *ffn_mix_k, *ffn_mix_r, *ffn_maa_k, *ffn_maa_r, *ffn_x_k;
    /* matrices */
    otensor *att_r, *att_k, *att_v, *att_o, *att_g;
    otensor *maa_w1, *decay_w1, *decay_w2;
    otensor *w1, *w2, *a1, *a2, *g1, *g2, *v1, *v2;
    otensor *ffn_k, *ffn_v, *ffn_r;
} olayer;

struct oracle_model {
    uint32_t n_vocab, n_embed, n_layer, data_type, version;
    int major, minor;
    int64_t head_count, head_size;
    int n_tensors;
    otensor tensors[ORACLE_MAX_TENSORS];
    otensor *emb, *head;
    float *ln0_w, *ln0_b, *lnout_w, *lnout_b;
    olayer * layers;
    float ** owned;
    int n_owned, cap_owned;
};

static otensor * find(oracle_model * m, const char * name) {
    for (int i = 0; i < m->n_tensors; i++) {
        if (strcmp(m->tensors[i].name, name) == 0) return &m->tensors[i];
    }
    return NULL;
}

static float * own(oracle_model * m, float * p) {
    if (m->n_owned == m->cap_owned) {
        m->cap_owned = m->cap_owned ? m->cap_owned * 2 : 256;
        m->owned = (float **)realloc(m->owned, sizeof(float *) * (size_t)m->cap_owned);
    }
    m->owned[m->n_owned++] = p;
    return p;
}

static float * as_f32(oracle_model * m, otensor * t) {
    float * out = (float *)malloc(sizeof(float) * (size_t)t->nel);
    oracle_dequantize_row((int)t->type, t->data, out, (int64_t)t->nel);
    return own(m, out);
}

static int g_err = 0;
#define OFAIL(...) do { fprintf(stderr, "oracle: " __VA_ARGS__); fprintf(stderr, "\n"); g_err = 1; return NULL; } while (0)

static otensor * need(oracle_model * m, const char * fmt, int layer) {
    char key[160];
    if (layer >= 0) snprintf(key, sizeof key, fmt, layer); else snprintf(key, sizeof key, "%s", fmt);
    otensor * t = find(m, key);
    if (!t) {
        fprintf(stderr, "oracle: model parameter %s not found\n", key);
        g_err = 1;
    }
    return t;
}

static float * needv(oracle_model * m, const char * fmt, int layer) {
    otensor * t = need(m, fmt, layer);
    return t ? as_f32(m, t) : NULL;
}

void oracle_free(oracle_model * m) {
    if (!m) return;
    for (int i = 0; i < m->n_tensors; i++) {
        free(m->tensors[i].name);
        free(m->tensors[i].data);
    }
    for (int i = 0; i < m->n_owned; i++) free(m->owned[i]);
    free(m->owned);
    free(m->layers);
    free(m);
}

oracle_model * oracle_load(const char * path) {
    FILE * f = fopen(path, "rb");
    if (!f) OFAIL("cannot open %s", path);
    struct stat st;
    if (fstat(fileno(f), &st) != 0) {
        fclose(f);
        OFAIL("cannot stat %s", path);
    }
    uint32_t hdr[6];
    if (fread(hdr, 4, 6, f) != 6) {
        fclose(f);
        OFAIL("short header");
    }
    /* rwkv_file_format.inc:115-142 */
    if (hdr[0] != 0x67676d66u || hdr[1] < 100 || hdr[1] > 101 || !type_supported(hdr[5]) ||
        (type_quantized(hdr[5]) && hdr[1] != 101)) {
        fclose(f);
        OFAIL("bad header (magic %08x version %u type %u)", hdr[0], hdr[1], hdr[5]);
    }
    oracle_model * m = (oracle_model *)calloc(1, sizeof(oracle_model));
    m->version = hdr[1];
    m->n_vocab = hdr[2];
    m->n_embed = hdr[3];
    m->n_layer = hdr[4];
    m->data_type = hdr[5];
    long pos = ftell(f);
    while (pos < (long)st.st_size) {
        uint32_t th[3];
        if (fread(th, 4, 3, f) != 3 || th[0] < 1 || th[0] > 3 || !type_supported(th[2]) ||
            m->n_tensors >= ORACLE_MAX_TENSORS) {
            fclose(f);
            oracle_free(m);
            OFAIL("bad tensor header");
        }
        otensor * t = &m->tensors[m->n_tensors];
        t->ndim = th[0];
        t->type = th[2];
        t->ne[0] = t->ne[1] = t->ne[2] = 1;
        if (fread(t->ne, 4, th[0], f) != th[0]) {
            fclose(f);
            oracle_free(m);
            OFAIL("bad tensor shape");
        }
        t->name = (char *)calloc(th[1] + 1, 1);
        if (fread(t->name, 1, th[1], f) != th[1]) {
            free(t->name);
            fclose(f);
            oracle_free(m);
            OFAIL("bad tensor name");
        }
        t->nel = (uint64_t)t->ne[0] * t->ne[1] * t->ne[2];
        size_t nb = tensor_nbytes(t->type, t->nel);
        t->data = (uint8_t *)malloc(nb ? nb : 1);
        if (fread(t->data, 1, nb, f) != nb) {
            free(t->name);
            free(t->data);
            fclose(f);
            oracle_free(m);
            OFAIL("short tensor data for %s", t->name);
        }
        m->n_tensors++;
        pos = ftell(f);
    }
    fclose(f);

    /* arch detection, rwkv_model_loading.inc:319-340 */
    m->major = 4;
    m->minor = 0;
    if (find(m, "blocks.0.att.ln_x.weight")) {
        m->major = 5;
        m->minor = find(m, "blocks.0.att.gate.weight") ? 2 : 1;
    }
    if (find(m, "blocks.0.att.time_maa_x")) {
        m->major = 6;
        m->minor = 0;
    }
    if (find(m, "blocks.0.att.r_k")) {
        m->major = 7;
        m->minor = 0;
    }

    g_err = 0;
    m->emb = need(m, "emb.weight", -1);
    m->ln0_w = needv(m, "blocks.0.ln0.weight", -1);
    m->ln0_b = needv(m, "blocks.0.ln0.bias", -1);
    m->lnout_w = needv(m, "ln_out.weight", -1);
    m->lnout_b = needv(m, "ln_out.bias", -1);
    m->head = need(m, "head.weight", -1);
    m->layers = (olayer *)calloc(m->n_layer, sizeof(olayer));
    for (uint32_t i = 0; i < m->n_layer && !g_err; i++) {
        olayer * L = &m->layers[i];
        int l = (int)i;
        L->ln1_w = needv(m, "blocks.%d.ln1.weight", l);
        L->ln1_b = needv(m, "blocks.%d.ln1.bias", l);
        L->ln2_w = needv(m, "blocks.%d.ln2.weight", l);
        L->ln2_b = needv(m, "blocks.%d.ln2.bias", l);
        L->att_k = need(m, "blocks.%d.att.key.weight", l);
        L->att_v = need(m, "blocks.%d.att.value.weight", l);
        L->att_r = need(m, "blocks.%d.att.receptance.weight", l);
        L->att_o = need(m, "blocks.%d.att.output.weight", l);
        L->ffn_k = need(m, "blocks.%d.ffn.key.weight", l);
        L->ffn_v = need(m, "blocks.%d.ffn.value.weight", l);
        if (m->major != 7) L->ffn_r = need(m, "blocks.%d.ffn.receptance.weight", l);
        if (m->major == 4 || m->major == 5) {
            L->att_mix_k = needv(m, "blocks.%d.att.time_mix_k", l);
            L->att_mix_v = needv(m, "blocks.%d.att.time_mix_v", l);
            L->att_mix_r = needv(m, "blocks.%d.att.time_mix_r", l);
            L->att_decay = needv(m, "blocks.%d.att.time_decay", l);
            L->ffn_mix_k = needv(m, "blocks.%d.ffn.time_mix_k", l);
            L->ffn_mix_r = needv(m, "blocks.%d.ffn.time_mix_r", l);
            if (m->major == 4 || m->minor < 2) L->att_first = needv(m, "blocks.%d.att.time_first", l);
        }
        if (m->major >= 5) {
            L->att_lnx_w = needv(m, "blocks.%d.att.ln_x.weight", l);
            L->att_lnx_b = needv(m, "blocks.%d.att.ln_x.bias", l);
        }
        if (m->major == 5 && m->minor >= 2) {
            L->att_faaaa = needv(m, "blocks.%d.att.time_faaaa", l);
            L->att_mix_g = needv(m, "blocks.%d.att.time_mix_g", l);
            L->att_g = need(m, "blocks.%d.att.gate.weight", l);
        }
        if (m->major == 6) {
            L->maa_x = needv(m, "blocks.%d.att.time_maa_x", l);
            L->maa[0] = needv(m, "blocks.%d.att.time_maa_w", l);
            L->maa[1] = needv(m, "blocks.%d.att.time_maa_k", l);
            L->maa[2] = needv(m, "blocks.%d.att.time_maa_v", l);
            L->maa[3] = needv(m, "blocks.%d.att.time_maa_r", l);
            L->maa[4] = needv(m, "blocks.%d.att.time_maa_g", l);
            L->maa_w1 = need(m, "blocks.%d.att.time_maa_w1", l);
            L->maa_w2 = needv(m, "blocks.%d.att.time_maa_w2", l);
            L->att_faaaa = needv(m, "blocks.%d.att.time_faaaa", l);
            L->att_decay = needv(m, "blocks.%d.att.time_decay", l);
            L->decay_w1 = need(m, "blocks.%d.att.time_decay_w1", l);
            L->decay_w2 = need(m, "blocks.%d.att.time_decay_w2", l);
            L->att_g = need(m, "blocks.%d.att.gate.weight", l);
            L->ffn_maa_k = needv(m, "blocks.%d.ffn.time_maa_k", l);
            L->ffn_maa_r = needv(m, "blocks.%d.ffn.time_maa_r", l);
        }
        if (m->major == 7) {
            L->x_rwkvag = needv(m, "blocks.%d.att.x_rwkvag", l);
            L->w0 = needv(m, "blocks.%d.att.w0", l);
            L->w1 = need(m, "blocks.%d.att.w1", l);
            L->w2 = need(m, "blocks.%d.att.w2", l);
            L->a0 = needv(m, "blocks.%d.att.a0", l);
            L->a1 = need(m, "blocks.%d.att.a1", l);
            L->a2 = need(m, "blocks.%d.att.a2", l);
            L->g1 = need(m, "blocks.%d.att.g1", l);
            L->g2 = need(m, "blocks.%d.att.g2", l);
            if (i != 0) {
                L->v0 = needv(m, "blocks.%d.att.v0", l);
                L->v1 = need(m, "blocks.%d.att.v1", l);
                L->v2 = need(m, "blocks.%d.att.v2", l);
            }
            L->r_k = needv(m, "blocks.%d.att.r_k", l);
            L->k_k = needv(m, "blocks.%d.att.k_k", l);
            L->k_a = needv(m, "blocks.%d.att.k_a", l);
            L->ffn_x_k = needv(m, "blocks.%d.ffn.x_k", l);
        }
    }
    if (g_err) {
        oracle_free(m);
        return NULL;
    }
    if (m->major == 7) {
        m->head_count = find(m, "blocks.0.att.r_k")->ne[1];
    } else if (m->major >= 5) {
        m->head_count = find(m, "blocks.0.att.time_decay")->ne[2];
    }
    if (m->head_count) m->head_size = (int64_t)m->n_embed / m->head_count;
    if (m->emb->ne[0] != m->n_embed || m->emb->ne[1] != m->n_vocab) {
        oracle_free(m);
        OFAIL("unexpected embedding shape");
    }
    return m;
}

static int64_t state_len(const oracle_model * m) {
    if (m->major >= 5) return (int64_t)m->n_embed * (2 + m->head_size) * m->n_layer;
    return (int64_t)m->n_embed * 5 * m->n_layer;
}

void oracle_info(const oracle_model * m, int64_t out[8]) {
    out[0] = m->n_vocab;
    out[1] = m->n_embed;
    out[2] = m->n_layer;
    out[3] = m->major;
    out[4] = m->minor;
    out[5] = m->head_count;
    out[6] = m->head_size;
    out[7] = state_len(m);
}

void oracle_init_state(const oracle_model * m, float * state) {
    int64_t n = state_len(m);
    memset(state, 0, sizeof(float) * (size_t)n);
    if (m->major >= 5) return;
    const int64_t C = m->n_embed;
    for (uint32_t i = 0; i < m->n_layer; i++) {
        for (int64_t c = 0; c < C; c++) state[i * 5 * C + 4 * C + c] = -1e30f;
    }
}

/* ------------------------------------------------------------------- ops */

/* ggml_norm (double accumulation) then *w +b, rwkv_operators.inc:93-97 */
static void norm_row(const float * x, float * y, int64_t n, float eps, const float * w, const float * b) {
    if ((g_variant & OV_GPU) && n % 64 == 0) {
        float mean, scale;
        ln_stats_gpu(x, n, eps, &mean, &scale);
        for (int64_t i = 0; i < n; i++) {
            float v = (x[i] - mean) * scale;
            if (w) v = v * w[i];
            if (b) v = v + b[i];
            y[i] = v;
        }
        return;
    }
    double sum = 0.0;
    float fs = 0.0f;
    for (int64_t ii = 0; ii < n; ii++) {
        const int64_t i = (g_variant & 1) ? n - 1 - ii : ii;
        if (g_variant & 4) fs += x[i]; else sum += (double)x[i];
    }
    if (g_variant & 4) sum = fs;
    const float mean = (float)(sum / (double)n);
    double sum2 = 0.0;
    float fs2 = 0.0f;
    for (int64_t i = 0; i < n; i++) {
        float v = x[i] - mean;
        y[i] = v;
        sum2 += (double)(v * v);
        fs2 += v * v;
    }
    if (g_variant & 4) sum2 = fs2;
    const float variance = (float)(sum2 / (double)n);
    const float scale = 1.0f / sqrtf(variance + eps);
    for (int64_t i = 0; i < n; i++) y[i] = y[i] * scale;
    if (w) for (int64_t i = 0; i < n; i++) y[i] = y[i] * w[i];
    if (b) for (int64_t i = 0; i < n; i++) y[i] = y[i] + b[i];
}

static inline float sigmoidf_(float x) { return 1.0f / (1.0f + o_exp(-x)); }
static inline float siluf_(float x) { return x / (1.0f + o_exp(-x)); }

static void mm(const otensor * W, const float * x, int64_t T, float * y) {
    oracle_matmul((int)W->type, W->data, W->ne[0], W->ne[1], x, T, y);
}

/* ggml_rwkv_wkv6 CPU semantics (called at rwkv_graph.inc:275,370).
 * state [H][S_i(key)][S_j(value)]; w indexed per token. */
static void wkv6(int64_t T, int64_t H, int64_t S, const float * k, const float * v, const float * r,
                 const float * u, const float * w, int w_per_token, float * state, float * y) {
    const int64_t C = H * S;
    if (g_variant & OV_GPU) {
        /* k_att6_dec / k_wkv6 / k_wkv6_s64: value column j, keys split in G groups of IPG */
        const int64_t G = (256 / S) < S ? (256 / S) : S, IPG = S / G;
        for (int64_t t = 0; t < T; t++) {
            const float * wt = w + (w_per_token ? t * C : 0);
            for (int64_t h = 0; h < H; h++) {
                float * st = state + h * S * S;
                const int64_t o = t * C + h * S;
                for (int64_t j = 0; j < S; j++) {
                    float part[64];
                    for (int64_t g = 0; g < G; g++) {
                        float acc = 0.0f, p4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                        for (int64_t ii = 0; ii < IPG; ii++) {
                            const int64_t i = g * IPG + ii;
                            const float prev = st[i * S + j];
                            const float kv = v[o + j] * k[o + i];
                            const float temp = kv * u[h * S + i] + prev;
                            const float tt = temp * r[o + i];
                            acc += tt;
                            p4[ii >> 2] += tt;
                            st[i * S + j] = prev * wt[h * S + i] + kv;
                        }
                        part[g] = IPG == 16 ? (p4[0] + p4[1]) + (p4[2] + p4[3]) : acc;
                    }
                    y[o + j] = bfly_f(part, (int)G);
                }
            }
        }
        return;
    }
    for (int64_t t = 0; t < T; t++) {
        const float * wt = w + (w_per_token ? t * C : 0);
        for (int64_t i = 0; i < C; i++) y[t * C + i] = 0.0f;
        for (int64_t h = 0; h < H; h++) {
            float * st = state + h * S * S;
            for (int64_t i = 0; i < S; i++) {
                const int64_t ti = t * C + h * S + i;
                const float kv_k = k[ti], r_v = r[ti], u_v = u[h * S + i], w_v = wt[h * S + i];
                for (int64_t j = 0; j < S; j++) {
                    const int64_t tj = t * C + h * S + j;
                    const float kv = v[tj] * kv_k;
                    const float prev = st[i * S + j];
                    const float temp = kv * u_v + prev;
                    y[tj] += temp * r_v;
                    st[i * S + j] = prev * w_v + kv;
                }
            }
        }
    }
}

/* rwkv_operators_wkv_v7.inc:37-107; state [H][i(value)][j(key)] */
static void wkv7(int64_t T, int64_t H, int64_t S, const float * r, const float * w, const float * k,
                 const float * v, const float * a, const float * b, float * state, float * y) {
    const int64_t C = H * S;
    if (g_variant & OV_GPU) {
        /* k_att7_dec / k_wkv7 / k_wkv7_s64: value row i, keys split in G groups of JPG (head size
           64: 16 groups of 4, k_wkv7_s64 / k_att7_dec; others: k_wkv7's min(256 / S, S) groups) */
        const int64_t G = S == 64 ? 16 : (256 / S) < S ? (256 / S) : S, JPG = S / G;
        for (int64_t t = 0; t < T; t++)
            for (int64_t h = 0; h < H; h++) {
                float * st = state + h * S * S;
                const int64_t th = t * C + h * S;
                for (int64_t i = 0; i < S; i++) {
                    float sa[64], acc[64];
                    for (int64_t g = 0; g < G; g++) {
                        float s = 0.0f;
                        for (int64_t jj = 0; jj < JPG; jj++) s += a[th + g * JPG + jj] * st[i * S + g * JPG + jj];
                        sa[g] = s;
                    }
                    const float sat = bfly_f(sa, (int)G);
                    const float vi = v[th + i];
                    for (int64_t g = 0; g < G; g++) {
                        float s = 0.0f;
                        for (int64_t jj = 0; jj < JPG; jj++) {
                            const int64_t j = g * JPG + jj;
                            const float kv = vi * k[th + j];
                            const float ns = st[i * S + j] * w[th + j] + kv + sat * b[th + j];
                            st[i * S + j] = ns;
                            s += ns * r[th + j];
                        }
                        acc[g] = s;
                    }
                    y[th + i] = bfly_f(acc, (int)G);
                }
            }
        return;
    }
    for (int64_t t = 0; t < T; t++) {
        for (int64_t h = 0; h < H; h++) {
            float * st = state + h * S * S;
            const int64_t th = t * C + h * S;
            for (int64_t i = 0; i < S; i++) {
                const float v_val = v[th + i];
                float sa = 0.0f;
                for (int64_t j = 0; j < S; j++) sa += a[th + j] * st[i * S + j];
                float acc = 0.0f;
                for (int64_t j = 0; j < S; j++) {
                    const float kv = v_val * k[th + j];
                    const float ns = st[i * S + j] * w[th + j] + kv + sa * b[th + j];
                    st[i * S + j] = ns;
                    acc += ns * r[th + j];
                }
                y[th + i] = acc;
            }
        }
    }
}

/* --------------------------------------------------------------- forward */

#define ALLOC(n) ((float *)calloc((size_t)(n), sizeof(float)))

/* LN(x) over T rows + token shift, rwkv_graph.inc:56-82.  Writes xa (normed) and xp
 * (previous-token normed), updates carry to xa[T-1]. */
static void carry_x(const float * x, int64_t T, int64_t C, const float * w, const float * b,
                    float * carry, float * xa, float * xp) {
    for (int64_t t = 0; t < T; t++) norm_row(x + t * C, xa + t * C, C, 1e-5f, w, b);
    memcpy(xp, carry, sizeof(float) * (size_t)C);
    if (T > 1) memcpy(xp + C, xa, sizeof(float) * (size_t)((T - 1) * C));
    memcpy(carry, xa + (T - 1) * C, sizeof(float) * (size_t)C);
}

/* ggml: add(mul(x, mu), sub(xp, mul(xp, mu))) */
static void mix_v4(const float * xa, const float * xp, const float * mu, int64_t T, int64_t C, float * out) {
    for (int64_t t = 0; t < T; t++)
        for (int64_t c = 0; c < C; c++) {
            const float a = xa[t * C + c], p = xp[t * C + c];
            out[t * C + c] = a * mu[c] + (p - p * mu[c]);
        }
}

static void group_norm(float * x, int64_t T, int64_t H, int64_t S, float eps, const float * w, const float * b) {
    if (g_variant & OV_GPU) {
        /* k_att6_dec / k_att7_dec / k_groupnorm: fp64 sums over the head's S lanes in wave_sum63's
         * tree (group_tree_sum_d: adjacent lanes first) */
        double buf[64];
        for (int64_t t = 0; t < T; t++)
            for (int64_t h = 0; h < H; h++) {
                float * p = x + t * H * S + h * S;
                for (int64_t i = 0; i < S; i++) buf[i] = (double)p[i];
                const float mean = (float)(tree_d(buf, (int)S) / (double)S);
                for (int64_t i = 0; i < S; i++) {
                    const float d = p[i] - mean;
                    buf[i] = (double)(d * d);
                }
                const float var = (float)(tree_d(buf, (int)S) / (double)S);
                const float scale = 1.0f / sqrtf(var + eps);
                for (int64_t i = 0; i < S; i++) {
                    float o = (p[i] - mean) * scale;
                    o = o * w[h * S + i];
                    p[i] = o + b[h * S + i];
                }
            }
        return;
    }
    float * tmp = ALLOC(S);
    for (int64_t t = 0; t < T; t++)
        for (int64_t h = 0; h < H; h++) {
            float * p = x + t * H * S + h * S;
            norm_row(p, tmp, S, eps, NULL, NULL);
            for (int64_t i = 0; i < S; i++) p[i] = tmp[i] * w[h * S + i] + b[h * S + i];
        }
    free(tmp);
}

static void layer_v4(const oracle_model * m, const olayer * L, float * x, int64_t T, float * st) {
    const int64_t C = m->n_embed;
    float * att_xx = st + C, * aa = st + 2 * C, * bb = st + 3 * C, * pp = st + 4 * C;
    float *xa = ALLOC(T * C), *xp = ALLOC(T * C), *xk = ALLOC(T * C), *xv = ALLOC(T * C), *xr = ALLOC(T * C);
    float *r = ALLOC(T * C), *k = ALLOC(T * C), *v = ALLOC(T * C), *o = ALLOC(T * C);
    /* rwkv_graph.inc:84-197 */
    carry_x(x, T, C, L->ln1_w, L->ln1_b, att_xx, xa, xp);
    mix_v4(xa, xp, L->att_mix_k, T, C, xk);
    mix_v4(xa, xp, L->att_mix_v, T, C, xv);
    mix_v4(xa, xp, L->att_mix_r, T, C, xr);
    mm(L->att_r, xr, T, r);
    for (int64_t i = 0; i < T * C; i++) r[i] = sigmoidf_(r[i]);
    mm(L->att_k, xk, T, k);
    mm(L->att_v, xv, T, v);
    for (int64_t t = 0; t < T; t++)
        for (int64_t c = 0; c < C; c++) {
            const float kt = k[t * C + c], vt = v[t * C + c];
            float ww = L->att_first[c] + kt;
            float qq = fmaxf(pp[c], ww);
            float e1 = o_exp(pp[c] - qq), e2 = o_exp(ww - qq);
            float a = e1 * aa[c] + e2 * vt;
            float bsum = e1 * bb[c] + e2;
            ww = pp[c] + L->att_decay[c];
            qq = fmaxf(ww, kt);
            e1 = o_exp(ww - qq);
            e2 = o_exp(kt - qq);
            aa[c] = e1 * aa[c] + e2 * vt;
            bb[c] = e1 * bb[c] + e2;
            pp[c] = qq;
            xk[t * C + c] = r[t * C + c] * (a / bsum);   /* reuse xk as r*wkv */
        }
    mm(L->att_o, xk, T, o);
    for (int64_t i = 0; i < T * C; i++) x[i] = x[i] + o[i];
    free(xa); free(xp); free(xk); free(xv); free(xr); free(r); free(k); free(v); free(o);
}

/* FFN v4/v5, rwkv_graph.inc:484-511 */
static void ffn_v4_v5(const oracle_model * m, const olayer * L, float * x, int64_t T, float * ffn_xx) {
    const int64_t C = m->n_embed, F = L->ffn_k->ne[1];
    float *xa = ALLOC(T * C), *xp = ALLOC(T * C), *xk = ALLOC(T * C), *xr = ALLOC(T * C);
    float *r = ALLOC(T * C), *k = ALLOC(T * F), *o = ALLOC(T * C);
    carry_x(x, T, C, L->ln2_w, L->ln2_b, ffn_xx, xa, xp);
    mix_v4(xa, xp, L->ffn_mix_k, T, C, xk);
    mix_v4(xa, xp, L->ffn_mix_r, T, C, xr);
    mm(L->ffn_r, xr, T, r);
    mm(L->ffn_k, xk, T, k);
    for (int64_t i = 0; i < T * F; i++) {
        float kk = k[i] > 0.0f ? k[i] : 0.0f;
        k[i] = kk * kk;
    }
    mm(L->ffn_v, k, T, o);
    for (int64_t i = 0; i < T * C; i++) x[i] = x[i] + sigmoidf_(r[i]) * o[i];
    free(xa); free(xp); free(xk); free(xr); free(r); free(k); free(o);
}

static void layer_v5(const oracle_model * m, const olayer * L, float * x, int64_t T, float * st) {
    const int64_t C = m->n_embed, H = m->head_count, S = m->head_size;
    float * att_xx = st + C, * heads = st + 2 * C;
    float *xa = ALLOC(T * C), *xp = ALLOC(T * C), *xk = ALLOC(T * C), *xv = ALLOC(T * C), *xr = ALLOC(T * C),
          *xg = ALLOC(T * C);
    float *r = ALLOC(T * C), *k = ALLOC(T * C), *v = ALLOC(T * C), *g = ALLOC(T * C), *y = ALLOC(T * C),
          *o = ALLOC(T * C);
    float *u = ALLOC(C), *w = ALLOC(C);
    /* rwkv_graph.inc:199-292 */
    carry_x(x, T, C, L->ln1_w, L->ln1_b, att_xx, xa, xp);
    mix_v4(xa, xp, L->att_mix_k, T, C, xk);
    mix_v4(xa, xp, L->att_mix_v, T, C, xv);
    mix_v4(xa, xp, L->att_mix_r, T, C, xr);
    const int v52 = m->minor >= 2;
    if (v52) mix_v4(xa, xp, L->att_mix_g, T, C, xg);
    mm(L->att_r, xr, T, r);
    mm(L->att_k, xk, T, k);
    mm(L->att_v, xv, T, v);
    if (v52) {
        mm(L->att_g, xg, T, g);
        for (int64_t i = 0; i < T * C; i++) g[i] = siluf_(g[i]);
    }
    for (int64_t h = 0; h < H; h++)
        for (int64_t i = 0; i < S; i++) {
            /* 5.2: faaaa/decay are [1,S,H]; 5.1: first/decay are [1,1,H], repeated over S */
            u[h * S + i] = v52 ? L->att_faaaa[h * S + i] : L->att_first[h];
            w[h * S + i] = v52 ? L->att_decay[h * S + i] : L->att_decay[h];
        }
    wkv6(T, H, S, k, v, r, u, w, 0, heads, y);
    group_norm(y, T, H, S, 1e-5f, L->att_lnx_w, L->att_lnx_b);
    if (v52) for (int64_t i = 0; i < T * C; i++) y[i] = y[i] * g[i];
    mm(L->att_o, y, T, o);
    for (int64_t i = 0; i < T * C; i++) x[i] = x[i] + o[i];
    free(xa); free(xp); free(xk); free(xv); free(xr); free(xg);
    free(r); free(k); free(v); free(g); free(y); free(o); free(u); free(w);
}

static void layer_v6(const oracle_model * m, const olayer * L, float * x, int64_t T, float * st) {
    const int64_t C = m->n_embed, H = m->head_count, S = m->head_size;
    const int64_t D5 = L->maa_w1->ne[1], D = D5 / 5, DW = L->decay_w1->ne[1];
    float * att_xx = st + C, * heads = st + 2 * C;
    float *xa = ALLOC(T * C), *xp = ALLOC(T * C), *sx = ALLOC(T * C), *xxx = ALLOC(T * C);
    float *lora = ALLOC(T * D5), *xs[5], *r = ALLOC(T * C), *k = ALLOC(T * C), *v = ALLOC(T * C),
          *g = ALLOC(T * C), *w = ALLOC(T * C), *y = ALLOC(T * C), *o = ALLOC(T * C), *dl = ALLOC(T * DW);
    for (int n = 0; n < 5; n++) xs[n] = ALLOC(T * C);
    /* rwkv_graph.inc:294-385 */
    carry_x(x, T, C, L->ln1_w, L->ln1_b, att_xx, xa, xp);
    for (int64_t i = 0; i < T * C; i++) {
        sx[i] = xp[i] - xa[i];
        xxx[i] = sx[i] * L->maa_x[i % C] + xa[i];
    }
    mm(L->maa_w1, xxx, T, lora);
    for (int64_t i = 0; i < T * D5; i++) lora[i] = o_tanh(lora[i]);
    /* bmm with time_maa_w2 [5][C][D] (ne=[D,C,5]); order w,k,v,r,g */
    for (int n = 0; n < 5; n++)
        for (int64_t t = 0; t < T; t++)
            for (int64_t c = 0; c < C; c++) {
                const float * w2 = L->maa_w2 + ((size_t)n * C + c) * D;
                const float * lv = lora + t * D5 + n * D;
                float mval;
                if (g_variant & OV_GPU) {
                    /* GPU association (k_v6_mix5 / k_v6_mix5_dec / k_v6_maa_dec): one fp32 fma
                       chain over i in order, like ggml's SIMD vec_dot_f32 lanes (fp32 fma) */
                    float a = 0.0f;
                    for (int64_t i = 0; i < D; i++) a = fmaf(w2[i], lv[i], a);
                    mval = a;
                } else {
                    double acc = 0.0;
                    for (int64_t i = 0; i < D; i++) acc += (double)(w2[i] * lv[i]);
                    mval = (float)acc;
                }
                xs[n][t * C + c] = (mval + L->maa[n][c]) * sx[t * C + c] + xa[t * C + c];
            }
    mm(L->att_r, xs[3], T, r);
    mm(L->att_k, xs[1], T, k);
    mm(L->att_v, xs[2], T, v);
    mm(L->att_g, xs[4], T, g);
    for (int64_t i = 0; i < T * C; i++) g[i] = siluf_(g[i]);
    mm(L->decay_w1, xs[0], T, dl);
    for (int64_t i = 0; i < T * DW; i++) dl[i] = o_tanh(dl[i]);
    mm(L->decay_w2, dl, T, w);
    for (int64_t i = 0; i < T * C; i++) {
        float ww = w[i] + L->att_decay[i % C];
        w[i] = o_exp(-o_exp(ww));
    }
    wkv6(T, H, S, k, v, r, L->att_faaaa, w, 1, heads, y);
    group_norm(y, T, H, S, 64e-5f, L->att_lnx_w, L->att_lnx_b);
    for (int64_t i = 0; i < T * C; i++) y[i] = y[i] * g[i];
    mm(L->att_o, y, T, o);
    for (int64_t i = 0; i < T * C; i++) x[i] = x[i] + o[i];
    free(xa); free(xp); free(sx); free(xxx); free(lora); free(r); free(k); free(v); free(g); free(w);
    free(y); free(o); free(dl);
    for (int n = 0; n < 5; n++) free(xs[n]);
}

/* FFN v6, rwkv_graph.inc:513-531 */
static void ffn_v6(const oracle_model * m, const olayer * L, float * x, int64_t T, float * ffn_xx) {
    const int64_t C = m->n_embed, F = L->ffn_k->ne[1];
    float *xa = ALLOC(T * C), *xp = ALLOC(T * C), *xk = ALLOC(T * C), *xr = ALLOC(T * C);
    float *r = ALLOC(T * C), *k = ALLOC(T * F), *o = ALLOC(T * C);
    carry_x(x, T, C, L->ln2_w, L->ln2_b, ffn_xx, xa, xp);
    for (int64_t i = 0; i < T * C; i++) {
        const float s = xp[i] - xa[i];
        xk[i] = s * L->ffn_maa_k[i % C] + xa[i];
        xr[i] = s * L->ffn_maa_r[i % C] + xa[i];
    }
    mm(L->ffn_r, xr, T, r);
    mm(L->ffn_k, xk, T, k);
    for (int64_t i = 0; i < T * F; i++) {
        float kk = k[i] > 0.0f ? k[i] : 0.0f;
        k[i] = kk * kk;
    }
    mm(L->ffn_v, k, T, o);
    for (int64_t i = 0; i < T * C; i++) x[i] = x[i] + sigmoidf_(r[i]) * o[i];
    free(xa); free(xp); free(xk); free(xr); free(r); free(k); free(o);
}

static void layer_v7(const oracle_model * m, const olayer * L, float * x, int64_t T, float * st, float * v_first,
                     int layer_index) {
    const int64_t C = m->n_embed, H = m->head_count, S = m->head_size;
    const int64_t DW = L->w1->ne[1], DA = L->a1->ne[1], DG = L->g1->ne[1];
    float * att_xx = st + C, * heads = st + 2 * C;
    float *xa = ALLOC(T * C), *xp = ALLOC(T * C), *xs[6];
    float *r = ALLOC(T * C), *g = ALLOC(T * C), *a = ALLOC(T * C), *w = ALLOC(T * C), *k = ALLOC(T * C),
          *kk = ALLOC(T * C), *v = ALLOC(T * C), *y = ALLOC(T * C), *o = ALLOC(T * C), *nb = ALLOC(T * C),
          *bb = ALLOC(T * C);
    int64_t DMAX = DW > DA ? DW : DA;
    if (DG > DMAX) DMAX = DG;
    if (L->v1 && L->v1->ne[1] > DMAX) DMAX = L->v1->ne[1];
    float * tmp = ALLOC(T * DMAX);
    for (int n = 0; n < 6; n++) xs[n] = ALLOC(T * C);
    /* rwkv_graph.inc:387-482 */
    carry_x(x, T, C, L->ln1_w, L->ln1_b, att_xx, xa, xp);
    for (int n = 0; n < 6; n++)
        for (int64_t i = 0; i < T * C; i++) {
            const float s = xp[i] - xa[i];
            xs[n][i] = s * L->x_rwkvag[n * C + i % C] + xa[i];
        }
    /* order r, w, k, v, a, g */
    mm(L->att_r, xs[0], T, r);
    mm(L->g1, xs[5], T, tmp);
    for (int64_t i = 0; i < T * DG; i++) tmp[i] = sigmoidf_(tmp[i]);
    mm(L->g2, tmp, T, g);
    mm(L->a1, xs[4], T, tmp);
    mm(L->a2, tmp, T, a);
    for (int64_t i = 0; i < T * C; i++) a[i] = sigmoidf_(a[i] + L->a0[i % C]);
    mm(L->w1, xs[1], T, tmp);
    for (int64_t i = 0; i < T * DW; i++) tmp[i] = o_tanh(tmp[i]);
    mm(L->w2, tmp, T, w);
    for (int64_t i = 0; i < T * C; i++) w[i] = o_exp(sigmoidf_(w[i] + L->w0[i % C]) * -0.606531f);
    mm(L->att_k, xs[2], T, k);
    for (int64_t i = 0; i < T * C; i++) kk[i] = k[i] * L->k_k[i % C];
    /* rwkv_l2norm per head, rwkv_operators.inc:40-82 */
    for (int64_t t = 0; t < T; t++)
        for (int64_t h = 0; h < H; h++) {
            float * p = kk + t * C + h * S;
            float sum = 0.0f;
            if (g_variant & OV_GPU) {
                float sq[64];
                for (int64_t i = 0; i < S; i++) sq[i] = p[i] * p[i];
                sum = bfly_f(sq, (int)S);
            } else {
                for (int64_t i = 0; i < S; i++) sum += p[i] * p[i];
            }
            const float scale = 1.0f / fmaxf(sqrtf(sum), 1e-12f);
            for (int64_t i = 0; i < S; i++) p[i] = p[i] * scale;
        }
    for (int64_t i = 0; i < T * C; i++) {
        const float ka = k[i] * L->k_a[i % C];
        k[i] = k[i] + (a[i] * ka - ka);
    }
    mm(L->att_v, xs[3], T, v);
    if (layer_index == 0) {
        memcpy(v_first, v, sizeof(float) * (size_t)(T * C));
    } else {
        mm(L->v1, xs[3], T, tmp);
        mm(L->v2, tmp, T, o);
        for (int64_t i = 0; i < T * C; i++) v[i] = v[i] + (v_first[i] - v[i]) * sigmoidf_(o[i] + L->v0[i % C]);
    }
    for (int64_t i = 0; i < T * C; i++) {
        nb[i] = -kk[i];
        bb[i] = kk[i] * a[i];
    }
    wkv7(T, H, S, r, w, k, v, nb, bb, heads, y);
    group_norm(y, T, H, S, 64e-5f, L->att_lnx_w, L->att_lnx_b);
    for (int64_t t = 0; t < T; t++)
        for (int64_t h = 0; h < H; h++) {
            const int64_t o0 = t * C + h * S;
            float sum = 0.0f;
            if (g_variant & OV_GPU) {
                float pr[64];
                for (int64_t i = 0; i < S; i++) pr[i] = (k[o0 + i] * r[o0 + i]) * L->r_k[h * S + i];
                sum = bfly_f(pr, (int)S);
            } else {
                for (int64_t i = 0; i < S; i++) sum += (k[o0 + i] * r[o0 + i]) * L->r_k[h * S + i];
            }
            for (int64_t i = 0; i < S; i++) y[o0 + i] = y[o0 + i] + v[o0 + i] * sum;
        }
    for (int64_t i = 0; i < T * C; i++) y[i] = y[i] * g[i];
    mm(L->att_o, y, T, o);
    for (int64_t i = 0; i < T * C; i++) x[i] = x[i] + o[i];
    free(xa); free(xp); free(r); free(g); free(a); free(w); free(k); free(kk); free(v); free(y); free(o);
    free(nb); free(bb); free(tmp);
    for (int n = 0; n < 6; n++) free(xs[n]);
}

/* FFN v7, rwkv_graph.inc:533-543 */
static void ffn_v7(const oracle_model * m, const olayer * L, float * x, int64_t T, float * ffn_xx) {
    const int64_t C = m->n_embed, F = L->ffn_k->ne[1];
    float *xa = ALLOC(T * C), *xp = ALLOC(T * C), *xk = ALLOC(T * C), *k = ALLOC(T * F), *o = ALLOC(T * C);
    carry_x(x, T, C, L->ln2_w, L->ln2_b, ffn_xx, xa, xp);
    for (int64_t i = 0; i < T * C; i++) xk[i] = (xp[i] - xa[i]) * L->ffn_x_k[i % C] + xa[i];
    mm(L->ffn_k, xk, T, k);
    for (int64_t i = 0; i < T * F; i++) {
        float kk = k[i] > 0.0f ? k[i] : 0.0f;
        k[i] = kk * kk;
    }
    mm(L->ffn_v, k, T, o);
    for (int64_t i = 0; i < T * C; i++) x[i] = x[i] + o[i];
    free(xa); free(xp); free(xk); free(k); free(o);
}

/* Layers [l0, l1) over T tokens (the unit of a layer pipeline stage).  x_io /
 * vfirst_io: [T][C] residual stream and (v7) layer-0 values entering l0, replaced by the ones
 * leaving l1 - 1; with l0 == 0 the tokens are embedded instead (x_io / vfirst_io may then be
 * NULL).  Only the state slices of layers [l0, l1) change.  Head on the last token when
 * l1 == n_layer and logits_out is given. */
int oracle_eval_layers(const oracle_model * m, const uint32_t * tokens, size_t Tsz, uint32_t l0, uint32_t l1,
                       float * x_io, float * vfirst_io, const float * state_in, float * state_out,
                       float * logits_out) {
    const int64_t T = (int64_t)Tsz, C = m->n_embed;
    if (T <= 0 || l0 > l1 || l1 > m->n_layer) return 1;
    if (l0 == 0) {
        if (!tokens) return 2;
        for (int64_t t = 0; t < T; t++)
            if (tokens[t] >= m->n_vocab) return 2;
    } else if (!x_io || (m->major == 7 && !vfirst_io)) {
        return 1;
    }
    const int64_t SL = state_len(m);
    float * st = ALLOC(SL);
    if (state_in) memcpy(st, state_in, sizeof(float) * (size_t)SL); else oracle_init_state(m, st);
    float * x = ALLOC(T * C), * v_first = ALLOC(T * C);
    float * row = ALLOC(C);
    if (l0 == 0) {
        /* rwkv_graph.inc:654-658 / :786-790 */
        for (int64_t t = 0; t < T; t++) {
            oracle_dequantize_row((int)m->emb->type,
                                  m->emb->data + tensor_nbytes(m->emb->type, (uint64_t)tokens[t] * C), row, C);
            norm_row(row, x + t * C, C, 1e-5f, m->ln0_w, m->ln0_b);
        }
    } else {
        memcpy(x, x_io, sizeof(float) * (size_t)(T * C));
        if (m->major == 7) memcpy(v_first, vfirst_io, sizeof(float) * (size_t)(T * C));
    }
    const int64_t per_layer = m->major >= 5 ? C * (2 + m->head_size) : 5 * C;
    for (uint32_t i = l0; i < l1; i++) {
        const olayer * L = &m->layers[i];
        float * ls = st + i * per_layer;
        switch (m->major) {
            case 4: layer_v4(m, L, x, T, ls); ffn_v4_v5(m, L, x, T, ls); break;
            case 5: layer_v5(m, L, x, T, ls); ffn_v4_v5(m, L, x, T, ls); break;
            case 6: layer_v6(m, L, x, T, ls); ffn_v6(m, L, x, T, ls); break;
            case 7: layer_v7(m, L, x, T, ls, v_first, (int)i); ffn_v7(m, L, x, T, ls); break;
            default: break;
        }
    }
    if (logits_out && l1 == m->n_layer) {
        /* rwkv_graph.inc:704-708 / :850-854: head(LN(x[T-1])) */
        norm_row(x + (T - 1) * C, row, C, 1e-5f, m->lnout_w, m->lnout_b);
        mm(m->head, row, 1, logits_out);
    }
    if (x_io) memcpy(x_io, x, sizeof(float) * (size_t)(T * C));
    if (vfirst_io && m->major == 7) memcpy(vfirst_io, v_first, sizeof(float) * (size_t)(T * C));
    if (state_out) memcpy(state_out, st, sizeof(float) * (size_t)SL);
    free(st); free(x); free(v_first); free(row);
    return 0;
}

int oracle_eval(const oracle_model * m, const uint32_t * tokens, size_t Tsz, const float * state_in,
                float * state_out, float * logits_out) {
    return oracle_eval_layers(m, tokens, Tsz, 0, m->n_layer, NULL, NULL, state_in, state_out, logits_out);
}

/* ------------------------------------------------------------- quantizer */

/* rwkv_quantize.inc:1-13 */
static int needs_quant(const char * name) {
    static const char * skip[] = {"att.v1", "att.v2", "att.g1", "att.g2", "att.a1", "att.a2",
                                  "att.w1", "att.w2", "att.r_k"};
    if (strcmp(name, "emb.weight") == 0 || strcmp(name, "head.weight") == 0) return 0;
    for (size_t i = 0; i < sizeof(skip) / sizeof(skip[0]); i++)
        if (strstr(name, skip[i])) return 0;
    return 1;
}

int oracle_quantize_file(const char * in_path, const char * out_path, const char * format) {
    int out_type = -1;
    if (strcmp(format, "Q4_0") == 0) out_type = OT_Q4_0;
    else if (strcmp(format, "Q4_1") == 0) out_type = OT_Q4_1;
    else if (strcmp(format, "Q5_0") == 0) out_type = OT_Q5_0;
    else if (strcmp(format, "Q5_1") == 0) out_type = OT_Q5_1;
    else if (strcmp(format, "Q8_0") == 0) out_type = OT_Q8_0;
    if (out_type < 0) return 1;
    FILE * in = fopen(in_path, "rb");
    if (!in) return 2;
    struct stat st;
    fstat(fileno(in), &st);
    uint32_t hdr[6];
    if (fread(hdr, 4, 6, in) != 6 || hdr[0] != 0x67676d66u || (hdr[5] != OT_FP32 && hdr[5] != OT_FP16)) {
        fclose(in);
        return 3;
    }
    FILE * out = fopen(out_path, "wb");
    if (!out) {
        fclose(in);
        return 4;
    }
    hdr[1] = 101;
    hdr[5] = (uint32_t)out_type;
    fwrite(hdr, 4, 6, out);
    int rc = 0;
    while (ftell(in) < (long)st.st_size) {
        uint32_t th[3], ne[3] = {1, 1, 1};
        if (fread(th, 4, 3, in) != 3 || th[0] < 1 || th[0] > 3 || fread(ne, 4, th[0], in) != th[0]) {
            rc = 5;
            break;
        }
        char * name = (char *)calloc(th[1] + 1, 1);
        if (fread(name, 1, th[1], in) != th[1]) {
            free(name);
            rc = 5;
            break;
        }
        const uint64_t n = (uint64_t)ne[0] * ne[1] * ne[2];
        const size_t nb = tensor_nbytes(th[2], n);
        uint8_t * data = (uint8_t *)malloc(nb ? nb : 1);
        if (fread(data, 1, nb, in) != nb) {
            free(name);
            free(data);
            rc = 5;
            break;
        }
        if ((th[2] == OT_FP32 || th[2] == OT_FP16) && th[0] == 2 && needs_quant(name)) {
            float * f = (float *)malloc(sizeof(float) * (size_t)n);
            oracle_dequantize_row((int)th[2], data, f, (int64_t)n);
            const size_t qb = tensor_nbytes((uint32_t)out_type, n);
            uint8_t * q = (uint8_t *)malloc(qb);
            for (uint32_t r = 0; r < ne[1]; r++)
                oracle_quantize_row(out_type, f + (size_t)r * ne[0],
                                    q + (size_t)r * (ne[0] / QK) * oracle_block_bytes(out_type), ne[0]);
            th[2] = (uint32_t)out_type;
            fwrite(th, 4, 3, out);
            fwrite(ne, 4, th[0], out);
            fwrite(name, 1, th[1], out);
            fwrite(q, 1, qb, out);
            free(f);
            free(q);
        } else {
            fwrite(th, 4, 3, out);
            fwrite(ne, 4, th[0], out);
            fwrite(name, 1, th[1], out);
            fwrite(data, 1, nb, out);
        }
        free(name);
        free(data);
    }
    fclose(in);
    fclose(out);
    return rc;
}
