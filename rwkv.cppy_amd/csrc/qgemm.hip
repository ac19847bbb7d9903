// qgemm.hip -- token-batched dequant GEMM for the sequence path (T > 1) on int8 MFMA.
//
// Y[t][m] = sum_b d_w[m,b] d_x[t,b] sumi(m,t,b) (+ m_w s_x for the _1 formats), the ggml block
// arithmetic of rwkv_graph.inc's ggml_mul_mat calls with Q8_0/Q8_1 activations.  One
// v_mfma_i32_16x16x32_i8 is exactly one 32-weight quantization block, so the MFMA produces the
// exact integer block dot sumi for a 16x16 (rows x tokens) tile; the fp32 scale arithmetic
// runs in the epilogue of every block and reproduces the decode matvec's association bit for
// bit: the blocks of class l = b mod 64 (lane l of k_mv / k_mm) are chained with fmaf in
// ascending b, and the 64 class sums are folded with wave_sum63's perfect binary tree (a binary
// counter over the classes).  So serial decode and sequence evaluation stay bit-identical.
//
// Operands come as tile records (common.hpp qg_*): per (row tile, block) one contiguous weight
// record, per (64-token tile, block) one contiguous activation record, so every copy
// instruction moves 1 KiB of consecutive bytes.  Workgroup = 4 waves as 2 (rows) x 2 (tokens)
// over a 32*TI-row x 64-token tile; a wave owns TI 16-row tiles x 2 16-token tiles.  Blocks are
// consumed in class-major order in chunks of 8 steps; each chunk's records are copied
// global->LDS (LDS DMA) by the four waves while the previous chunk is computed from the other
// LDS buffer, and within a chunk the LDS operands of step k+1 are read while step k's epilogue
// runs.
#include "device_common.hpp"
#include "kernels.hpp"

#include <stdio.h>
#include <stdlib.h>
#include <type_traits>

// m0 in the copy asm's clobber list is a reserved register: the compiler re-sets m0 before each of
// its own uses (none in this file besides these copies)
#pragma clang diagnostic ignored "-Winline-asm"

namespace rwkvmi {

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

// Global->LDS copy (LDS DMA) of one 1-KiB piece: buffer_load_dwordx4 ... lds puts lane i's 16
// bytes from base + soff + voff + OFF at LDS m0 + OFF + 16 i (tools/bufdma_check.hip).  Issued as
// inline asm on purpose: the compiler cannot tell a copy into one LDS buffer from reads of the
// other and would drain vmcnt before every LDS read; the kernel orders the copies itself
// (s_waitcnt vmcnt(0) + barrier per chunk, qg_chunk_done).  M0 is written in the same statement
// (the compiler does not preserve it) and needs one wait state before the load.
template <int OFF>
__device__ __forceinline__ void qg_bdma(v4i_t rsrc, unsigned soff, unsigned m0, unsigned voff) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen offset:%4 lds" ::"v"(voff),
                 "s"(m0), "s"(rsrc), "s"(soff), "i"(OFF)
                 : "m0");
}

// raw buffer descriptor over [base, base + 4 GiB) (gfx9 dword3 0x00020000)
__device__ __forceinline__ v4i_t qg_rsrc(const void * base) {
    v4i_t r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned long)base);
    r.y = __builtin_amdgcn_readfirstlane((int)((unsigned long)base >> 32));
    r.z = -1;
    r.w = 0x00020000;
    return r;
}

// One record of BYTES into LDS at m0: full 1-KiB pieces plus a partial last piece
template <int BYTES, int P = 0>
__device__ __forceinline__ void qg_record(v4i_t rsrc, unsigned soff, unsigned m0, int lane) {
    if constexpr (P * 1024 < BYTES) {
        if constexpr ((P + 1) * 1024 <= BYTES) {
            qg_bdma<P * 1024>(rsrc, soff, m0, lane * 16);
        } else if (lane * 16 < BYTES - P * 1024) {
            qg_bdma<P * 1024>(rsrc, soff, m0, lane * 16);
        }
        qg_record<BYTES, P + 1>(rsrc, soff, m0, lane);
    }
}

// All of this wave's copies have landed; the barrier then publishes every wave's copies.
__device__ __forceinline__ void qg_chunk_done() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

constexpr int QG_STEPS = 8;  // blocks per chunk

template <int WF>
struct QGLayout {
    static constexpr bool ONE = qg_one(WF);
    static constexpr int TI = 2;
    static constexpr int ROWS = qg_rows(WF);        // = 32 * TI
    static constexpr int WB = qg_w_bytes(WF);       // weight record
    static constexpr int AB = qg_a_bytes(ONE);      // activation record (stride)
    static constexpr int AC = QG_A_S;               // of which copied: the int8 values and d (Q8_1's s
                                                    // feeds k_qg_msum, not this kernel)
    static constexpr int STEP = WB + AC;            // LDS bytes per step: [weight rec][act rec]
    static constexpr int BUF = STEP * QG_STEPS;
    static constexpr int WP = (WB + 1023) / 1024;   // copy instructions per record
    static constexpr int AP = (AC + 1023) / 1024;
    static constexpr int JOBS = WP + AP;
    static_assert(ROWS == 32 * TI && WB % 16 == 0 && AB % 16 == 0 && AC % 16 == 0, "qgemm layout");
};

// Class-major walk over the blocks: class l (= b mod 64) has n = q + (l < rem) blocks, q = nb/64,
// rem = nb%64; step s of the walk is block l + 64 u.  Scalar state, advanced one step at a time.
struct QGWalk {
    int q, rem, l, u, n;
    __device__ __forceinline__ void init(int nb, int l0 = 0) {
        q = nb >> 6;
        rem = nb & 63;
        l = l0;
        u = 0;
        n = q + (l0 < rem ? 1 : 0);
    }
    __device__ __forceinline__ int block() const { return l + 64 * u; }
    __device__ __forceinline__ void next() {
        if (++u == n) {
            l++;
            u = 0;
            n = q + (l < rem ? 1 : 0);
        }
    }
};

// This wave's share of chunk c: steps 8c + wave and 8c + wave + 4 (the walk is at the first of
// them and is left at 8(c+1) + wave).
template <int WF>
__device__ __forceinline__ void qg_load_chunk(v4i_t rw, v4i_t ra, unsigned lds_buf, int c, QGWalk & wk, int nsteps,
                                              int wave, int lane) {
    using Lt = QGLayout<WF>;
#pragma unroll
    for (int h2 = 0; h2 < 2; h2++) {
        const int k = wave + 4 * h2;
        if (c * QG_STEPS + k < nsteps) {
            const int b = wk.block();
            const unsigned m = lds_buf + k * Lt::STEP;
            qg_record<Lt::WB>(rw, (unsigned)(b * Lt::WB), m, lane);
            qg_record<Lt::AC>(ra, (unsigned)(b * Lt::AB), m + Lt::WB, lane);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) wk.next();
    }
}

// LDS operands of one step for one wave
template <int TI>
struct QGOps {
    long af[TI], xf[2];
    float4 sd[TI];  // d of the 4 D-layout rows 4h..4h+3 of each 16-row tile
    float dx[2];
};

// The 8-byte operand reads stay single ds_read_b64 (2 LDS cycles, 64 banks): the compiler would
// otherwise pair reads of consecutive steps into ds_read2st64_b64, which the LDS serves as two
// 16-lane-group accesses over 32 banks (8 cycles per pair, and tokens t / t + 8 of the activation
// record then share banks).  QG_MERGED_READS restores the compiler's pairing (A/B builds).
#ifdef QG_MERGED_READS
typedef const long qg_op_t;
#else
typedef __attribute__((address_space(3))) const volatile long qg_op_t;
#endif

template <int WF>
__device__ __forceinline__ void qg_read_ops(const char * sp, QGOps<QGLayout<WF>::TI> & o, int wr, int wt, int r16,
                                            int h) {
    using Lt = QGLayout<WF>;
#pragma unroll
    for (int i = 0; i < Lt::TI; i++) {
        o.af[i] = *(qg_op_t *)(sp + qg_w_off(wr + 16 * i + r16, h * 8));  // int8 row, k = 8h..8h+7
        const int ro = wr + 16 * i + 4 * h;
        o.sd[i] = *(const float4 *)(sp + qg_w_d(WF) + ro * 4);
    }
    const char * ap = sp + Lt::WB;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int tl = wt + 16 * j + r16;
        o.xf[j] = *(qg_op_t *)(ap + (h >> 1) * QG_TOK * 16 + tl * 16 + (h & 1) * 8);
        o.dx[j] = *(const float *)(ap + QG_A_D + tl * 4);
    }
}

typedef float qf2_t __attribute__((ext_vector_type(2)));

// The MFMA accumulates each block's integer dot onto QG_BIAS = 0x4B400000 (1.5 * 2^23 as a float),
// so the result read as a float is 12582912 + sumi exactly (|sumi| < 2^22), and one packed
// subtraction recovers (float)sumi for two outputs: no per-output int->float conversion.
constexpr int QG_BIAS = 0x4B400000;
constexpr float QG_BIAS_F = 12582912.0f;

// The TI x 2 MFMAs of one step (one quantization block) from this step's LDS operands
template <int TI>
__device__ __forceinline__ void qg_mfma(const QGOps<TI> & cur, v4i_t (&sv)[TI][2]) {
    const v4i_t bias = {QG_BIAS, QG_BIAS, QG_BIAS, QG_BIAS};
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) sv[i][j] = __builtin_amdgcn_mfma_i32_16x16x32_i8(cur.af[i], cur.xf[j], bias, 0, 0, 0);
}

// The fp32 block epilogue: acc = fma(d_w * d_x, sumi, acc), rows in pairs (packed f32: bitwise the
// scalar operations, tools/pk_probe.hip); FIRST: the class's first block (its chain starts from 0)
template <bool FIRST, int TI>
__device__ __forceinline__ void qg_epi(const QGOps<TI> & cur, const v4i_t (&sv)[TI][2], float (&acc)[TI][2][4]) {
    const qf2_t nbias = {-QG_BIAS_F, -QG_BIAS_F};
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int qp = 0; qp < 2; qp++) {
            const qf2_t dw = qp ? qf2_t{cur.sd[i].z, cur.sd[i].w} : qf2_t{cur.sd[i].x, cur.sd[i].y};
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const qf2_t dx = {cur.dx[j], cur.dx[j]};
                const qf2_t si = qf2_t{__int_as_float(sv[i][j][2 * qp]), __int_as_float(sv[i][j][2 * qp + 1])} + nbias;
                const qf2_t a0 = FIRST ? qf2_t{0.0f, 0.0f} : qf2_t{acc[i][j][2 * qp], acc[i][j][2 * qp + 1]};
                const qf2_t a = __builtin_elementwise_fma(dw * dx, si, a0);
                acc[i][j][2 * qp] = a.x;
                acc[i][j][2 * qp + 1] = a.y;
            }
        }
}

// y[t][m] = epi(total + t2), t2 = the m*s total (m2, _1 formats; k_qg_msum) or +0.0f, as k_mm's
// red + red2.  A lane holds rows 4h..4h+3 of one token: one 16-byte access per (token, 4 rows)
// when aligned.
template <int TI>
__device__ __forceinline__ void qg_store(const MMEntry & E, const float * m2, int T, int M, int tok0, int row0, int wt,
                                         int wr, int r16, int h, const float (&tot)[TI][2][4]) {
    if constexpr (TI == 2) {
        if (E.fuse_emit) {
            // The wave's 32 rows (wr % 32 == 0) of a token are one quantization block of the next
            // matmul's input: lanes r16 + 16 h hold rows 16 i + 4 h + q.  quant32 / store32's values:
            // amax and sum over the block by xor-16/32 lane exchanges (order-free), ggml rounding.
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int t = tok0 + wt + 16 * j + r16;
                const int tc = min(t, T - 1);
                float v[2][4];
                float am = 0.0f;
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const int mb = row0 + wr + 16 * i + 4 * h;
                    float t2q[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                    if (m2)
#pragma unroll
                        for (int q = 0; q < 4; q++) t2q[q] = m2[(size_t)(mb + q) * T + tc];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        v[i][q] = apply_epi_v(E, mb + q, tot[i][j][q] + t2q[q], 0.0f, 0.0f);
                        am = fmaxf(am, fabsf(v[i][q]));
                    }
                }
                am = fmaxf(am, __shfl_xor(am, 16));
                am = fmaxf(am, __shfl_xor(am, 32));
                const float d = am / 127.f;
                const float id = (am != 0.0f) ? 127.f / am : 0.0f;
                uint32_t packed[2];
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    packed[i] = 0;
#pragma unroll
                    for (int q = 0; q < 4; q++) packed[i] |= ((uint32_t)(int)rintf(v[i][q] * id) & 0xffu) << (8 * q);
                }
                if (t < T) {
                    uint8_t * rec = E.out.tq + ((size_t)(t / QG_TOK) * (M >> 5) + ((row0 + wr) >> 5)) * qg_a_bytes(false);
                    const int tl = t % QG_TOK;
#pragma unroll
                    for (int i = 0; i < 2; i++) *(uint32_t *)(rec + i * QG_TOK * 16 + tl * 16 + 4 * h) = packed[i];
                    if (h == 0) ((float *)(rec + QG_A_D))[tl] = f16_round(d);
                }
            }
            return;
        }
    }
    const bool vec = ((E.ldy | M) & 3) == 0 && (((uintptr_t)E.y | (uintptr_t)E.aux) & 15) == 0;
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int t = tok0 + wt + 16 * j + r16;
            const int m0 = row0 + wr + 16 * i + 4 * h;
            if (t >= T || m0 >= M) continue;
            float acc[4];
#pragma unroll
            for (int q = 0; q < 4; q++) acc[q] = tot[i][j][q] + (m2 && m0 + q < M ? m2[(size_t)(m0 + q) * T + t] : 0.0f);
            float * yp = E.y + (size_t)t * E.ldy + m0;
            if (vec) {
                float4 yv = make_float4(0.f, 0.f, 0.f, 0.f), av = yv;
                if (epi_reads_y(E.epi)) yv = *(const float4 *)yp;
                if (epi_reads_aux(E.epi)) av = *(const float4 *)(E.aux + (size_t)t * E.ldy + m0);
                float4 o;
                o.x = apply_epi_v(E, m0, acc[0], yv.x, av.x);
                o.y = apply_epi_v(E, m0 + 1, acc[1], yv.y, av.y);
                o.z = apply_epi_v(E, m0 + 2, acc[2], yv.z, av.z);
                o.w = apply_epi_v(E, m0 + 3, acc[3], yv.w, av.w);
                *(float4 *)yp = o;
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (m0 + q < M) yp[q] = apply_epi(E, t, m0 + q, acc[q]);
            }
        }
}

// Split-K: one split's subtree sums to its entry's partials [S][T][M]
template <int TI>
__device__ __forceinline__ void qg_store_part(float * part, int sidx, int T, int M, int tok0, int row0, int wt, int wr,
                                              int r16, int h, const float (&sub)[TI][2][4]) {
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int t = tok0 + wt + 16 * j + r16;
            const int m0 = row0 + wr + 16 * i + 4 * h;
            if (t >= T) continue;
            float * pp = part + ((size_t)sidx * T + t) * M + m0;
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (m0 + q < M) pp[q] = sub[i][j][q];
        }
}

// Class-pair fold: the odd class (in c) closes N >= 1 levels of the binary counter: v = c, then
// v = st[k] + v for k < N, into st[N] (N < 6) or the total (N = 6).  Packed f32 over output pairs
// (v_pk_add_f32: per element the scalar add's bits; this file builds without the SLP vectorizer).
template <int TI, int N>
__device__ __forceinline__ void qg_fold(float (&st)[6][TI][2][4], const float (&c)[TI][2][4], float (&tot)[TI][2][4]) {
#pragma unroll
    for (int i = 0; i < TI; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                qf2_t v = {c[i][j][q], c[i][j][q + 1]};
#pragma unroll
                for (int kk = 0; kk < N; kk++) v = qf2_t{st[kk][i][j][q], st[kk][i][j][q + 1]} + v;
                if constexpr (N < 6) {
                    st[N][i][j][q] = v.x;
                    st[N][i][j][q + 1] = v.y;
                } else {
                    tot[i][j][q] = v.x;
                    tot[i][j][q + 1] = v.y;
                }
            }
}

// K = 2048 (64 blocks: every class is one block, the walk is block order): the same arithmetic
// as k_qgemm with the step bookkeeping resolved at compile time -- each 8-step chunk is
// straight-line code (the class-pair folds after steps 1, 3, 5 close 1, 2, 1 levels; after step
// 7, 3 + ctz(~chunk) levels), and the copy walk is blocks 8c + wave, 8c + wave + 4.
// SPLIT > 1 (split-K when a group has few tiles): workgroup s of a tile runs chunks
// [s * NCHL, (s + 1) * NCHL) -- a complete subtree of the perfect binary tree over the 64 classes --
// and stores that subtree sum (and, _1 formats, the m*s subtree) to its entry's partials;
// k_qg_combine adds the SPLIT subtrees with the tree's top levels and applies the epilogue (and
// the emission), so results equal the unsplit kernel bit for bit.
template <int WF, int SPLIT = 1>
__global__ __launch_bounds__(256) void k_qgemm_k64(MMGroup g) {
    using Lt = QGLayout<WF>;
    constexpr bool ONE = Lt::ONE;
    constexpr int TI = Lt::TI;
    constexpr int NB = 64, NCH = NB / QG_STEPS, NCHL = NCH / SPLIT;
    __shared__ __attribute__((aligned(16))) char smem[2][Lt::BUF];
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MMEntry & E = g.e[e];
    const int M = E.W.M, T = g.T;
    const int tilesT = (T + QG_TOK - 1) / QG_TOK;
    const int local0 = (int)blockIdx.x - E.block0;
    const int sidx = local0 % SPLIT, local = local0 / SPLIT, ch0 = sidx * NCHL;
    const int mtile = local / tilesT, ttile = local % tilesT;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r16 = lane & 15, h = lane >> 4;
    const int row0 = mtile * Lt::ROWS, tok0 = ttile * QG_TOK;
    const int wr = (wave & 1) * 16 * TI, wt = (wave >> 1) * 32;
    const v4i_t rw = qg_rsrc(E.W.gt + (size_t)mtile * NB * Lt::WB);
    const v4i_t ra = qg_rsrc(E.in.tq + (size_t)ttile * NB * Lt::AB);
    const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long)(lds_void_t *)&smem[0][0]);
    auto load = [&](int c, unsigned buf) {
#pragma unroll
        for (int h2 = 0; h2 < 2; h2++) {
            const int k = wave + 4 * h2, b = c * QG_STEPS + k;
            const unsigned m = buf + k * Lt::STEP;
            qg_record<Lt::WB>(rw, (unsigned)(b * Lt::WB), m, lane);
            qg_record<Lt::AC>(ra, (unsigned)(b * Lt::AB), m + Lt::WB, lane);
        }
    };
    const float * m2 = ONE ? g.m2 + E.moff : nullptr;
    float st[6][TI][2][4];
    float tot[TI][2][4];
    float c[TI][2][4];
    load(ch0, lds0);
    qg_chunk_done();
    if (NCHL > 1) load(ch0 + 1, lds0 + Lt::BUF);
    QGOps<TI> cur;
    qg_read_ops<WF>(smem[0], cur, wr, wt, r16, h);
#pragma unroll 1
    for (int ch = 0; ch < NCHL; ch++) {  // local chunk index (the subtree's own tree)
        const char * buf = smem[ch & 1];
#pragma unroll
        for (int k = 0; k < QG_STEPS; k++) {
            v4i_t sv[TI][2];
            qg_mfma<TI>(cur, sv);
            QGOps<TI> nxt = cur;
            if (k + 1 < QG_STEPS) qg_read_ops<WF>(buf + (k + 1) * Lt::STEP, nxt, wr, wt, r16, h);
            if (k & 1) {
                qg_epi<true, TI>(cur, sv, c);
                if (k == 1 || k == 5) qg_fold<TI, 1>(st, c, tot);
                else if (k == 3) qg_fold<TI, 2>(st, c, tot);
                else {
                    switch (__builtin_ctz(~ch)) {
                        case 0: qg_fold<TI, 3>(st, c, tot); break;
                        case 1: qg_fold<TI, 4>(st, c, tot); break;
                        case 2: qg_fold<TI, 5>(st, c, tot); break;
                        default: qg_fold<TI, 6>(st, c, tot); break;
                    }
                }
            } else {
                qg_epi<true, TI>(cur, sv, st[0]);
            }
            cur = nxt;
        }
        if (ch + 1 < NCHL) {
            qg_chunk_done();  // chunk ch+1 has landed and buffer ch&1 is free
            if (ch + 2 < NCHL) load(ch0 + ch + 2, lds0 + (ch & 1) * Lt::BUF);
            qg_read_ops<WF>(smem[(ch + 1) & 1], cur, wr, wt, r16, h);
        }
    }
    if constexpr (SPLIT == 1) {
        qg_store<TI>(E, m2, T, M, tok0, row0, wt, wr, r16, h, tot);
    } else {
        // the subtree over this split's 8 * NCHL classes sits at level 3 + log2(NCHL)
        constexpr int LEV = NCHL == 1 ? 3 : NCHL == 2 ? 4 : 5;
        (void)m2;
        qg_store_part<TI>(g.part + E.poff, sidx, T, M, tok0, row0, wt, wr, r16, h, st[LEV]);
    }
}

// Split-K combine for a whole group: the top of the class tree over the SPLIT subtrees (8: three
// levels, 4: two), then qg_store's total (+ 0.0f, or + the m*s total for the _1 formats), the
// entry's epilogue, y, and -- for emitting entries -- the next matmul's input (emit32: one
// quantization block per 32 consecutive rows of a token, one half-wave).
template <int SPLIT, bool ONE>
__global__ __launch_bounds__(256) void k_qg_combine(MMGroup g) {
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].cblock0) e++;
    const MMEntry & E = g.e[e];
    const int M = E.W.M, T = g.T;
    const size_t i = (size_t)((int)blockIdx.x - E.cblock0) * 256 + threadIdx.x;
    if (i >= (size_t)T * M) return;  // T * M % 32 == 0: half-waves stay whole
    const int t = (int)(i / M), m = (int)(i % M);
    const float * pp = g.part + E.poff + (size_t)t * M + m;
    const size_t ss = (size_t)T * M;
    auto tree = [&](const float * p) {
        float v[SPLIT];
#pragma unroll
        for (int s = 0; s < SPLIT; s++) v[s] = p[s * ss];
        if constexpr (SPLIT == 8) return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
        else if constexpr (SPLIT == 2) return v[0] + v[1];
        else return (v[0] + v[1]) + (v[2] + v[3]);
    };
    const float tot = tree(pp);
    float acc;
    if constexpr (ONE) acc = tot + g.m2[E.moff + (size_t)m * T + t];
    else acc = tot + 0.0f;
    const float v = apply_epi(E, t, m, acc);
    if (E.y) E.y[(size_t)t * E.ldy + m] = v;  // (k_fmm's emit-only entries have none)
    if (E.emit) emit32(E.out, t, m, v);
}

// SPLIT > 1: workgroup s of a tile walks classes [s * 64 / SPLIT, (s + 1) * 64 / SPLIT) only -- a
// complete subtree of the class tree -- and stores the subtree sums (qg_store_part) for k_qg_combine.
template <int WF, int SPLIT = 1>
__global__ __launch_bounds__(256) void k_qgemm(MMGroup g) {
    using Lt = QGLayout<WF>;
    constexpr bool ONE = Lt::ONE;
    constexpr int TI = Lt::TI;
    constexpr int CPS = 64 / SPLIT;  // classes per split
    __shared__ __attribute__((aligned(16))) char smem[2][Lt::BUF];
    int e = 0;
#pragma unroll 1
    while (e + 1 < g.n && (int)blockIdx.x >= g.e[e + 1].block0) e++;
    const MMEntry & E = g.e[e];
    const int M = E.W.M, K = E.W.K, T = g.T, nb = K >> 5;
    const int tilesT = (T + QG_TOK - 1) / QG_TOK;
    const int local0 = (int)blockIdx.x - E.block0;
    const int sidx = local0 % SPLIT, local = local0 / SPLIT, l0 = sidx * CPS;
    const int mtile = local / tilesT, ttile = local % tilesT;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r16 = lane & 15, h = lane >> 4;
    const int row0 = mtile * Lt::ROWS, tok0 = ttile * QG_TOK;
    const int wr = (wave & 1) * 16 * TI, wt = (wave >> 1) * 32;  // this wave's tile-local row / token
    const v4i_t rw = qg_rsrc(E.W.gt + (size_t)mtile * nb * Lt::WB);
    const v4i_t ra = qg_rsrc(E.in.tq + (size_t)ttile * nb * Lt::AB);
    const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long)(lds_void_t *)&smem[0][0]);
    const int cq = nb >> 6, crem = nb & 63;  // class sizes for the consumer
    // this split's steps: the blocks of classes [l0, l0 + CPS)
    const int nsteps = CPS * cq + min(max(crem - l0, 0), CPS);
    QGWalk ld;  // the loader's walk (this wave's steps)
    ld.init(nb, l0);
    for (int i = 0; i < wave; i++) ld.next();

    // Per output: class sums in a binary counter (wave_sum63's tree).  Classes are walked in
    // pairs: the even class accumulates straight into level 0 (st[0]), the odd one into c, and
    // the pair then folds upward -- no copies or resets of accumulators between classes (each
    // class's first block starts its chain from 0 in a peeled step).
    float st[6][TI][2][4];
    float tot[TI][2][4];
    float c[TI][2][4];
    const int nchunks = (nsteps + QG_STEPS - 1) / QG_STEPS;

    int k = 0, cb = 0, cn = 1;  // step within the chunk, its buffer, next chunk to issue
    // one block: MFMAs from this step's LDS operands, then the fp32 block epilogue into acc
    // LDS operands of the current step live in registers (cur); the next step's are read while
    // this step's epilogue runs, except across a chunk boundary (its buffer is not ready yet).
    QGOps<TI> cur;
    auto step = [&](auto first, float (&acc)[TI][2][4]) {
        constexpr bool FIRST = decltype(first)::value;
        // Chunk consumed: switch buffers (wave-uniform).  Done before this step's MFMAs, not
        // after them, so no branch separates an MFMA from the reads of its result.
        if (k == QG_STEPS) {
            k = 0;
            qg_chunk_done();  // the next chunk has landed and this buffer is free
#if defined(QG_PROBE) && QG_PROBE == 2
            if (cn < nchunks && cn < 2)  // tools/gemm_probe: compute only
#else
            if (cn < nchunks)
#endif
                qg_load_chunk<WF>(rw, ra, lds0 + cb * Lt::BUF, cn, ld, nsteps, wave, lane);
            cn++;
            cb ^= 1;
            qg_read_ops<WF>(smem[cb], cur, wr, wt, r16, h);
        }
#if defined(QG_PROBE) && QG_PROBE == 1
        if (0)  // tools/gemm_probe: copies only
#endif
        {
            v4i_t sv[TI][2];
            qg_mfma<TI>(cur, sv);
            QGOps<TI> nxt = cur;
            if (k + 1 < QG_STEPS) qg_read_ops<WF>(smem[cb] + (k + 1) * Lt::STEP, nxt, wr, wt, r16, h);
            qg_epi<FIRST, TI>(cur, sv, acc);
            cur = nxt;
        }
        k++;
    };
    using T1 = std::integral_constant<bool, true>;
    using T0 = std::integral_constant<bool, false>;
    auto zero_acc = [&](float (&acc)[TI][2][4]) {
#pragma unroll
        for (int i = 0; i < TI; i++)
#pragma unroll
            for (int j = 0; j < 2; j++)
#pragma unroll
                for (int q = 0; q < 4; q++) acc[i][j][q] = 0.0f;
    };
    // all blocks of class l into acc (a class without blocks, nb < 64, is a zero leaf)
    auto run_class = [&](int l, float (&acc)[TI][2][4]) {
        const int n = cq + (l < crem ? 1 : 0);
        if (n == 0) {
            zero_acc(acc);
            return;
        }
        step(T1{}, acc);
        for (int u = 1; u < n; u++) step(T0{}, acc);
    };

    // odd class l (in c) closes ctz(~l) >= 1 levels: v = c, then v = st[k] + v for k < N
#define QG_CASE(N, DST)                                                           \
    case N: {                                                                     \
        _Pragma("unroll") for (int i = 0; i < TI; i++)                            \
        _Pragma("unroll") for (int j = 0; j < 2; j++)                             \
        _Pragma("unroll") for (int q = 0; q < 4; q += 2) {                        \
            qf2_t v = {c[i][j][q], c[i][j][q + 1]};                               \
            for (int kk = 0; kk < N; kk++)                                        \
                v = qf2_t{st[kk][i][j][q], st[kk][i][j][q + 1]} + v;              \
            DST[i][j][q] = v.x;                                                   \
            DST[i][j][q + 1] = v.y;                                               \
        }                                                                         \
        break;                                                                    \
    }

    if (nchunks > 0) qg_load_chunk<WF>(rw, ra, lds0, 0, ld, nsteps, wave, lane);
    qg_chunk_done();
    if (nchunks > 1) qg_load_chunk<WF>(rw, ra, lds0 + Lt::BUF, 1, ld, nsteps, wave, lane);
    cn = 2;
    qg_read_ops<WF>(smem[0], cur, wr, wt, r16, h);
    for (int pr = 0; pr < CPS / 2; pr++) {  // pairs of this split's classes; folds by the relative index
        run_class(l0 + 2 * pr, st[0]);
        run_class(l0 + 2 * pr + 1, c);
        switch (__builtin_ctz(~(2 * pr + 1))) {
            QG_CASE(1, st[1])
            QG_CASE(2, st[2])
            QG_CASE(3, st[3])
            QG_CASE(4, st[4])
            QG_CASE(5, st[5])
            default:
            QG_CASE(6, tot)
        }
    }
#undef QG_CASE
    // copies of a partial last chunk (or of none) were never waited for: drain before exit
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    if constexpr (SPLIT == 1) {
        qg_store<TI>(E, ONE ? g.m2 + E.moff : nullptr, T, M, tok0, row0, wt, wr, r16, h, tot);
    } else {
        constexpr int LEV = SPLIT == 8 ? 3 : SPLIT == 4 ? 4 : 5;  // the subtree of CPS classes
        qg_store_part<TI>(g.part + E.poff, sidx, T, M, tok0, row0, wt, wr, r16, h, st[LEV]);
    }
}

// The _1 formats' m*s chains, in the matvec's association: for class l (= b mod 64) the chain
// acc = acc + m_w[b] * s_x[b] over b = l + 64 u ascending, from 0; the 64 class sums folded by
// wave_sum63's tree (the binary counter of the GEMM).  Independent of the int8 dot, so it runs as
// its own VALU pass ahead of the GEMM -- whose tiles then carry one chain, 64 rows, like _0 -- and
// the GEMM epilogue (or k_qg_combine) adds these totals: the same y bits.
// Workgroup = 64 rows x 64 tokens (lane: 4 rows x 4 tokens; wave w: tokens 16w..16w+15).  Stages of 8 classes: all
// their blocks' m_w (64 rows) and s_x (32 tokens) are copied to LDS with coalesced loads -- the next
// stage's in flight while this one is accumulated -- so a block costs a lane two b128 reads (4 rows'
// m_w, 4 tokens' s_x) for 16 multiply-adds.
// Output m2[row][token] (row-major over rows).
// The m*s pass's arithmetic in packed f32 (v_pk_mul_f32 / v_pk_add_f32: per element the scalar
// operations' bits, tools/pk_probe.hip; this file builds without the SLP vectorizer, so the packing
// is spelled out): acc[j] = acc[j] + w * x[j] over pairs of outputs, and the class-tree folds.
// m_w and s_x are fp16 values, so w * x is exact in f32 and acc + w * x IS fmaf(w, x, acc): one
// v_pk_fma_f32 per pair instead of a v_pk_mul_f32 and a v_pk_add_f32 (the same bits).
template <int N>
__device__ __forceinline__ void qm_mac_row(float * acc, float w, const float (&x)[N]) {
    const qf2_t w2 = {w, w};
#pragma unroll
    for (int j = 0; j < N; j += 2) {
        qf2_t a = {acc[j], acc[j + 1]};
        const qf2_t x2 = {x[j], x[j + 1]};
        a = __builtin_elementwise_fma(w2, x2, a);  // = a + w * x bit for bit: m_w * s_x is exact
        acc[j] = a.x;
        acc[j + 1] = a.y;
    }
}
// v = st[kk] + v for kk < NL, into st[NL] (NL < 6) or st[0] (NL = 6: the total), pairs of outputs
template <int NL, int NO>
__device__ __forceinline__ void qm_close(float (&st)[6][NO], const float (&acc)[NO]) {
#pragma unroll
    for (int k = 0; k < NO; k += 2) {
        qf2_t v = {acc[k], acc[k + 1]};
#pragma unroll
        for (int kk = 0; kk < NL; kk++) v = qf2_t{st[kk][k], st[kk][k + 1]} + v;
        st[NL < 6 ? NL : 0][k] = v.x;
        st[NL < 6 ? NL : 0][k + 1] = v.y;
    }
}

constexpr int QM_CLS = 8;  // classes per stage
// NMAX = blocks per class rounded up to 1 / 2 / 4 / 8 (K <= 16384); slot (u, lc) at u * 8 + lc holds
// m_w of the workgroup's 64 rows and s_x of its 32 tokens for block lc + 8 sg + 64 u
// FULL: every class has at least one block (K >= 2048): a class's chain starts with its first
// multiply-add on a literal 0 -- no zeroed accumulators.
template <int NMAX, bool FULL>
__global__ __launch_bounds__(256) void k_qg_msum(MMGroup g) {
    constexpr int NSLOT = QM_CLS * NMAX;
    __shared__ __attribute__((aligned(16))) float qw[2][NSLOT][64];
    __shared__ __attribute__((aligned(16))) float qx[2][NSLOT][64];
    const int T = g.T, tgs = (T + 63) / 64;
    int e = 0, base = 0;
#pragma unroll 1
    for (; e + 1 < g.n; e++) {
        const int n_e = (g.e[e].W.M + 63) / 64 * tgs;
        if ((int)blockIdx.x < base + n_e) break;
        base += n_e;
    }
    const MMEntry & E = g.e[e];
    const int M = E.W.M, nb = E.W.K >> 5, MS = qm_stride(M);
    const int local = (int)blockIdx.x - base;
    const int rt = local / tgs, tg = local % tgs;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rq = lane & 15, tq = lane >> 4;  // this lane: rows 4 rq + r, tokens 16 wave + 4 tq + c
    const int r0 = rt * 64, tok0 = tg * 64;
    const int cq = nb >> 6, crem = nb & 63;
    const size_t AB = qg_a_bytes(true);
    // loaders: slot wave + 4 k -- m_w of row lane, s_x of token lane.  A block past its class's count
    // is clamped (loaded, never read).
    const float * wrow = E.W.mt + min(r0 + lane, MS - 1);
    const int tx = min(tok0 + lane, T - 1);
    const float * xrow = (const float *)(E.in.tq + (size_t)(tx / QG_TOK) * nb * AB + QG_A_S) + tx % QG_TOK;
    constexpr int LS = NSLOT / 4;
    float lw[LS], lx[LS];
    auto blk = [&](int sg, int sl) {
        const int lc = sl & 7, u = sl >> 3, l = sg * QM_CLS + lc;
        return min(u < cq + (l < crem ? 1 : 0) ? l + 64 * u : l, nb - 1);
    };
    auto gload = [&](int sg) {
#pragma unroll
        for (int k = 0; k < LS; k++) {
            const int b = blk(sg, wave + 4 * k);
            lw[k] = wrow[(size_t)b * MS];
            lx[k] = xrow[(size_t)b * (AB / 4)];
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int k = 0; k < LS; k++) {
            qw[buf][wave + 4 * k][lane] = lw[k];
            qx[buf][wave + 4 * k][lane] = lx[k];
        }
    };
    float st[6][16], acc[16];
#pragma unroll
    for (int k = 0; k < 16; k++) acc[k] = 0.0f;
#define QM_CLOSE(N)                                                   \
    case N: {                                                         \
        qm_close<N, 16>(st, acc);  /* N = 6: the total, into st[0] */ \
        break;                                                        \
    }
    gload(0);
    lstore(0);
    __syncthreads();
#pragma unroll 1
    for (int sg = 0; sg < 64 / QM_CLS; sg++) {
        if (sg + 1 < 64 / QM_CLS) gload(sg + 1);  // in flight under this stage
        const int buf = sg & 1;
        // a class's operands (all NMAX slots; slots past its block count hold stale values, never
        // used) are read before the previous class's arithmetic (NMAX <= 2: double-buffered registers)
        struct Ops {
            float4 w[NMAX], x[NMAX];
        };
        auto rd = [&](Ops & o, int lc) {
#pragma unroll
            for (int u = 0; u < NMAX; u++) {
                o.w[u] = *(const float4 *)&qw[buf][u * 8 + lc][4 * rq];
                o.x[u] = *(const float4 *)&qx[buf][u * 8 + lc][16 * wave + 4 * tq];
            }
        };
        auto mac = [&](const Ops & o, int n) {
#pragma unroll
            for (int u = 0; u < NMAX; u++) {
                if (u >= n) break;  // uniform
                const float wv[4] = {o.w[u].x, o.w[u].y, o.w[u].z, o.w[u].w};
                const float xv[4] = {o.x[u].x, o.x[u].y, o.x[u].z, o.x[u].w};
#pragma unroll
                for (int r = 0; r < 4; r++) qm_mac_row<4>(acc + 4 * r, wv[r], xv);
            }
        };
        auto fold = [&](int l) {
            if ((l & 1) == 0) {
#pragma unroll
                for (int k = 0; k < 16; k++) st[0][k] = acc[k];
            } else {
                switch (__builtin_ctz(~l)) { QM_CLOSE(1) QM_CLOSE(2) QM_CLOSE(3) QM_CLOSE(4) QM_CLOSE(5) default: QM_CLOSE(6) }
            }
#pragma unroll
            for (int k = 0; k < 16; k++) acc[k] = 0.0f;
        };
        if constexpr (NMAX <= 2) {
            // the stage's 8 classes as a static 3-level subtree (class pairs in two accumulator
            // sets, the binary counter's levels 1 and 2 in named registers), then levels 3.. by the
            // stage's own counter: the same additions as fold(), without its copies and branches
            Ops o0, o1;
            float aA[16], aB[16], p1[16], p2[16];
            auto macf = [&](float (&a)[16], const Ops & o, int n) {
#pragma unroll
                for (int k = 0; k < 16; k++) a[k] = 0.0f;
#pragma unroll
                for (int u = 0; u < NMAX; u++) {
                    if (!(FULL && u == 0) && u >= n) break;  // uniform
                    const float wv[4] = {o.w[u].x, o.w[u].y, o.w[u].z, o.w[u].w};
                    const float xv[4] = {o.x[u].x, o.x[u].y, o.x[u].z, o.x[u].w};
#pragma unroll
                    for (int r = 0; r < 4; r++) qm_mac_row<4>(a + 4 * r, wv[r], xv);
                }
            };
            auto addl = [](float (&v)[16], const float (&t)[16]) {  // v = t + v
#pragma unroll
                for (int k = 0; k < 16; k += 2) {
                    const qf2_t r = qf2_t{t[k], t[k + 1]} + qf2_t{v[k], v[k + 1]};
                    v[k] = r.x;
                    v[k + 1] = r.y;
                }
            };
            auto put = [](float (&d)[16], const float (&v)[16]) {
#pragma unroll
                for (int k = 0; k < 16; k++) d[k] = v[k];
            };
            rd(o0, 0);
#pragma unroll
            for (int lc = 0; lc < QM_CLS; lc += 2) {
                const int l = sg * QM_CLS + lc;
                rd(o1, lc + 1);
                macf(aA, o0, cq + (l < crem ? 1 : 0));
                if (lc + 2 < QM_CLS) rd(o0, lc + 2);
                macf(aB, o1, cq + (l + 1 < crem ? 1 : 0));
                addl(aB, aA);  // class l + 1 (odd): st[0] + acc
                if (lc == 0 || lc == 4) {
                    put(p1, aB);  // level 1
                } else if (lc == 2) {
                    addl(aB, p1);
                    put(p2, aB);  // level 2
                } else {
                    addl(aB, p1);
                    addl(aB, p2);
                    switch (__builtin_ctz(~sg)) {  // levels 3.. : class 8 sg + 7's counter
                        case 0: put(st[3], aB); break;
                        case 1: addl(aB, st[3]); put(st[4], aB); break;
                        case 2: addl(aB, st[3]); addl(aB, st[4]); put(st[5], aB); break;
                        default: addl(aB, st[3]); addl(aB, st[4]); addl(aB, st[5]); put(st[0], aB); break;
                    }
                }
            }
        } else {
            // 4 blocks of a class at a time (their reads issued together)
#pragma unroll 1
            for (int lc = 0; lc < QM_CLS; lc++) {
                const int l = sg * QM_CLS + lc, n = cq + (l < crem ? 1 : 0);
                float4 w4[1][4], x4[1][4];
                auto rd4 = [&](int h, int u0) {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int u = min(u0 + q, NMAX - 1);
                        w4[h][q] = *(const float4 *)&qw[buf][u * 8 + lc][4 * rq];
                        x4[h][q] = *(const float4 *)&qx[buf][u * 8 + lc][16 * wave + 4 * tq];
                    }
                };
                auto mac4 = [&](int h, int u0) {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if (u0 + q >= n) break;  // uniform
                        const float wv[4] = {w4[h][q].x, w4[h][q].y, w4[h][q].z, w4[h][q].w};
                        const float xv[4] = {x4[h][q].x, x4[h][q].y, x4[h][q].z, x4[h][q].w};
#pragma unroll
                        for (int r = 0; r < 4; r++) qm_mac_row<4>(acc + 4 * r, wv[r], xv);
                    }
                };
                rd4(0, 0);
                mac4(0, 0);
                if (NMAX > 4 && n > 4) {
                    rd4(0, 4);
                    mac4(0, 4);
                }
                fold(l);
            }
        }
        if (sg + 1 < 64 / QM_CLS) lstore((sg + 1) & 1);
        __syncthreads();
    }
#undef QM_CLOSE
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int row = r0 + 4 * rq + r;
        if (row >= M) continue;
        float * out = g.m2 + E.moff + (size_t)row * T;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const int t = tok0 + 16 * wave + 4 * tq + c;
            if (t < T) out[t] = st[0][4 * r + c];
        }
    }
}

// The long-class form (5-8 blocks per class: K > 8192): lane = row, wave = 8 tokens, workgroup = 64
// rows x 32 tokens; a lane's m_w is one b32 read and the wave's 8 s_x two broadcast b128 reads per
// block (the 4 x 4 register tiles of k_qg_msum need 260 VGPRs at this depth: one wave per SIMD).
template <int NMAX, bool FULL>
__global__ __launch_bounds__(256) void k_qg_msum_rows(MMGroup g) {
    constexpr int NSLOT = QM_CLS * NMAX;
    __shared__ __attribute__((aligned(16))) float qw[2][NSLOT][64];
    __shared__ __attribute__((aligned(16))) float qx[2][NSLOT][32];
    const int T = g.T, tgs = (T + 31) / 32;
    int e = 0, base = 0;
#pragma unroll 1
    for (; e + 1 < g.n; e++) {
        const int n_e = (g.e[e].W.M + 63) / 64 * tgs;
        if ((int)blockIdx.x < base + n_e) break;
        base += n_e;
    }
    const MMEntry & E = g.e[e];
    const int M = E.W.M, nb = E.W.K >> 5, MS = qm_stride(M);
    const int local = (int)blockIdx.x - base;
    const int rt = local / tgs, tg = local % tgs;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r0 = rt * 64, tok0 = tg * 32;
    const int cq = nb >> 6, crem = nb & 63;
    const size_t AB = qg_a_bytes(true);
    // loaders: m_w row lane of slots wave + 4 k; s_x token tid & 31 of slots (tid >> 5) + 8 k.  A block
    // past its class's count is clamped (loaded, never read).
    const float * wrow = E.W.mt + min(r0 + lane, MS - 1);
    const int tx = min(tok0 + (tid & 31), T - 1);
    const float * xrow = (const float *)(E.in.tq + (size_t)(tx / QG_TOK) * nb * AB + QG_A_S) + tx % QG_TOK;
    constexpr int LW = NSLOT / 4, LX = NSLOT / 8;
    float lw[LW], lx[LX];
    auto blk = [&](int sg, int sl) {
        const int lc = sl & 7, u = sl >> 3, l = sg * QM_CLS + lc;
        return u < cq + (l < crem ? 1 : 0) ? l + 64 * u : l;  // (l < nb whenever the class has a block)
    };
    auto gload = [&](int sg) {
#pragma unroll
        for (int k = 0; k < LW; k++) lw[k] = wrow[(size_t)min(blk(sg, wave + 4 * k), nb - 1) * MS];
#pragma unroll
        for (int k = 0; k < LX; k++) lx[k] = xrow[(size_t)min(blk(sg, (tid >> 5) + 8 * k), nb - 1) * (AB / 4)];
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int k = 0; k < LW; k++) qw[buf][wave + 4 * k][lane] = lw[k];
#pragma unroll
        for (int k = 0; k < LX; k++) qx[buf][(tid >> 5) + 8 * k][tid & 31] = lx[k];
    };
    float st[6][8], acc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = 0.0f;
#define QM_CLOSE(N)                                                   \
    case N: {                                                         \
        qm_close<N, 8>(st, acc);  /* N = 6: the total, into st[0] */  \
        break;                                                        \
    }
    gload(0);
    lstore(0);
    __syncthreads();
#pragma unroll 1
    for (int sg = 0; sg < 64 / QM_CLS; sg++) {
        if (sg + 1 < 64 / QM_CLS) gload(sg + 1);  // in flight under this stage
        const int buf = sg & 1;
        // a class's operands (all NMAX slots; slots past its block count hold stale values, never
        // used) are read before the previous class's arithmetic (NMAX <= 2: double-buffered registers)
        struct Ops {
            float w[NMAX];
            float4 s0[NMAX], s1[NMAX];
        };
        auto rd = [&](Ops & o, int lc) {
#pragma unroll
            for (int u = 0; u < NMAX; u++) {
                o.w[u] = qw[buf][u * 8 + lc][lane];
                o.s0[u] = *(const float4 *)&qx[buf][u * 8 + lc][8 * wave];
                o.s1[u] = *(const float4 *)&qx[buf][u * 8 + lc][8 * wave + 4];
            }
        };
        auto mac = [&](const Ops & o, int n) {
#pragma unroll
            for (int u = 0; u < NMAX; u++) {
                if (u >= n) break;  // uniform
                const float sx[8] = {o.s0[u].x, o.s0[u].y, o.s0[u].z, o.s0[u].w, o.s1[u].x, o.s1[u].y, o.s1[u].z, o.s1[u].w};
                qm_mac_row<8>(acc, o.w[u], sx);
            }
        };
        auto fold = [&](int l) {
            if ((l & 1) == 0) {
#pragma unroll
                for (int k = 0; k < 8; k++) st[0][k] = acc[k];
            } else {
                switch (__builtin_ctz(~l)) { QM_CLOSE(1) QM_CLOSE(2) QM_CLOSE(3) QM_CLOSE(4) QM_CLOSE(5) default: QM_CLOSE(6) }
            }
#pragma unroll
            for (int k = 0; k < 8; k++) acc[k] = 0.0f;
        };
        if constexpr (NMAX <= 2) {
            Ops o0, o1;
            rd(o0, 0);
#pragma unroll
            for (int lc = 0; lc < QM_CLS; lc += 2) {
                const int l = sg * QM_CLS + lc;
                rd(o1, lc + 1);
                mac(o0, cq + (l < crem ? 1 : 0));
                fold(l);
                if (lc + 2 < QM_CLS) rd(o0, lc + 2);
                mac(o1, cq + (l + 1 < crem ? 1 : 0));
                fold(l + 1);
            }
        } else if constexpr (FULL) {
            // FULL (every class >= 1 block): the stage's 8 classes as a static subtree, as in
            // k_qg_msum; each class's first 4 blocks peeled so its chain starts on a literal 0
            float aA[8], aB[8], p1[8], p2[8];
            auto macr = [&](float (&a)[8], int lc, int n) {
#pragma unroll
                for (int k = 0; k < 8; k++) a[k] = 0.0f;
                auto step4 = [&](int u0, bool first) {
                    float w4[4];
                    float4 a4[4], b4[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int u = min(u0 + q, NMAX - 1);
                        w4[q] = qw[buf][u * 8 + lc][lane];
                        a4[q] = *(const float4 *)&qx[buf][u * 8 + lc][8 * wave];
                        b4[q] = *(const float4 *)&qx[buf][u * 8 + lc][8 * wave + 4];
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if (!(first && q == 0) && u0 + q >= n) break;  // uniform
                        const float sx[8] = {a4[q].x, a4[q].y, a4[q].z, a4[q].w, b4[q].x, b4[q].y, b4[q].z, b4[q].w};
                        qm_mac_row<8>(a, w4[q], sx);
                    }
                };
                step4(0, true);
#pragma unroll 1
                for (int u0 = 4; u0 < n; u0 += 4) step4(u0, false);
            };
            auto addl = [](float (&v)[8], const float (&t)[8]) {  // v = t + v
#pragma unroll
                for (int k = 0; k < 8; k += 2) {
                    const qf2_t r = qf2_t{t[k], t[k + 1]} + qf2_t{v[k], v[k + 1]};
                    v[k] = r.x;
                    v[k + 1] = r.y;
                }
            };
            auto put = [](float (&d)[8], const float (&v)[8]) {
#pragma unroll
                for (int k = 0; k < 8; k++) d[k] = v[k];
            };
#pragma unroll
            for (int lc = 0; lc < QM_CLS; lc += 2) {
                const int l = sg * QM_CLS + lc;
                macr(aA, lc, cq + (l < crem ? 1 : 0));
                macr(aB, lc + 1, cq + (l + 1 < crem ? 1 : 0));
                addl(aB, aA);
                if (lc == 0 || lc == 4) {
                    put(p1, aB);
                } else if (lc == 2) {
                    addl(aB, p1);
                    put(p2, aB);
                } else {
                    addl(aB, p1);
                    addl(aB, p2);
                    switch (__builtin_ctz(~sg)) {
                        case 0: put(st[3], aB); break;
                        case 1: addl(aB, st[3]); put(st[4], aB); break;
                        case 2: addl(aB, st[3]); addl(aB, st[4]); put(st[5], aB); break;
                        default: addl(aB, st[3]); addl(aB, st[4]); addl(aB, st[5]); put(st[0], aB); break;
                    }
                }
            }
        } else {
            // 4 blocks of a class at a time (their reads issued together), in ascending order: the
            // registers stay bounded for any NMAX (16: K <= 32768, e.g. a 20480-wide FFN value)
#pragma unroll 1
            for (int lc = 0; lc < QM_CLS; lc++) {
                const int l = sg * QM_CLS + lc, n = cq + (l < crem ? 1 : 0);
#pragma unroll 1
                for (int u0 = 0; u0 < n; u0 += 4) {
                    float w4[4];
                    float4 a4[4], b4[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int u = min(u0 + q, NMAX - 1);
                        w4[q] = qw[buf][u * 8 + lc][lane];
                        a4[q] = *(const float4 *)&qx[buf][u * 8 + lc][8 * wave];
                        b4[q] = *(const float4 *)&qx[buf][u * 8 + lc][8 * wave + 4];
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if (u0 + q >= n) break;  // uniform
                        const float sx[8] = {a4[q].x, a4[q].y, a4[q].z, a4[q].w, b4[q].x, b4[q].y, b4[q].z, b4[q].w};
                        qm_mac_row<8>(acc, w4[q], sx);
                    }
                }
                fold(l);
            }
        }
        if (sg + 1 < 64 / QM_CLS) lstore((sg + 1) & 1);
        __syncthreads();
    }
#undef QM_CLOSE
    const int r = r0 + lane;
    if (r >= M) return;
    float * out = g.m2 + E.moff + (size_t)r * T + tok0 + 8 * wave;
#pragma unroll
    for (int k = 0; k < 8; k++)
        if (tok0 + 8 * wave + k < T) out[k] = st[0][k];
}

// The combine of a split group whose entries' partials sit at g.part + poff (k_fmm's split form)
bool launch_qg_combine(hipStream_t st, MMGroup & g, int split) {
    int cblocks = 0;
    for (int i = 0; i < g.n; i++) {
        g.e[i].cblock0 = cblocks;
        cblocks += (int)(((size_t)g.T * g.e[i].W.M + 255) / 256);
    }
    if (split == 4) RK_LAUNCH((k_qg_combine<4, false>), dim3(cblocks), dim3(256), 0, st, g);
    else if (split == 8) RK_LAUNCH((k_qg_combine<8, false>), dim3(cblocks), dim3(256), 0, st, g);
    else return false;
    HIP_OK(hipGetLastError());
    return true;
}

// Every entry must have y (the engine gives emitting entries a scratch y); emission into the
// next matmul's activation format is a separate launch_act_from_f32 pass by the caller.  The
// weights need their tile records (upload_mat) and the activations must be token tiles.
int g_qgemm_generic = 0;  // 1: K = 2048 through the generic kernel too (tools, comparison)
int kQgCUs = 256;          // compute units of the device (set_mv_device_cus): the split-K threshold

bool launch_qgemm(hipStream_t st, MMGroup & g, int wtype) {
    const int rows = qg_rows(wtype);
    const int tilesT = (g.T + QG_TOK - 1) / QG_TOK;
    int blocks = 0;
    for (int i = 0; i < g.n; i++) {
        MMEntry & e = g.e[i];
        if (e.W.type != wtype || !e.W.gt || e.W.K % 32 || !e.y || e.in.fmt != act_fmt_for(wtype) || !e.in.tiled ||
            !e.in.tq) {
            fprintf(stderr, "rwkv: qgemm entry %d not supported (type %d)\n", i, e.W.type);
            return false;
        }
        e.block0 = blocks;
        blocks += (e.W.M + rows - 1) / rows * tilesT;
    }
    if (!blocks) return true;
    if (qg_one(wtype)) {
        // the m*s chain totals first (k_qg_msum), read by the GEMM epilogue / the combine
        size_t mfl = 0;
        int mblocks = 0, mblocks8 = 0, nmax = 0;
        bool full = true;  // every entry's classes hold >= 1 block
        const int tgs = (g.T + 63) / 64;
        for (int i = 0; i < g.n; i++) {
            if (!g.e[i].W.mt) {
                fprintf(stderr, "rwkv: qgemm _1 entry %d without mins\n", i);
                return false;
            }
            g.e[i].moff = mfl;
            mfl += (size_t)g.T * g.e[i].W.M;
            mblocks += (g.e[i].W.M + 63) / 64 * tgs;
            mblocks8 += (g.e[i].W.M + 63) / 64 * ((g.T + 31) / 32);
            const int nbi = g.e[i].W.K / 32, nmi = nbi / 64 + (nbi % 64 ? 1 : 0);
            nmax = std::max(nmax, nmi);
            full = full && nbi >= 64;
        }
        if (!g.m2 || g.m2_floats < mfl) {
            fprintf(stderr, "rwkv: qgemm _1 group needs %zu m*s floats, has %zu\n", mfl, g.m2 ? g.m2_floats : (size_t)0);
            return false;
        }
        // the 4 x 4 register-tile form over 64-token tiles; the row form (32-token tiles) for 32 or
        // fewer tokens (contexts) and for classes of 5-8 blocks
        const bool rows = g.T <= 32 || nmax > 4;
        if (rows && nmax <= 1) RK_LAUNCH((k_qg_msum_rows<1, false>), dim3(mblocks8), dim3(256), 0, st, g);
        else if (rows && nmax <= 2) RK_LAUNCH((k_qg_msum_rows<2, false>), dim3(mblocks8), dim3(256), 0, st, g);
        else if (rows && nmax <= 4) RK_LAUNCH((k_qg_msum_rows<4, false>), dim3(mblocks8), dim3(256), 0, st, g);
        else if (rows && nmax <= 8 && full) RK_LAUNCH((k_qg_msum_rows<8, true>), dim3(mblocks8), dim3(256), 0, st, g);
        else if (rows && nmax <= 8) RK_LAUNCH((k_qg_msum_rows<8, false>), dim3(mblocks8), dim3(256), 0, st, g);
        else if (rows && nmax <= 16) RK_LAUNCH((k_qg_msum_rows<16, false>), dim3(mblocks8), dim3(256), 0, st, g);
        else if (nmax <= 1 && full) RK_LAUNCH((k_qg_msum<1, true>), dim3(mblocks), dim3(256), 0, st, g);
        else if (nmax <= 1) RK_LAUNCH((k_qg_msum<1, false>), dim3(mblocks), dim3(256), 0, st, g);
        else if (nmax <= 2 && full) RK_LAUNCH((k_qg_msum<2, true>), dim3(mblocks), dim3(256), 0, st, g);
        else if (nmax <= 2) RK_LAUNCH((k_qg_msum<2, false>), dim3(mblocks), dim3(256), 0, st, g);
        else if (nmax <= 4) RK_LAUNCH((k_qg_msum<4, false>), dim3(mblocks), dim3(256), 0, st, g);
        else {
            fprintf(stderr, "rwkv: qgemm _1 group: K above the m*s pass's 32768\n");
            return false;
        }
        HIP_OK(hipGetLastError());
    }
    // Q8_0 emission fused into the epilogue (the Q4_0 / Q5_0 / Q8_0 GEMMs: a wave holds 32 rows)
    for (int i = 0; i < g.n; i++) {
        MMEntry & e = g.e[i];
        e.fuse_emit = e.emit && e.out.tiled && e.out.fmt == A_Q8_0 && e.out.tq && e.out.K == e.W.M &&
                      e.W.M % 64 == 0 && e.ldy == e.W.M && e.epi != EPI_ADD && e.epi != EPI_SIGMUL_ADD &&
                      e.epi != EPI_VMIX7 && e.epi != EPI_DECAY6 && e.epi != EPI_DECAY7 && e.epi != EPI_SIGMOID_BIAS;
    }
    const dim3 grid(blocks), block(256);
    bool k64 = true;
    for (int i = 0; i < g.n; i++) k64 = k64 && g.e[i].W.K == 2048;
    // split-K when the group has few tiles (batched decode's 64-context tiles, small-M entries such
    // as the v6 maa LoRA W1): every tile's class tree in 4 or 8 subtrees on as many workgroups,
    // combined (epilogue, emission) by k_qg_combine -- the same bits as the unsplit kernel
    int split = g.split;
    if (split == 0) split = blocks >= 2 * kQgCUs ? 1 : blocks * 4 >= 2 * kQgCUs ? 4 : 8;
    if (split != 1 && split != 2 && split != 4 && split != 8) split = 1;
    size_t pfl = 0;
    if (split > 1) {
        for (int i = 0; i < g.n; i++) {
            g.e[i].poff = pfl;
            pfl += (size_t)split * g.T * g.e[i].W.M;
        }
        if (!g.part || g.part_floats < pfl || g_qgemm_generic) split = 1;
        for (int i = 0; i < g.n; i++)
            if (g.e[i].W.M % 32) split = 1;  // combine: one emission block per half-wave
    }
    if (split > 1) {
        // workgroup ranges of the entries in the split grid (SPLIT workgroups per tile)
        for (int i = 0; i < g.n; i++) g.e[i].block0 *= split;
        const dim3 sgrid(blocks * split);
#define QG_SPLIT_L(WFv, SP)                                                                    \
    do {                                                                                       \
        if (k64) RK_LAUNCH((k_qgemm_k64<WFv, SP>), sgrid, block, 0, st, g);      \
        else RK_LAUNCH((k_qgemm<WFv, SP>), sgrid, block, 0, st, g);                   \
    } while (0)
#define QG_SPLIT_T(SP)                                                                         \
    do {                                                                                       \
        switch (wtype) {                                                                       \
            case W_Q4_0: QG_SPLIT_L(W_Q4_0, SP); break;                                        \
            case W_Q4_1: QG_SPLIT_L(W_Q4_1, SP); break;                                        \
            case W_Q5_0: QG_SPLIT_L(W_Q5_0, SP); break;                                        \
            case W_Q5_1: QG_SPLIT_L(W_Q5_1, SP); break;                                        \
            case W_Q8_0: QG_SPLIT_L(W_Q8_0, SP); break;                                        \
            default: fprintf(stderr, "rwkv: qgemm type %d unsupported\n", wtype); return false; \
        }                                                                                      \
    } while (0)
        if (split == 2) QG_SPLIT_T(2);
        else if (split == 4) QG_SPLIT_T(4);
        else QG_SPLIT_T(8);
#undef QG_SPLIT_T
#undef QG_SPLIT_L
        HIP_OK(hipGetLastError());
        int cblocks = 0;
        for (int i = 0; i < g.n; i++) {
            g.e[i].cblock0 = cblocks;
            g.e[i].fuse_emit = g.e[i].emit;  // the combine emits
            cblocks += (int)(((size_t)g.T * g.e[i].W.M + 255) / 256);
        }
        const bool one = qg_one(wtype);
        if (split == 2) {
            if (one) RK_LAUNCH((k_qg_combine<2, true>), dim3(cblocks), block, 0, st, g);
            else RK_LAUNCH((k_qg_combine<2, false>), dim3(cblocks), block, 0, st, g);
        } else if (split == 4) {
            if (one) RK_LAUNCH((k_qg_combine<4, true>), dim3(cblocks), block, 0, st, g);
            else RK_LAUNCH((k_qg_combine<4, false>), dim3(cblocks), block, 0, st, g);
        } else {
            if (one) RK_LAUNCH((k_qg_combine<8, true>), dim3(cblocks), block, 0, st, g);
            else RK_LAUNCH((k_qg_combine<8, false>), dim3(cblocks), block, 0, st, g);
        }
        HIP_OK(hipGetLastError());
        return true;
    }
    if (k64 && !g_qgemm_generic) {
        switch (wtype) {
            case W_Q4_0: RK_LAUNCH(k_qgemm_k64<W_Q4_0>, grid, block, 0, st, g); break;
            case W_Q4_1: RK_LAUNCH(k_qgemm_k64<W_Q4_1>, grid, block, 0, st, g); break;
            case W_Q5_0: RK_LAUNCH(k_qgemm_k64<W_Q5_0>, grid, block, 0, st, g); break;
            case W_Q5_1: RK_LAUNCH(k_qgemm_k64<W_Q5_1>, grid, block, 0, st, g); break;
            case W_Q8_0: RK_LAUNCH(k_qgemm_k64<W_Q8_0>, grid, block, 0, st, g); break;
            default: fprintf(stderr, "rwkv: qgemm type %d unsupported\n", wtype); return false;
        }
        HIP_OK(hipGetLastError());
        return true;
    }
    switch (wtype) {
        case W_Q4_0: RK_LAUNCH(k_qgemm<W_Q4_0>, grid, block, 0, st, g); break;
        case W_Q4_1: RK_LAUNCH(k_qgemm<W_Q4_1>, grid, block, 0, st, g); break;
        case W_Q5_0: RK_LAUNCH(k_qgemm<W_Q5_0>, grid, block, 0, st, g); break;
        case W_Q5_1: RK_LAUNCH(k_qgemm<W_Q5_1>, grid, block, 0, st, g); break;
        case W_Q8_0: RK_LAUNCH(k_qgemm<W_Q8_0>, grid, block, 0, st, g); break;
        default: fprintf(stderr, "rwkv: qgemm type %d unsupported\n", wtype); return false;
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
