// selftest.hip -- kernel self-test entry points (include/rwkv_mi355x.h): run one kernel on
// host-provided operands so tests can check it against the oracle's primitive of the same
// name (oracle_quantize_act, oracle_matmul) without whole-model noise.
#include <string.h>

#include <vector>

#include "../../include/rwkv_mi355x.h"
#include "engine.hpp"
#include "kernels.hpp"

using namespace rwkvmi;

namespace {

struct DevBufs {
    std::vector<void *> p;
    void * alloc(size_t n) {
        void * q = nullptr;
        if (hipMalloc(&q, n + 64) != hipSuccess) return nullptr;
        (void)hipMemset(q, 0, n + 64);
        p.push_back(q);
        return q;
    }
    ~DevBufs() {
        for (void * q : p) (void)hipFree(q);
    }
};

bool make_act(DevBufs & b, int fmt, int T, int K, ActBuf & a) {
    memset(&a, 0, sizeof(a));
    a.fmt = fmt;
    a.K = K;
    const size_t n = (size_t)T * K, nb = n / 32 + 1;
    a.f = (float *)b.alloc(n * 4);
    a.h = (__half *)b.alloc(n * 2);
    a.q = (int8_t *)b.alloc(n);
    a.d = (float *)b.alloc(nb * 4);
    a.s = (float *)b.alloc(nb * 4);
    a.qsum = (int *)b.alloc(nb * 4);
    a.tq = (uint8_t *)b.alloc(((size_t)T + QG_TOK - 1) / QG_TOK * (K / 32) * qg_a_bytes(true));
    return a.f && a.h && a.q && a.d && a.s && a.qsum && a.tq;
}

}  // namespace

extern "C" RWKV_API bool rwkv_mi355x_selftest_quantize_act(int wtype, const float * x, int T, int K, int8_t * q,
                                                           float * d, float * s) {
    if (K % 32 || T <= 0) return false;
    DevBufs b;
    ActBuf a;
    const int fmt = act_fmt_for(wtype);
    float * dx = (float *)b.alloc((size_t)T * K * 4);
    if (!dx || !make_act(b, fmt, T, K, a)) return false;
    if (hipMemcpy(dx, x, (size_t)T * K * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
    if (!launch_act_from_f32(nullptr, dx, T, K, a)) return false;
    if (hipDeviceSynchronize() != hipSuccess) return false;
    const size_t nb = (size_t)T * K / 32;
    if (q && hipMemcpy(q, a.q, (size_t)T * K, hipMemcpyDeviceToHost) != hipSuccess) return false;
    if (d && hipMemcpy(d, a.d, nb * 4, hipMemcpyDeviceToHost) != hipSuccess) return false;
    if (s && hipMemcpy(s, a.s, nb * 4, hipMemcpyDeviceToHost) != hipSuccess) return false;
    return true;
}

static bool selftest_mm(int wtype, const void * W, int K, int M, const float * x, int T, float * y, bool mfma,
                        int split = 0) {
    if (K % 32 || T <= 0 || M <= 0) return false;
    HostTensor ht;
    ht.name = "selftest";
    ht.type = (uint32_t)wtype;
    ht.ndim = 2;
    ht.ne[0] = (uint32_t)K;
    ht.ne[1] = (uint32_t)M;
    const size_t nbytes = type_nbytes(ht.type, ht.nel());
    if (!nbytes) return false;
    ht.data.assign((const uint8_t *)W, (const uint8_t *)W + nbytes);
    DeviceModel dm;
    DMat dmat{};
    bool ok = upload_mat(dm, &ht, dmat, false, false);
    DevBufs b;
    ActBuf a;
    float * dx = (float *)b.alloc((size_t)T * K * 4);
    float * dy = (float *)b.alloc((size_t)T * M * 4);
    ok = ok && dx && dy && make_act(b, act_fmt_for(wtype), T, K, a);
    a.tiled = mfma ? 1 : 0;  // the GEMM reads token tiles, k_mm row-major blocks
    ok = ok && hipMemcpy(dx, x, (size_t)T * K * 4, hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && launch_act_from_f32(nullptr, dx, T, K, a);
    if (ok) {
        MMGroup g;
        memset(&g, 0, sizeof(g));
        g.n = 1;
        g.T = T;
        g.e[0].W = dmat;
        g.e[0].in = a;
        g.e[0].y = dy;
        g.e[0].ldy = M;
        g.e[0].epi = EPI_STORE;
        g.split = split;
        g.fmm = 1;  // the f32-MFMA form for float weights whenever it applies (T >= 16)
        g.part_floats = (size_t)8 * T * M;
        g.part = (float *)b.alloc(g.part_floats * 4);
        ok = g.part != nullptr;
        if (mfma) {
            g.m2_floats = (size_t)T * M;
            g.m2 = (float *)b.alloc(g.m2_floats * 4);
            ok = ok && g.m2 != nullptr;
        }
        ok = ok && (mfma ? launch_qgemm(nullptr, g, wtype) : launch_mm_group(nullptr, g, wtype));
    }
    ok = ok && hipDeviceSynchronize() == hipSuccess;
    ok = ok && hipMemcpy(y, dy, (size_t)T * M * 4, hipMemcpyDeviceToHost) == hipSuccess;
    free_model(dm);
    return ok;
}

extern "C" RWKV_API bool rwkv_mi355x_selftest_matmul(int wtype, const void * W, int K, int M, const float * x, int T,
                                                     float * y) {
    return selftest_mm(wtype, W, K, M, x, T, y, false, 1);  // unsplit (the float matmuls' reference form)
}

extern "C" RWKV_API bool rwkv_mi355x_selftest_gemm(int wtype, const void * W, int K, int M, const float * x, int T,
                                                   float * y) {
    if (!wtype_quantized(wtype) || T < 2) return false;
    return selftest_mm(wtype, W, K, M, x, T, y, true);
}

// The same with the split-K form chosen: 1 = unsplit, 4 / 8 = that many class subtrees + combine
// (quantized: the int8-MFMA GEMM; F16 / F32 over 16+ tokens, K >= 512: k_fmm).
extern "C" RWKV_API bool rwkv_mi355x_selftest_gemm_split(int wtype, const void * W, int K, int M, const float * x,
                                                         int T, float * y, int split) {
    if (split != 1 && split != 2 && split != 4 && split != 8) return false;
    if (wtype_quantized(wtype)) return T >= 2 && selftest_mm(wtype, W, K, M, x, T, y, true, split);
    return (wtype == W_F16 || wtype == W_F32) && T >= 16 && K >= 512 && selftest_mm(wtype, W, K, M, x, T, y, false, split);
}

// WKV-6 (v5 / v6) over T tokens of one context: chunked = 0 the serial k_wkv6_s64 (decode's
// association), 1 the chunk-parallel form (wkv_chunk.hip).  k, v, r, w: [T][H*64] (w: [H*64] when
// w_per_token = 0); u: [H*64]; state_in / state_out: [H][64][64]; y: [T][H*64]; all host.
extern "C" RWKV_API bool rwkv_mi355x_selftest_wkv6(int T, int H, int chunked, int w_per_token, const float * k,
                                                  const float * v, const float * r, const float * u, const float * w,
                                                  const float * state_in, float * state_out, float * y) {
    if (T < 1 || H < 1 || !k || !v || !r || !u || !w || !state_in || !state_out || !y) return false;
    if (chunked && !wkv6_chunked_supported(T, 64, 0)) return false;
    const size_t C = (size_t)H * 64, TC = (size_t)T * C, SN = C * 64, WN = w_per_token ? TC : C;
    DevBufs b;
    float *dk = (float *)b.alloc(TC * 4), *dv = (float *)b.alloc(TC * 4), *dr = (float *)b.alloc(TC * 4),
          *du = (float *)b.alloc(C * 4), *dw = (float *)b.alloc(WN * 4), *dsi = (float *)b.alloc(SN * 4),
          *dso = (float *)b.alloc(SN * 4), *dy = (float *)b.alloc(TC * 4), *ra = (float *)b.alloc(TC * 4),
          *kb = (float *)b.alloc(TC * 4), *sc = (float *)b.alloc(wkv6_chunked_scratch_floats(T, H) * 4);
    if (!dk || !dv || !dr || !du || !dw || !dsi || !dso || !dy || !ra || !kb || !sc) return false;
    const std::pair<float *, const float *> up[] = {{dk, k}, {dv, v}, {dr, r}, {dy, y}};
    for (const auto & p : up)
        if (hipMemcpy(p.first, p.second, TC * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
    if (hipMemcpy(du, u, C * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dw, w, WN * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dsi, state_in, SN * 4, hipMemcpyHostToDevice) != hipSuccess)
        return false;
    const bool ok = chunked ? launch_wkv6_chunked(nullptr, T, H, dk, dv, dr, du, dw, w_per_token, dsi, dso, dy, ra, kb, sc)
                            : launch_wkv6(nullptr, T, H, 64, dk, dv, dr, du, dw, w_per_token, dsi, dso, dy, 0);
    if (!ok || hipDeviceSynchronize() != hipSuccess) return false;
    return hipMemcpy(y, dy, TC * 4, hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(state_out, dso, SN * 4, hipMemcpyDeviceToHost) == hipSuccess;
}

// WKV-7 over T tokens of one context: chunked = 0 the serial k_wkv7_s64 (decode's association), 1 the
// chunk-parallel form (wkv7_chunk.hip).  r, w, k, v, a, b: [T][H*64]; state_in / state_out:
// [H][64 value rows][64 key columns]; y: [T][H*64]; all host.
extern "C" RWKV_API bool rwkv_mi355x_selftest_wkv7(int T, int H, int chunked, const float * r, const float * w,
                                                  const float * k, const float * v, const float * a, const float * b,
                                                  const float * state_in, float * state_out, float * y) {
    if (T < 1 || H < 1 || !r || !w || !k || !v || !a || !b || !state_in || !state_out || !y) return false;
    if (chunked && !wkv7_chunked_supported(T, 64, 0)) return false;
    const size_t C = (size_t)H * 64, TC = (size_t)T * C, SN = C * 64;
    DevBufs bf;
    float *dr = (float *)bf.alloc(TC * 4), *dw = (float *)bf.alloc(TC * 4), *dk = (float *)bf.alloc(TC * 4),
          *dv = (float *)bf.alloc(TC * 4), *da = (float *)bf.alloc(TC * 4), *db = (float *)bf.alloc(TC * 4),
          *dsi = (float *)bf.alloc(SN * 4), *dso = (float *)bf.alloc(SN * 4), *dy = (float *)bf.alloc(TC * 4),
          *sc = chunked ? (float *)bf.alloc(wkv7_chunked_scratch_floats(T, H) * 4) : nullptr;
    if (!dr || !dw || !dk || !dv || !da || !db || !dsi || !dso || !dy || (chunked && !sc)) return false;
    const std::pair<float *, const float *> up[] = {{dr, r}, {dw, w}, {dk, k}, {dv, v}, {da, a}, {db, b}, {dy, y}};
    for (const auto & p : up)
        if (hipMemcpy(p.first, p.second, TC * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
    if (hipMemcpy(dsi, state_in, SN * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
    const bool ok = chunked ? launch_wkv7_chunked(nullptr, T, H, dr, dw, dk, dv, da, db, dsi, dso, dy, sc)
                            : launch_wkv7(nullptr, T, H, 64, dr, dw, dk, dv, da, db, dsi, dso, dy, 0);
    if (!ok || hipDeviceSynchronize() != hipSuccess) return false;
    return hipMemcpy(y, dy, TC * 4, hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(state_out, dso, SN * 4, hipMemcpyDeviceToHost) == hipSuccess;
}
