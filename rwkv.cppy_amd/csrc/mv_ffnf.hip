// mv_ffnf.hip -- launcher of the one-launch decode channel mix (mv_ffnf.hpp).
#include "mv_ffnf.hpp"

#include <string.h>

namespace rwkvmi {

extern template bool launch_ffn_fused_t<W_Q4_0>(hipStream_t, const FfnFused &, int, bool, int, int, dim3, int);
extern template bool launch_ffn_fused_t<W_Q4_1>(hipStream_t, const FfnFused &, int, bool, int, int, dim3, int);
extern template bool launch_ffn_fused_t<W_Q5_0>(hipStream_t, const FfnFused &, int, bool, int, int, dim3, int);
extern template bool launch_ffn_fused_t<W_Q5_1>(hipStream_t, const FfnFused &, int, bool, int, int, dim3, int);
extern template bool launch_ffn_fused_t<W_Q8_0>(hipStream_t, const FfnFused &, int, bool, int, int, dim3, int);

extern int kQgCUs;

bool ffn_fused_supported(const FfnFused & f, int form, bool hasr) {
    const MVEntry & k = f.e[0];
    const int t = k.W.type, C = k.W.K, F = k.W.M;
    if (!wtype_quantized(t) || !f.kg || !f.x || !f.err || (hasr && !f.rg)) return false;
    if (!(form == 0 && hasr) && !(form == 1)) return false;
    if (k.src != SRC_LNMIX || k.form != form || !k.emit || k.act_out.fmt != act_fmt_for(t) || k.act_out.tiled) return false;
    if (C % 64 || C > 4096 || F % 32 || F / 32 > 512) return false;
    // Only where the whole grid is resident at once with the consumers' value rows in registers:
    // at most 4 units per lane (v6-1B6, v4-169M: 1.6 and 0.7 workgroups per CU) -- v7-2.9B (5 units,
    // 1.9 per CU) measured 1871 vs 1838 us/token and v5-7B (7 units, 3.3 per CU: the consumers
    // start a round late) 2029 vs 1528 against the two launches
    const int np = F / 32 + (hasr ? C / 32 : 0);
    if (f.co) {
        // co-resident form: one value row per consumer wave on the np producer workgroups, all np
        // resident at once -- at one 512-thread workgroup per CU (the Q8_0 forms hold up to 204
        // VGPRs), so np <= the device's compute units
        if (mv_units(t, F) > 8 || 8 * np < C || np > kQgCUs) return false;
    } else if (mv_units(t, F) > 4 || np + C / (8 * FF_RC) > 2 * kQgCUs) {
        return false;
    }
    if (f.wv.type != t || f.wv.M != C || f.wv.K != F) return false;
    if (hasr) {
        const MVEntry & r = f.e[1];
        if (r.src != SRC_LNMIX || r.form != form || r.W.type != t || r.W.K != C || r.W.M != C || r.emit) return false;
        if (r.x != k.x || r.lnw != k.lnw || r.lnb != k.lnb || r.carry != k.carry) return false;
    }
    return true;
}

bool launch_ffn_fused(hipStream_t st, FfnFused & f, int form, bool hasr) {
    if (!ffn_fused_supported(f, form, hasr)) {
        fprintf(stderr, "rwkv: fused channel-mix decode: unsupported shape\n");
        return false;
    }
    const int t = f.e[0].W.type, C = f.e[0].W.K, F = f.e[0].W.M;
    f.e[0].block0 = 0;
    f.e[1].block0 = F / 32;
    f.np = F / 32 + (hasr ? C / 32 : 0);
    const dim3 grid(f.co ? f.np : f.np + (C + 8 * FF_RC - 1) / (8 * FF_RC));
    const int fmt = act_fmt_for(t);
    const int lds = std::max(lds_bytes_for(fmt, C), lds_bytes_for(fmt, F));
    const int uv = mv_units(t, F), lnp = C <= 2048 ? 32 : 64;
    bool ok = false;
    switch (t) {
        case W_Q4_0: ok = launch_ffn_fused_t<W_Q4_0>(st, f, form, hasr, uv, lnp, grid, lds); break;
        case W_Q4_1: ok = launch_ffn_fused_t<W_Q4_1>(st, f, form, hasr, uv, lnp, grid, lds); break;
        case W_Q5_0: ok = launch_ffn_fused_t<W_Q5_0>(st, f, form, hasr, uv, lnp, grid, lds); break;
        case W_Q5_1: ok = launch_ffn_fused_t<W_Q5_1>(st, f, form, hasr, uv, lnp, grid, lds); break;
        case W_Q8_0: ok = launch_ffn_fused_t<W_Q8_0>(st, f, form, hasr, uv, lnp, grid, lds); break;
        default: break;
    }
    if (!ok) return false;
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
