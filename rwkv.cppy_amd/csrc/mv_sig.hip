// mv_sig.hip -- launcher of k_mvsig (mv_common.hpp): the decode channel mix's value and receptance
// matvecs in one launch (rwkv_graph.inc:484-531).
#include "mv_common.hpp"

#include <stdlib.h>
#include <string.h>

namespace rwkvmi {

void mv_fill_hot(const MVEntry & e, MVHot & h) {
    memset(&h, 0, sizeof(h));
    h.qs = e.W.qs;
    h.qh = e.W.qh;
    h.sc = e.W.sc;
    h.aq = e.act.q;
    h.ad = e.act.d;
    h.as = e.act.s;
    h.aqsum = e.act.qsum;
    h.y = e.y;
    h.M = e.W.M;
    h.K = e.W.K;
    h.epi = e.epi;
}

bool mv_sigmul_supported(const MVEntry & ev, const MVEntry & er) {
    const int t = ev.W.type;
    if (!wtype_quantized(t) || er.W.type != t || ev.W.M != er.W.M) return false;
    if (ev.src != SRC_ACT || er.src != SRC_ACT || !ev.y || ev.W.K % 32 || er.W.K % 32) return false;
    if (ev.act.fmt != act_fmt_for(t) || er.act.fmt != act_fmt_for(t) || ev.act.K != ev.W.K || er.act.K != er.W.K)
        return false;
    if (ev.act.tiled || er.act.tiled) return false;
    return mv_units(t, ev.W.K) <= 8 && mv_units(t, er.W.K) <= 2;
}

template <int WF, int U>
static void launch_sig_u2(hipStream_t st, const MVHot & hv, const MVHot & hr, int u2, dim3 grid) {
    if (u2 <= 1) RK_LAUNCH((k_mvsig<WF, 2, U, 1>), grid, dim3(256), 0, st, hv, hr);
    else RK_LAUNCH((k_mvsig<WF, 2, U, 2>), grid, dim3(256), 0, st, hv, hr);
}

template <int WF>
static void launch_sig_t(hipStream_t st, const MVHot & hv, const MVHot & hr, int u, int u2, dim3 grid) {
    if (u <= 1) launch_sig_u2<WF, 1>(st, hv, hr, u2, grid);
    else if (u <= 2) launch_sig_u2<WF, 2>(st, hv, hr, u2, grid);
    else if (u <= 4) launch_sig_u2<WF, 4>(st, hv, hr, u2, grid);
    else launch_sig_u2<WF, 8>(st, hv, hr, u2, grid);
}

bool launch_mv_sigmul(hipStream_t st, const MVEntry & ev, const MVEntry & er) {
    if (!mv_sigmul_supported(ev, er)) {
        fprintf(stderr, "rwkv: channel-mix value+receptance launch: unsupported shape\n");
        return false;
    }
    MVHot hv, hr;
    mv_fill_hot(ev, hv);
    mv_fill_hot(er, hr);
    const int u = mv_units(ev.W.type, ev.W.K), u2 = mv_units(er.W.type, er.W.K);
    const dim3 grid((ev.W.M + 7) / 8);
    switch (ev.W.type) {
        case W_Q4_0: launch_sig_t<W_Q4_0>(st, hv, hr, u, u2, grid); break;
        case W_Q4_1: launch_sig_t<W_Q4_1>(st, hv, hr, u, u2, grid); break;
        case W_Q5_0: launch_sig_t<W_Q5_0>(st, hv, hr, u, u2, grid); break;
        case W_Q5_1: launch_sig_t<W_Q5_1>(st, hv, hr, u, u2, grid); break;
        default: launch_sig_t<W_Q8_0>(st, hv, hr, u, u2, grid); break;
    }
    HIP_OK(hipGetLastError());
    return true;
}

}  // namespace rwkvmi
