// mv_ffnf_q8_0.hip -- k_ffn_fused instantiations for Q8_0 weights (one weight type per translation unit,
// so the launch shapes compile in parallel; mv_ffnf.hpp).
#include "mv_ffnf.hpp"

namespace rwkvmi {
template bool launch_ffn_fused_t<W_Q8_0>(hipStream_t, const FfnFused &, int, bool, int, int, dim3, int);
}  // namespace rwkvmi
