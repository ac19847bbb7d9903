// mv_q8_0.hip -- decode matvec launch shapes for weight type W_Q8_0 (see mv_common.hpp).
#include "mv_common.hpp"

namespace rwkvmi {
template bool launch_mv_shape<W_Q8_0>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
}  // namespace rwkvmi
