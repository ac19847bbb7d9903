// mv_generic.hip -- decode matvec launch shapes for weight type -1 (see mv_common.hpp).
#include "mv_common.hpp"

namespace rwkvmi {
template bool launch_mv_shape<-1>(hipStream_t, MVGroup &, int, int, int, bool, dim3);
}  // namespace rwkvmi
