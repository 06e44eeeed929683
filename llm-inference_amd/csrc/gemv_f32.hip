// GEMV instantiations for float weights (see gemv.hip, gemv_launch.h).
#include "gemv_launch.h"

namespace llmi {
namespace gemv_detail {
template int launch_epi<float>(const GemvArgs& a, int grid, hipStream_t s);
}  // namespace gemv_detail
}  // namespace llmi
