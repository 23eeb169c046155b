// vdb_scan8_i1l.hip — instantiation unit of the int8 candidate pass: int8 (one plane), L2
// (every KP / load policy / step-end variant; kernel in vdb_scan8_kernel.h).
#include "vdb_scan8_kernel.h"

namespace vdb {
S8_UNIT(launch_scan8_i1l, PREC_I8, 1, 4, 4)
}  // namespace vdb
