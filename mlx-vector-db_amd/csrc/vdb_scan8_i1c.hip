// vdb_scan8_i1c.hip — instantiation unit of the int8 candidate pass: int8 (one plane), cosine
// (every KP / load policy / step-end variant; kernel in vdb_scan8_kernel.h).
#include "vdb_scan8_kernel.h"

namespace vdb {
S8_UNIT(launch_scan8_i1c, PREC_I8, 0, 4, 2)
}  // namespace vdb
