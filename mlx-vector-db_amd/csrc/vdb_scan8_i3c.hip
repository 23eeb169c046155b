// vdb_scan8_i3c.hip — instantiation unit of the int8 candidate pass: int8 x3 (two planes), cosine
// (every KP / load policy / step-end variant; kernel in vdb_scan8_kernel.h).
#include "vdb_scan8_kernel.h"

namespace vdb {
S8_UNIT(launch_scan8_i3c, PREC_I8X3, 0, 2, 2)
}  // namespace vdb
