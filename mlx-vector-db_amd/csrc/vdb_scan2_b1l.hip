// vdb_scan2_b1l.hip — instantiation unit of the split candidate pass: bf16, L2
// (every KP / load policy / step-end variant; kernel in vdb_scan2_kernel.h).
#include "vdb_scan2_kernel.h"

namespace vdb {
S2_UNIT(launch_scan2_b1l, 2, 1, 4, 4)
}  // namespace vdb

S2_STAMP_READER(b1l)
