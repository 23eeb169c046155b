// vdb_scan2_b3c.hip — instantiation unit of the split candidate pass: bf16x3, cosine
// (every KP / load policy / step-end variant; kernel in vdb_scan2_kernel.h).
#include "vdb_scan2_kernel.h"

namespace vdb {
S2_UNIT(launch_scan2_b3c, 1, 0, 2, VDB_S2_QLDS_PX)
}  // namespace vdb

S2_STAMP_READER(b3c)
