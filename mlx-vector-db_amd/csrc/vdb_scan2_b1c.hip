// vdb_scan2_b1c.hip — instantiation unit of the split candidate pass: bf16, cosine
// (every KP / load policy / step-end variant; kernel in vdb_scan2_kernel.h).
#include "vdb_scan2_kernel.h"

namespace vdb {
#ifndef VDB_S2_B1_PX
#define VDB_S2_B1_PX 4
#endif
S2_UNIT(launch_scan2_b1c, 2, 0, VDB_S2_B1_PX, 4)
}  // namespace vdb

S2_STAMP_READER(b1c)
