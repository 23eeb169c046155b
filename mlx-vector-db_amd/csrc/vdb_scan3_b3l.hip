// vdb_scan3_b3l.hip — instantiation unit of the large-batch split candidate pass
// (precision 1, metric 1; kernel in vdb_scan3_kernel.h).
#include "vdb_scan3_kernel.h"

namespace vdb {
S3_UNIT(launch_scan3_b3l, 1, 1, VDB_S3_RING_1, VDB_S3_PQ)
}  // namespace vdb
