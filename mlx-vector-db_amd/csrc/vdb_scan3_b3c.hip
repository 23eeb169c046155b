// vdb_scan3_b3c.hip — instantiation unit of the large-batch split candidate pass
// (precision 1, metric 0; kernel in vdb_scan3_kernel.h).
#include "vdb_scan3_kernel.h"

namespace vdb {
S3_UNIT(launch_scan3_b3c, 1, 0, VDB_S3_RING_1, VDB_S3_PQ)
}  // namespace vdb
