// vdb_scan3_b1c.hip — instantiation unit of the large-batch split candidate pass
// (precision 2, metric 0; kernel in vdb_scan3_kernel.h).
#include "vdb_scan3_kernel.h"

namespace vdb {
S3_UNIT(launch_scan3_b1c, 2, 0, VDB_S3_RING_2, VDB_S3_PQ)
}  // namespace vdb
