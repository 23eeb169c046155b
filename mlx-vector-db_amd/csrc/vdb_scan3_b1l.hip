// vdb_scan3_b1l.hip — instantiation unit of the large-batch split candidate pass
// (precision 2, metric 1; kernel in vdb_scan3_kernel.h).
#include "vdb_scan3_kernel.h"

namespace vdb {
S3_UNIT(launch_scan3_b1l, 2, 1, VDB_S3_RING_2, VDB_S3_PQ)
}  // namespace vdb
