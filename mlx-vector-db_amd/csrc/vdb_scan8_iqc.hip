// vdb_scan8_iqc.hip — instantiation unit of the int8 candidate pass: the xh plane against the
// 16-bit query (PREC_I8Q), cosine (every KP / load policy / step-end variant; kernel in
// vdb_scan8_kernel.h).
#include "vdb_scan8_kernel.h"

namespace vdb {
S8_UNIT(launch_scan8_iqc, PREC_I8Q, 0, 4, 4)
}  // namespace vdb
