// vdb_scan8_i1c.hip — instantiation unit of the int8 candidate pass: int8 (one plane), cosine
// (every KP / load policy / step-end variant; kernel in vdb_scan8_kernel.h).
#include "vdb_scan8_kernel.h"

#ifndef VDB_S8_PX1
#define VDB_S8_PX1 4  // corpus groups in flight, query operand from L2 (A/B: make variant VDEFS=-DVDB_S8_PX1=8)
#endif

namespace vdb {
S8_UNIT(launch_scan8_i1c, PREC_I8, 0, VDB_S8_PX1, 4)
}  // namespace vdb

#ifdef VDB_STAMP8
extern "C" int vdb_debug_scan8_stamps_i1c(unsigned long long* out, int n_waves) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vdb::g_scan8_stamps), (size_t)n_waves * 12 * sizeof(unsigned long long));
}
#endif
