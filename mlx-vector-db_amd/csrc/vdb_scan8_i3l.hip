// vdb_scan8_i3l.hip — instantiation unit of the int8 candidate pass: int8 x3 (two planes), L2
// (every KP / load policy / step-end variant; kernel in vdb_scan8_kernel.h).
#include "vdb_scan8_kernel.h"

namespace vdb {
S8_UNIT(launch_scan8_i3l, PREC_I8X3, 1, 2, 2)
}  // namespace vdb

#ifdef VDB_STAMP8
extern "C" int vdb_debug_scan8_stamps_i3l(unsigned long long* out, int n_waves) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vdb::g_scan8_stamps), (size_t)n_waves * 12 * sizeof(unsigned long long));
}
#endif
