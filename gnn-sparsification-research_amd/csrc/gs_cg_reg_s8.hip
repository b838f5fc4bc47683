// gs_cg_reg_s8.hip -- instantiations of the split form of k_cg_regwide (q in registers,
// P workgroups per column) with 8 threads per chain (gs_cg_wide.hpp); a file of its
// own so it builds in parallel with gs_cg_reg_g8.hip.
#include "gs_cg_reg.hpp"
#include "gs_cg_wide.hpp"

namespace gs {
GS_REGWIDE_SPLIT_DEF(8)
}  // namespace gs
