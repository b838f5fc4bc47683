// gs_cg_reg_r2.hip -- instantiations of k_cg_regres (the 256-thread form) with 2 thread(s)
// per chain (gs_cg_reg.hpp); a file of its own so it builds in parallel with gs_cg_reg_g2.hip.
#include "gs_cg_reg.hpp"

namespace gs {
GS_REGRES_LAUNCH_DEF(2)
}  // namespace gs
