// gs_cg_reg_r4.hip -- instantiations of k_cg_regres (the 256-thread form) with 4 thread(s)
// per chain (gs_cg_reg.hpp); a file of its own so it builds in parallel with gs_cg_reg_g4.hip.
#include "gs_cg_reg.hpp"

namespace gs {
GS_REGRES_LAUNCH_DEF(4)
}  // namespace gs
