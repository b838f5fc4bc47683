// gs_cg_reg_g2.hip -- instantiations of k_cg_regwide with 2 thread(s) per chain
// (gs_cg_wide.hpp); one file per G (and gs_cg_reg_r*.hip for k_cg_regres) so the builds
// run in parallel.
#include "gs_cg_reg.hpp"
#include "gs_cg_wide.hpp"

namespace gs {
GS_REGWIDE_LAUNCH_DEF(2)
}  // namespace gs
