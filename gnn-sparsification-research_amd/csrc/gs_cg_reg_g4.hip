// gs_cg_reg_g4.hip -- instantiations of k_cg_regres and k_cg_regwide with 4 thread(s) per chain
// (gs_cg_reg.hpp); one file per G so the builds run in parallel.
#include "gs_cg_reg.hpp"
#include "gs_cg_wide.hpp"

namespace gs {
GS_REGRES_LAUNCH_DEF(4)
GS_REGWIDE_LAUNCH_DEF(4)
}  // namespace gs
