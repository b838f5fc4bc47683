// gs_cg_reg_g2.hip -- instantiations of k_cg_regres with 2 thread(s) per chain
// (gs_cg_reg.hpp); one file per G so the builds run in parallel.
#include "gs_cg_reg.hpp"

namespace gs {
GS_REGRES_LAUNCH_DEF(2)
}  // namespace gs
