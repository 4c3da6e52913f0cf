// gh_inst_slots0.hip — explicit instantiations of the slot family's kernels (see gh_inst.h)
#include <hip/hip_runtime.h>
#include "gh_inst.h"

GH_SL_UNIT0(GH_TEMPLATE)
