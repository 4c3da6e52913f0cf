// gh_inst_slots3.hip — explicit instantiations of the slot family's kernels (see gh_inst.h)
#include <hip/hip_runtime.h>
#include "gh_inst.h"

GH_SL_UNIT3(GH_TEMPLATE)
