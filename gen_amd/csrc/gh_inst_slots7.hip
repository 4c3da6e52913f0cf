// gh_inst_slots7.hip — explicit instantiations of the slot family's kernels for models with a library slot or the switching latent (see gh_inst.h)
#include <hip/hip_runtime.h>
#include "gh_inst.h"

GH_SL_UNIT7(GH_TEMPLATE)
