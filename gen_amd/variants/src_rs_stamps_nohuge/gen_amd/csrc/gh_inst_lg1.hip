// gh_inst_lg1.hip — explicit instantiations of LG-SSM kernels (see gh_inst.h)
#include <hip/hip_runtime.h>
#include "gh_inst.h"

GH_LG_UNIT1(GH_TEMPLATE)
