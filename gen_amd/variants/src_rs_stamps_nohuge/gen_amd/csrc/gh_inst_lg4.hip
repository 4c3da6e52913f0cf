// gh_inst_lg4.hip — explicit instantiations of LG-SSM kernels (see gh_inst.h)
#include <hip/hip_runtime.h>
#include "gh_inst.h"

GH_LG_UNIT4(GH_TEMPLATE)
