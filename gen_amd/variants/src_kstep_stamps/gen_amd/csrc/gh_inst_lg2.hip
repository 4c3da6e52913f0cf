// gh_inst_lg2.hip — explicit instantiations of LG-SSM kernels (see gh_inst.h)
#include <hip/hip_runtime.h>
#include "gh_inst.h"

GH_LG_UNIT2(GH_TEMPLATE)

// (the stamps live in this unit's code object: the LG-SSM kernels of d = 10, 11)
extern "C" int gh_debug_ks_stamps(uint64_t* out, int n) {
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(gh::g_ks_stamps), sizeof(uint64_t) * 4 * (size_t)n) == hipSuccess ? 0 : 5;
}
