// gh_inst_pmmh.hip — the PMMH kernel (config C5) in its own unit, built with
// fma_c as a plain fma (see gh_pmmh.h); gh_api.hip launches it by its host stub.
#define GH_FMA_C_PLAIN
#define GH_PMMH_KERNEL
#include <hip/hip_runtime.h>
#include "gh_pmmh.h"
