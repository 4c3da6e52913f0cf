// gh_inst.h — the per-model kernels of the LG-SSM family (LGModel<D, S> for
// d = 1..16 and the four exact-zero structures, LGOptModel<D>) are explicitly
// instantiated in gh_inst_lg*.hip and only declared (extern template) in
// gh_api.hip, so the library's ~600 kernels compile in parallel translation
// units.  The kernels' host stubs are ordinary external symbols: a launch in
// gh_api.hip finds the code object registered by the instantiating unit.
#pragma once
#include "gh_kernels.h"
#include "gh_rejuv.h"
#include "gh_scores.h"
#include "gh_simulate.h"
#include "gh_csmc.h"
#include "gh_slots.h"

// X is `extern template` (declaration) or `template` (definition)
#define GH_LG_KERNELS(X, D, S)                                                                               \
  X __global__ void gh::k_step<gh::LGModel<D, S>, true>(const double*, gh::LGParams, gh::StepObs, gh::StepArgs); \
  X __global__ void gh::k_step<gh::LGModel<D, S>, false>(const double*, gh::LGParams, gh::StepObs, gh::StepArgs); \
  X __global__ void gh::k_step<gh::LGModel<D, S>, false, true>(const double*, gh::LGParams, gh::StepObs,         \
                                                               gh::StepArgs);                                    \
  X __global__ void gh::k_rejuv<gh::LGModel<D, S>, true>(const double*, gh::LGParams, gh::StepObs, gh::RejuvArgs); \
  X __global__ void gh::k_rejuv<gh::LGModel<D, S>, false>(const double*, gh::LGParams, gh::StepObs,              \
                                                          gh::RejuvArgs);                                        \
  X __global__ void gh::k_mh_drift<gh::LGModel<D, S>, true>(const double*, gh::LGParams, gh::StepObs,            \
                                                            gh::RejuvArgs, gh::DriftSd);                         \
  X __global__ void gh::k_mh_drift<gh::LGModel<D, S>, false>(const double*, gh::LGParams, gh::StepObs,           \
                                                             gh::RejuvArgs, gh::DriftSd);                        \
  X __global__ void gh::k_scores<gh::LGModel<D, S>>(const double*, gh::LGParams, gh::ScoreArgs,                 \
                                                    const gh::DevScalars*);                                      \
  X __global__ void gh::k_simulate<gh::LGModel<D, S>>(const double*, gh::LGParams, gh::SimArgs);                 \
  X __global__ void gh::k_mr_slot_scores<gh::LGModel<D, S>>(const double*, gh::LGParams, gh::StepObs, int,     \
                                                             const double*, const double*, const int32_t*,       \
                                                             const double*, int64_t, int64_t, int64_t, double*,  \
                                                             int*);                                              \
  X __global__ void gh::k_pin_pre<gh::LGModel<D, S>, true>(const double*, gh::LGParams, gh::StepObs, gh::PinArgs); \
  X __global__ void gh::k_pin_pre<gh::LGModel<D, S>, false>(const double*, gh::LGParams, gh::StepObs, gh::PinArgs);

#define GH_LGO_KERNELS(X, D)                                                                                   \
  X __global__ void gh::k_step<gh::LGOptModel<D>, true>(const double*, gh::LGParams, gh::StepObs, gh::StepArgs); \
  X __global__ void gh::k_step<gh::LGOptModel<D>, false>(const double*, gh::LGParams, gh::StepObs, gh::StepArgs); \
  X __global__ void gh::k_step<gh::LGOptModel<D>, false, true>(const double*, gh::LGParams, gh::StepObs,           \
                                                               gh::StepArgs);                                      \
  X __global__ void gh::k_step<gh::LGLinModel<D>, true>(const double*, gh::LGParams, gh::StepObs, gh::StepArgs); \
  X __global__ void gh::k_step<gh::LGLinModel<D>, false>(const double*, gh::LGParams, gh::StepObs, gh::StepArgs); \
  X __global__ void gh::k_step<gh::LGLinModel<D>, false, true>(const double*, gh::LGParams, gh::StepObs,           \
                                                               gh::StepArgs);

#define GH_LG_DIM(X, D)      \
  GH_LG_KERNELS(X, D, 0)     \
  GH_LG_KERNELS(X, D, 1)     \
  GH_LG_KERNELS(X, D, 2)     \
  GH_LG_KERNELS(X, D, 3)     \
  GH_LGO_KERNELS(X, D)

// the dimensions of each instantiating unit (gh_inst_lg<k>.hip), balanced by
// kernel size (the mat-vec grows as d^2)
#define GH_LG_UNIT0(X) GH_LG_DIM(X, 1) GH_LG_DIM(X, 2) GH_LG_DIM(X, 3) GH_LG_DIM(X, 4) GH_LG_DIM(X, 5) GH_LG_DIM(X, 6)
#define GH_LG_UNIT1(X) GH_LG_DIM(X, 7) GH_LG_DIM(X, 8) GH_LG_DIM(X, 9)
#define GH_LG_UNIT2(X) GH_LG_DIM(X, 10) GH_LG_DIM(X, 11)
#define GH_LG_UNIT3(X) GH_LG_DIM(X, 12) GH_LG_DIM(X, 13)
#define GH_LG_UNIT4(X) GH_LG_DIM(X, 14)
#define GH_LG_UNIT5(X) GH_LG_DIM(X, 15)
#define GH_LG_UNIT6(X) GH_LG_DIM(X, 16)

// the slot family (gh_slots.h): SlotModel<D> for d = 1..16, in gh_inst_slots<k>.hip
#define GH_SL_KERNELS_L(X, D, L)                                                                                     \
  X __global__ void gh::k_step<gh::SlotModel<D, L>, true>(const double*, gh::SlotParams, gh::StepObs, gh::StepArgs); \
  X __global__ void gh::k_step<gh::SlotLinModel<D, L>, true>(const double*, gh::SlotParams, gh::StepObs,             \
                                                          gh::StepArgs);                                          \
  X __global__ void gh::k_step<gh::SlotLinModel<D, L>, false>(const double*, gh::SlotParams, gh::StepObs,            \
                                                           gh::StepArgs);                                         \
  X __global__ void gh::k_step<gh::SlotLinModel<D, L>, false, true>(const double*, gh::SlotParams, gh::StepObs,      \
                                                                 gh::StepArgs);                                   \
  X __global__ void gh::k_step<gh::SlotModel<D, L>, false>(const double*, gh::SlotParams, gh::StepObs, gh::StepArgs); \
  X __global__ void gh::k_step<gh::SlotModel<D, L>, false, true>(const double*, gh::SlotParams, gh::StepObs,          \
                                                              gh::StepArgs);                                     \
  X __global__ void gh::k_rejuv<gh::SlotModel<D, L>, true>(const double*, gh::SlotParams, gh::StepObs, gh::RejuvArgs); \
  X __global__ void gh::k_rejuv<gh::SlotModel<D, L>, false>(const double*, gh::SlotParams, gh::StepObs,              \
                                                         gh::RejuvArgs);                                         \
  X __global__ void gh::k_mh_drift<gh::SlotModel<D, L>, true>(const double*, gh::SlotParams, gh::StepObs,            \
                                                           gh::RejuvArgs, gh::DriftSd);                          \
  X __global__ void gh::k_mh_drift<gh::SlotModel<D, L>, false>(const double*, gh::SlotParams, gh::StepObs,           \
                                                            gh::RejuvArgs, gh::DriftSd);                         \
  X __global__ void gh::k_scores<gh::SlotModel<D, L>>(const double*, gh::SlotParams, gh::ScoreArgs,                 \
                                                   const gh::DevScalars*);                                       \
  X __global__ void gh::k_simulate<gh::SlotModel<D, L>>(const double*, gh::SlotParams, gh::SimArgs);                 \
  X __global__ void gh::k_mr_slot_scores<gh::SlotModel<D, L>>(const double*, gh::SlotParams, gh::StepObs, int,     \
                                                            const double*, const double*, const int32_t*,        \
                                                            const double*, int64_t, int64_t, int64_t, double*,   \
                                                            int*);                                               \
  X __global__ void gh::k_pin_pre<gh::SlotModel<D, L>, true>(const double*, gh::SlotParams, gh::StepObs, gh::PinArgs); \
  X __global__ void gh::k_pin_pre<gh::SlotModel<D, L>, false>(const double*, gh::SlotParams, gh::StepObs, gh::PinArgs);
// (L: the extended instantiations — a library slot or the switching latent — gh_inst_slots4..7.hip)
#define GH_SL_KERNELS(X, D) GH_SL_KERNELS_L(X, D, false)
#define GH_SLL_KERNELS(X, D) GH_SL_KERNELS_L(X, D, true)
#define GH_SL_UNIT0(X) \
  GH_SL_KERNELS(X, 1) GH_SL_KERNELS(X, 2) GH_SL_KERNELS(X, 3) GH_SL_KERNELS(X, 4) GH_SL_KERNELS(X, 5) GH_SL_KERNELS(X, 6)
#define GH_SL_UNIT1(X) GH_SL_KERNELS(X, 7) GH_SL_KERNELS(X, 8) GH_SL_KERNELS(X, 9) GH_SL_KERNELS(X, 10)
#define GH_SL_UNIT2(X) GH_SL_KERNELS(X, 11) GH_SL_KERNELS(X, 12) GH_SL_KERNELS(X, 13)
#define GH_SL_UNIT3(X) GH_SL_KERNELS(X, 14) GH_SL_KERNELS(X, 15) GH_SL_KERNELS(X, 16)
#define GH_SL_UNIT4(X) \
  GH_SLL_KERNELS(X, 1) GH_SLL_KERNELS(X, 2) GH_SLL_KERNELS(X, 3) GH_SLL_KERNELS(X, 4) GH_SLL_KERNELS(X, 5) GH_SLL_KERNELS(X, 6)
#define GH_SL_UNIT5(X) GH_SLL_KERNELS(X, 7) GH_SLL_KERNELS(X, 8) GH_SLL_KERNELS(X, 9) GH_SLL_KERNELS(X, 10)
#define GH_SL_UNIT6(X) GH_SLL_KERNELS(X, 11) GH_SLL_KERNELS(X, 12) GH_SLL_KERNELS(X, 13)
#define GH_SL_UNIT7(X) GH_SLL_KERNELS(X, 14) GH_SLL_KERNELS(X, 15) GH_SLL_KERNELS(X, 16)

#define GH_EXTERN_TEMPLATE extern template
#define GH_TEMPLATE template
