"""gen_amd — MI355X-native particle-inference engine for Gen's SMC hot path.

The product is libgen_hip.so (hand-written HIP kernels for gfx950 behind the
C ABI in include/gen_hip.h).  This package is its Python host mirror of Gen's
inference API (src/inference/particle_filter.jl, importance.jl); see
DESIGN.md.  Importing it does not touch the GPU; the first call does.
"""
from .choicemap import ChoiceMap, EmptyChoiceMap, Selection, choicemap, select
from .models import BayesianLinearRegression, DiscreteHMM, KitagawaSSM, LinearGaussianSSM, Model, SlotSSM
from .pf import (
    Context,
    NoChange,
    GaussianProposal,
    LinearGaussianProposal,
    OptimalProposal,
    conditional_particle_filter_step,
    conditional_smc,
    get_particle,
    initialize_conditional_particle_filter,
    particle_gibbs,
    ParticleFilterState,
    UnknownChange,
    default_context,
    get_log_weights,
    get_traces,
    importance_resampling,
    importance_sampling,
    initialize_particle_filter,
    log_ml_estimate,
    maybe_resample,
    maybe_resample_async,
    metropolis_hastings,
    gaussian_drift,
    GaussianDriftProposal,
    mh,
    particle_filter_step,
    rejuvenate,
    ObservationBatch,
    prepare_observations,
    run_particle_filter,
    sample_unweighted_traces,
    set_default_context,
)
from .simulate import SimulatedTraces, simulate
from . import dists
from ._lib import GenHipError

__all__ = [
    "ChoiceMap", "EmptyChoiceMap", "choicemap", "BayesianLinearRegression", "DiscreteHMM", "KitagawaSSM", "LinearGaussianSSM", "Model", "SlotSSM",
    "Context", "GaussianProposal", "NoChange", "OptimalProposal", "ParticleFilterState", "UnknownChange", "default_context",
    "get_log_weights", "get_traces", "importance_resampling", "importance_sampling",
    "initialize_particle_filter", "log_ml_estimate", "maybe_resample", "maybe_resample_async",
    "particle_filter_step", "rejuvenate", "run_particle_filter", "sample_unweighted_traces", "set_default_context",
    "conditional_particle_filter_step", "conditional_smc", "get_particle", "initialize_conditional_particle_filter",
    "particle_gibbs", "GenHipError", "ObservationBatch", "prepare_observations", "Selection", "select",
    "metropolis_hastings", "mh", "simulate", "SimulatedTraces", "dists", "gaussian_drift", "GaussianDriftProposal",
]
