"""bench.py — particle-steps/sec of Gen's particle-filter hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): 10-dim linear-Gaussian SSM (Static
DSL + Unfold), bootstrap particle filter with 2^20 particles per GPU,
systematic resampling at ESS < N/2, synthetic observations simulated from the
model.  One "step" = one pass of the hot path over the particle set: the
reference's caller loop body {maybe_resample!; particle_filter_step!}
(test/inference/particle_filter.jl:157-162) for one time step.

value = whole-job particle-steps/s = N_global * K / (max over ranks of the
timed region).  Multi-GPU (torchrun): particles shard across ranks (weak
scaling, 2^20 per GPU) and the ranks form ONE filter: RCCL all-gathers the
(max, sum, sum^2) weight triple every step and the integer CDF totals plus
the ancestor states on resample steps.

Also reported:
  roofline     achieved HBM GB/s of the dominant kernel (k_step) from its
               algorithmic bytes (16d+16 per particle-step, +4 on resample
               steps) / its hipEvent-timed average duration on its stream;
               traffic = PMC HBM bytes per launch from profiles/ when present.
  cpu_baseline the CPU oracle (C restatement of Gen's PF, 1 core) on a bounded
               sample of the same workload, timed on this host; its "parity"
               entry runs the GPU filter and the oracle on the same
               observations, seed and 2^16 particles and reports the log-ML
               relative difference (north star: <= 1e-6) and whether the final
               ancestors agree bit for bit.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--particles", type=int, default=1 << 20, help="particles per GPU")
    p.add_argument("--d", type=int, default=10)
    p.add_argument("--model", default="lgssm", choices=["lgssm", "kitagawa"],
                   help="lgssm: C2 (the headline); kitagawa: the C4 nonlinear SSM")
    p.add_argument("--resampler", default="systematic")
    p.add_argument("--proposal", default="default", choices=["default", "optimal"],
                   help="optimal: the LG-SSM's locally optimal proposal (a custom proposal; not the headline)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-history", action="store_true")
    p.add_argument("--ess-threshold", type=float, default=None, help="default N/2 (the reference's default)")
    p.add_argument("--no-kernel-timing", action="store_true", help="no hipEvents around the step kernel")
    p.add_argument("--transport", default="rccl", choices=["rccl", "gloo"],
                   help="multi-GPU collectives: RCCL (default) or the host-staged gloo transport "
                        "(ranks may share a GPU; a correctness rehearsal, not a benchmark)")
    p.add_argument("--time-every", type=int, default=None,
                   help="time every k-th step kernel with launch events (default: steps // 2, i.e. two timed "
                        "launches in the timed region; each timed launch costs the run 25-60 us, measured)")
    return p.parse_args()


def cpu_parity(model, ys, n, resampler, proposal):
    """The GPU filter and the CPU restatement of Gen's filter (oracle/) on the
    same workload, seed and N = n over every observation of the run: their
    log-ML estimates (the north star's "within 1e-6 relative on fixed RNG
    seeds") and whether the final ancestors agree bit for bit."""
    import gen_amd as gen
    from oracle import oracle as O

    prop = gen.OptimalProposal if proposal == "optimal" else None
    st = gen.initialize_particle_filter(model, (1,), {("chain", 1, "y"): ys[0]},
                                        *((prop, (), n) if prop is not None else (n,)), seed=42, resampler=resampler)
    gen.run_particle_filter(st, list(ys[1:]), None, proposal=prop)
    gpu = gen.log_ml_estimate(st)
    gpu_parents = st.parents
    st.close()
    orc = O.run_pf(model, ys, n, 42, resampler=O.SYSTEMATIC if resampler == "systematic" else O.MULTINOMIAL,
                   proposal=O.OPTIMAL if prop is not None else O.DEFAULT, record_history=False)
    cpu = orc.log_ml_estimate()
    return {"particles": n, "steps": len(ys), "seed": 42, "log_ml_gpu": gpu, "log_ml_cpu": cpu,
            "rel": abs(gpu - cpu) / abs(cpu), "parents_bitexact": bool((gpu_parents == orc.parents()).all())}


def cpu_baseline(model, ys, budget_s):
    """The oracle (scalar C, 1 core) on N = 2^14 particles, as many steps of
    the same workload as fit in ~budget_s seconds."""
    from oracle import oracle as O

    n = 1 << 14
    pf = O.OraclePF(model, n, 42, record_history=False)
    t0 = time.perf_counter()
    pf.init(ys[0])
    steps = 0
    i = 1
    while time.perf_counter() - t0 < budget_s:
        pf.maybe_resample()
        pf.step(ys[i % len(ys)])
        i += 1
        steps += 1
    dt = time.perf_counter() - t0
    return {
        "value": n * (steps + 1) / dt,
        "unit": "particle-steps/s",
        "cores": 1,
        "kind": "port",
        "sample": f"oracle/gh_oracle.c (C restatement of Gen's PF, not Gen.jl: no Julia on the box), "
                  f"LG-SSM d={model.d}, N={n}, {steps + 1} steps incl. init, {dt:.1f} s",
    }


def main():
    a = parse()
    if a.time_every is None:
        a.time_every = max(1, a.steps // 2)
    import gen_amd as gen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        if a.transport == "gloo":
            import torch

            from gen_amd.transport import GlooTransport

            ctx = gen.Context(device=local % max(1, torch.cuda.device_count()), transport=GlooTransport())
        else:
            uid = [gen.Context.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            ctx = gen.Context(device=local, rank=rank, world=world, unique_id=uid[0])
    else:
        ctx = gen.Context(device=0)
    gen.set_default_context(ctx)

    if a.model == "lgssm":
        model = gen.LinearGaussianSSM.benchmark(a.d)
    else:
        model = gen.KitagawaSSM(10.0, 1.0)  # examples/pmmh/run.jl:69 (var_x = 10, var_y = 1)
    T = a.warmup + a.steps + 1
    _, ys = model.simulate(T, np.random.default_rng(2 if a.model == "lgssm" else 3))
    n_global = a.particles * world
    prop = gen.OptimalProposal if a.proposal == "optimal" else None
    init_args = (prop, (), n_global) if prop is not None else (n_global,)
    st = gen.initialize_particle_filter(
        model, (1,), {("chain", 1, "y"): ys[0]}, *init_args, seed=42, resampler=a.resampler,
        record_history=not a.no_history, history_capacity=T + 2, time_kernels=0 if a.no_kernel_timing else a.time_every,
    )
    gen.run_particle_filter(st, list(ys[1 : 1 + a.warmup]), a.ess_threshold, proposal=prop)
    ctx.synchronize()
    st.kernel_time_ms(reset=True)
    ess0, did0 = st.ess_history()

    def barrier():
        ctx.synchronize()
        if dist is not None:
            dist.barrier()

    # the observations of the timed steps, marshalled into the C ABI's gh_obs
    # array before the clock starts (inputs ready, as the workload's data)
    batch = gen.prepare_observations(model, list(ys[1 + a.warmup : 1 + a.warmup + a.steps]))
    barrier()
    t0 = time.perf_counter()
    gen.run_particle_filter(st, batch, a.ess_threshold, proposal=prop)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch

        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    kms, kcount = st.kernel_time_ms()
    ess, did = st.ess_history()
    n_res = int(did[a.warmup : a.warmup + a.steps].sum())  # resamples ahead of the timed steps
    lml = gen.log_ml_estimate(st)

    d = a.d if a.model == "lgssm" else 1
    bytes_pp = 16 * d + 16 + 4.0 * n_res / max(1, a.steps)
    achieved = bytes_pp * st.n_local / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    traffic = None
    # PMC HBM bytes per step-kernel launch of the profiled configs (tools/pmc_json.py)
    pmc = None
    if a.model == "lgssm" and a.d == 10 and a.particles == 1 << 20 and prop is None:
        pmc = os.path.join(ROOT, "profiles", "pmc_k_step.json")
    elif a.model == "kitagawa" and a.particles == 1 << 21:
        pmc = os.path.join(ROOT, "profiles", "pmc_k_step_kitagawa.json")
    if pmc is not None and os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    value = n_global * a.steps / dt
    log_ml_error = None
    if a.model == "lgssm":
        exact = model.kalman_log_marginal(ys[: 1 + a.warmup + a.steps])
        log_ml_error = {"reference": "Kalman filter (exact)", "exact": exact,
                        "abs": abs(lml - exact), "rel": abs(lml - exact) / abs(exact)}
    out = {
        "metric": ("particle-steps/sec (whole node) + log-ML error vs CPU ref, 1M-particle SSM" if a.model == "lgssm"
                   else "particle-steps/sec (whole node), nonlinear SSM (C4)"),
        "value": value,
        "unit": "particle-steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic (observations simulated from the model, numpy seed {2 if a.model == 'lgssm' else 3})",
        "config": {
            "workload": (f"C2: {a.d}-dim linear-Gaussian SSM " + ("optimal-proposal PF" if prop else "bootstrap PF")
                         if a.model == "lgssm" else
                         "C4: Kitagawa nonlinear SSM bootstrap PF") + f", {a.particles} particles/GPU, "
                        f"systematic resampling at ESS<N/2, record_history={not a.no_history}",
            "particles_global": n_global,
            "d": d,
            "resampler": a.resampler,
            "parallelism": f"particle-dp{world}",
            "resample_steps_timed": n_res,
            "log_ml": lml,
        },
        # log-ML error against the exact answer of the CPU reference's target
        # (Kalman filter over the same observations; C2 only).  The estimate's
        # Monte-Carlo error at this N dominates it; parity with the CPU
        # restatement of Gen's filter at equal seeds is 1e-9 (tests/).
        "log_ml_error": log_ml_error,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": (f"k_step<LGOptModel<{a.d}>,false>" if prop else f"k_step<LGModel<{a.d},3>,false>")
                      if a.model == "lgssm" else "k_step<KitModel,false>",
            "kernel_avg_ms": kms,
            "kernel_launches": kcount,
            "bytes_per_particle_step": bytes_pp,
            # the whole step (every kernel and gap) against the same bytes
            "step_frac": bytes_pp * n_global / world / (dt / a.steps) / 1e9 / HBM_PEAK_GBS,
        },
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(model, ys, a.cpu_seconds)
        # same seed, same observations, N = 2^16: GPU vs the CPU restatement
        par = cpu_parity(model, ys, 1 << 16, a.resampler, a.proposal)
        out["cpu_baseline"]["parity"] = par
        if out["log_ml_error"] is not None:
            out["log_ml_error"]["vs_cpu_reference_same_seed"] = {"particles": par["particles"], "rel": par["rel"]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    st.close()
    if dist is not None:
        dist.barrier()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
