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
               algorithmic bytes (16d+16 per particle-step: on a resample
               step the log-weight is not read, and the 4-byte range mark
               read and the 4-byte ancestor record take its 8 bytes) / its
               hipEvent-timed average duration on its stream;
               traffic = PMC HBM bytes per launch from profiles/ when present;
               step_frac = the same bytes per whole step / ms_per_step / peak.
  cpu_baseline the CPU oracle (C restatement of Gen's PF) on a bounded sample
               of the same workload, timed on this host with the OpenMP build
               on the CPU share the GPU box gives this job (OMP_NUM_THREADS;
               the host's CPU count, affinity and cgroup quota are recorded
               beside it) and on one core (median of 5 repetitions each); its
               "parity" entry runs the GPU filter and the oracle on the
               headline configuration itself — the same observations (every
               step of the run), seed and 2^20 particles — and reports the
               log-ML relative difference (north star: <= 1e-6) and whether
               the final states and ancestors agree bit for bit.
  secondary    (one GPU, rank 0) the other GPU configurations of BASELINE.json
               measured in the same run, each with its own CPU baseline:
               C4 the nonlinear SSM at 2^21 particles per GPU (the 8-GPU
               scaling config's shard), C3 coal RJMCMC 2^20 chains x 1000
               steps, C5 PMMH 2^16 chains x 256 inner particles.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse(argv=None):
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
    p.add_argument("--cpu-seconds", type=float, default=1.5, help="seconds per CPU repetition (5 per baseline)")
    p.add_argument("--no-secondary", action="store_true", help="skip the C3 / C4 / C5 measurements")
    p.add_argument("--no-history", action="store_true")
    p.add_argument("--ess-threshold", type=float, default=None, help="default N/2 (the reference's default)")
    p.add_argument("--force-multirank", action="store_true",
                   help="one GPU on the multi-rank code path (a one-rank RCCL communicator; profiling)")
    p.add_argument("--no-kernel-timing", action="store_true", help="no hipEvents around the step kernel")
    p.add_argument("--transport", default="peer", choices=["peer", "rccl", "gloo"],
                   help="multi-GPU exchange: peer (default: the ranks' kernels store into each other's mapped "
                        "mailboxes and row buffers, IPC handles swapped over gloo; falls back to RCCL if the "
                        "mapping fails), RCCL collectives, or the host-staged gloo transport (ranks may share a "
                        "GPU; a correctness rehearsal, not a benchmark)")
    p.add_argument("--time-every", type=int, default=None,
                   help="time every k-th step kernel with launch events (default: steps // 5, at most 10, so at "
                        "least 5 launches of the timed region are averaged in kernel_avg_ms)")
    return p.parse_args(argv)


# ------------------------------------------------------------ CPU baselines
def host_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:  # cgroup v2 CPU bandwidth: "max 100000" or "<quota> <period>"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def median_rate(fn, reps=5):
    """fn() -> (units, seconds); the median rate over reps repetitions."""
    rates = []
    for _ in range(reps):
        u, dt = fn()
        rates.append(u / dt)
    return statistics.median(rates), rates


def cpu_pair(make_sample, unit, sample_desc, reps=5):
    """The oracle on the job's CPU share (OpenMP build, omp_get_max_threads()
    threads) and on one core, median of `reps` repetitions each: the OpenMP
    value is the reported baseline, `cores` the threads it used."""
    from oracle import oracle as O

    out = {}
    for omp in (True, False):
        O.set_openmp(omp)
        threads = O.num_threads()
        med, rates = median_rate(make_sample(threads), reps)
        out[omp] = {"value": med, "cores": threads, "repetitions": [round(r, 1) for r in rates]}
    O.set_openmp(False)
    host = host_info()
    cores = out[True]["cores"]
    why = None
    if cores != host["affinity_cpus"]:
        why = (f"{cores} threads = OMP_NUM_THREADS={host['OMP_NUM_THREADS']} set by the GPU box: this job's CPU "
               f"share of a host whose {host['affinity_cpus']} CPUs serve every GPU of the machine")
    return {
        "value": out[True]["value"],
        "unit": unit,
        "cores": cores,
        "cores_note": why,
        "kind": "port",
        "sample": sample_desc + " (oracle/gh_oracle.c, the C restatement of Gen's algorithm — not Gen.jl: no "
                                f"Julia on the box; OpenMP build on {cores} threads, median of 5)",
        "single_core": {"value": out[False]["value"], "cores": 1, "repetitions": out[False]["repetitions"]},
        "repetitions": out[True]["repetitions"],
        "host": host,
    }


def pf_cpu_baseline(model, ys, budget_s):
    """The oracle's PF on a bounded sample of the same workload: N = 2^14
    particles per thread, as many {maybe_resample!; step} as fit in budget_s."""
    from oracle import oracle as O

    def make(threads):
        n = (1 << 14) * max(1, threads)

        def sample():
            pf = O.OraclePF(model, n, 42, record_history=False)
            pf.init(ys[0])
            t0 = time.perf_counter()
            steps, i = 0, 1
            while time.perf_counter() - t0 < budget_s:
                pf.maybe_resample()
                pf.step(ys[i % len(ys)])
                i += 1
                steps += 1
            return n * steps, time.perf_counter() - t0
        return sample

    name = f"LG-SSM d={model.d}" if hasattr(model, "A") else "Kitagawa SSM"
    return cpu_pair(make, "particle-steps/s", f"{name}, N = 2^14 per thread, {budget_s:.1f} s per repetition")


def cpu_parity(model, ys, n, resampler, proposal):
    """The GPU filter and the CPU restatement of Gen's filter (oracle/, the
    OpenMP build: identical results on any thread count) on the same
    workload, seed and N = n over every observation of the run: their log-ML
    estimates (the north star's "within 1e-6 relative on fixed RNG seeds")
    and whether the final states and ancestors agree bit for bit."""
    import gen_amd as gen
    from oracle import oracle as O

    prop = gen.OptimalProposal if proposal == "optimal" else None
    st = gen.initialize_particle_filter(model, (1,), {("chain", 1, "y"): ys[0]},
                                        *((prop, (), n) if prop is not None else (n,)), seed=42, resampler=resampler)
    gen.run_particle_filter(st, list(ys[1:]), None, proposal=prop)
    gpu = gen.log_ml_estimate(st)
    gpu_parents = st.parents
    gpu_states = st.states()
    st.close()
    O.set_openmp(True)
    t0 = time.perf_counter()
    orc = O.run_pf(model, ys, n, 42, resampler=O.SYSTEMATIC if resampler == "systematic" else O.MULTINOMIAL,
                   proposal=O.OPTIMAL if prop is not None else O.DEFAULT, record_history=False)
    cpu_s = time.perf_counter() - t0
    O.set_openmp(False)
    cpu = orc.log_ml_estimate()
    return {"particles": n, "steps": len(ys), "seed": 42, "log_ml_gpu": gpu, "log_ml_cpu": cpu,
            "rel": abs(gpu - cpu) / abs(cpu), "parents_bitexact": bool((gpu_parents == orc.parents()).all()),
            "states_bitexact": bool(np.array_equal(gpu_states.T.view(np.uint64), orc.state().view(np.uint64))),
            "cpu_seconds": round(cpu_s, 2)}


def pmc_profile(name):
    path = os.path.join(ROOT, "profiles", name)
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


def set_traffic(roofline, pmc, tol=0.15):
    """roofline.traffic = the committed PMC profile's HBM bytes per launch —
    only when that profile timed the same kernel this run timed: its
    rocprofv3 average within `tol` of this run's event average (a stale file,
    made from other code, is not passed off as this run's traffic)."""
    roofline["traffic"] = None
    if not pmc or "hbm_bytes_per_launch" not in pmc:
        roofline["traffic_note"] = "no PMC profile for this configuration"
        return
    kms = roofline.get("kernel_avg_ms") or 0.0
    pms = pmc.get("avg_duration_ns", 0.0) * 1e-6
    roofline["traffic_source"] = pmc.get("source")
    if kms <= 0 or pms <= 0 or abs(pms - kms) > tol * kms:
        roofline["traffic_note"] = (f"null: the PMC profile's kernel average ({pms * 1e3:.2f} us, {pmc.get('source')}) "
                                    f"differs from this run's ({kms * 1e3:.2f} us) by more than {tol:.0%}")
        return
    roofline["traffic"] = pmc["hbm_bytes_per_launch"]
    roofline["traffic_profile_avg_ms"] = pms


# --------------------------------------------------------------- PF runs
def pf_run(gen, ctx, dist, world, a, model, particles, kernel_name, bytes_fn, loop="run"):
    """One filter: init, warm-up steps, then the timed region over K steps
    (barrier + device sync on both sides, max over ranks).  loop: "run" =
    gh_pf_run (the batched loop); "cbc" = the reference caller loop, one
    gh_pf_maybe_resample(did, ess) + gh_pf_step per step through the C ABI as
    a Julia ccall shim issues them (test/inference/particle_filter.jl:130-137);
    "cbc_async" = the same with the decision not asked for (NULL did / ess)."""
    T = a.warmup + a.steps + 1
    seed_data = 2 if isinstance(model, gen.LinearGaussianSSM) else 3
    _, ys = model.simulate(T, np.random.default_rng(seed_data))
    n_global = particles * world
    prop = gen.OptimalProposal if a.proposal == "optimal" and isinstance(model, gen.LinearGaussianSSM) else None
    init_args = (prop, (), n_global) if prop is not None else (n_global,)
    st = gen.initialize_particle_filter(
        model, (1,), {("chain", 1, "y"): ys[0]}, *init_args, seed=42, resampler=a.resampler,
        record_history=not a.no_history, history_capacity=T + 2, time_kernels=0 if a.no_kernel_timing else a.time_every,
        ctx=ctx,
    )
    if dist is not None:  # (the ranks' allocations and first launches take different times)
        ctx.synchronize()
        dist.barrier()
    gen.run_particle_filter(st, list(ys[1 : 1 + a.warmup]), a.ess_threshold, proposal=prop)
    ctx.synchronize()
    st.kernel_time_ms(reset=True)
    # the observations of the timed steps, marshalled into the C ABI's gh_obs
    # array before the clock starts (inputs ready, as the workload's data)
    batch = gen.prepare_observations(model, list(ys[1 + a.warmup : 1 + a.warmup + a.steps]))

    def barrier():
        ctx.synchronize()
        if dist is not None:
            dist.barrier()

    if loop != "run":
        import ctypes

        from gen_amd import _lib

        lib = _lib.load()
        thr = float(n_global / 2 if a.ess_threshold is None else a.ess_threshold)
        did, ess = ctypes.c_int(), ctypes.c_double()
        pd, pe = (ctypes.byref(did), ctypes.byref(ess)) if loop == "cbc" else (None, None)
        obs = [ctypes.byref(batch.arr[i]) for i in range(a.steps)]
        mr_fn, step_fn, h = lib.gh_pf_maybe_resample, lib.gh_pf_step, st.h
    barrier()
    t0 = time.perf_counter()
    if loop == "run":
        gen.run_particle_filter(st, batch, a.ess_threshold, proposal=prop)
    else:
        for i in range(a.steps):
            rc = mr_fn(h, thr, pd, pe) or step_fn(h, obs[i], 0)
            if rc:
                _lib.check(rc)
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
    bytes_pp = bytes_fn(n_res)
    achieved = bytes_pp * st.n_local / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    st.close()
    return {
        "ys": ys, "dt": dt, "n_global": n_global, "n_res": n_res, "lml": lml, "prop": prop,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": kernel_name,
            "kernel_avg_ms": kms,
            "kernel_launches": kcount,
            "bytes_per_particle_step": bytes_pp,
            # the whole step (every kernel and gap) against the same bytes
            "step_frac": bytes_pp * particles / (dt / a.steps) / 1e9 / HBM_PEAK_GBS,
        } | ({"kernel_time_note": ("multi-rank: a resample step's kernel is split; the timed launch is part 1 "
                                   "over every tile (slots taking received rows skipped), the part-2 re-runs "
                                   "of those tiles are not in kernel_avg_ms")} if world > 1 else {}),
    }


# ------------------------------------------------------------ secondaries
def secondary_c4(gen, ctx, a):
    """C4: the nonlinear (Kitagawa) SSM at 2^21 particles — one GPU's shard of
    the 16M-particle 8-GPU configuration (BASELINE.json configs[3])."""
    model = gen.KitagawaSSM(10.0, 1.0)  # examples/pmmh/run.jl:69 (var_x = 10, var_y = 1)
    n = 1 << 21
    r = pf_run(gen, ctx, None, 1, a, model, n, "k_step_pairs<KitModel,false>",
               lambda n_res: 16 * 1 + 16)
    set_traffic(r["roofline"], pmc_profile("pmc_k_step_kitagawa.json"))
    out = {
        "metric": "particle-steps/sec, nonlinear SSM (C4 shard)",
        "value": n * a.steps / r["dt"],
        "unit": "particle-steps/s",
        "ms_per_step": r["dt"] * 1e3 / a.steps,
        "steps": a.steps,
        "config": {"workload": "C4: Kitagawa SSM bootstrap PF, 2097152 particles (one GPU's shard of 16M), "
                               f"systematic resampling at ESS<N/2, record_history={not a.no_history}",
                   "resample_steps_timed": r["n_res"], "log_ml": r["lml"]},
        "roofline": r["roofline"],
    }
    if not a.no_cpu_baseline:
        out["cpu_baseline"] = pf_cpu_baseline(model, r["ys"], a.cpu_seconds)
    return out


def secondary_slots(gen, ctx, a):
    """Slot-described Unfold kernels (GH_FAMILY_SLOTS) at the C2
    size: a count SSM (2-d affine latent; Poisson, normal, Bernoulli and
    categorical addresses, every one observed each step), a switching linear
    dynamical system and a model with dependent addresses and a gamma library
    slot (both on the extended instantiations), and the C2 model written as
    slots, beside the hand-lowered family on the same data — the generic
    functor's price."""
    n = a.particles
    T = a.warmup + a.steps + 1

    def timed(model, obs, init_cm):
        st = gen.initialize_particle_filter(model, (1,), init_cm, n, seed=42,
                                            record_history=not a.no_history, history_capacity=T + 2, ctx=ctx)
        gen.run_particle_filter(st, list(obs[1 : 1 + a.warmup]), a.ess_threshold)
        batch = gen.prepare_observations(model, list(obs[1 + a.warmup : 1 + a.warmup + a.steps]))
        ctx.synchronize()
        t0 = time.perf_counter()
        gen.run_particle_filter(st, batch, a.ess_threshold)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        _, did = st.ess_history()
        n_res = int(did[a.warmup : a.warmup + a.steps].sum())
        st.close()
        return {"ms_per_step": dt * 1e3 / a.steps, "particle_steps_per_s": n * a.steps / dt, "resample_steps_timed": n_res}

    count = gen.SlotSSM(
        {"form": "affine", "A": [[0.9, 0.05], [0.0, 0.8]], "b": [0.0, 0.1], "Q": [[0.05, 0.01], [0.01, 0.04]],
         "mu0": [0.5, 0.0], "P0": [[0.3, 0.0], [0.0, 0.3]]},
        [{"name": "count", "dist": "poisson", "h": [1.0, 0.5], "c": 0.2},
         {"name": "z", "dist": "normal", "h": [0.3, -0.2], "c": 0.1, "sd": 0.7},
         {"name": "on", "dist": "bernoulli", "h": [1.5, 0.0], "c": -0.3},
         {"name": "kind", "dist": "categorical", "W": [[1.0, 0.0], [0.0, 1.0], [-1.0, 1.0]], "c": [0.0, 0.2, -0.1]}])
    _, cys = count.simulate(T, np.random.default_rng(5))
    # the extended instantiations: two latent addresses (a switching linear-Gaussian
    # state), and dependent addresses with a library (gamma) slot
    slds = gen.SlotSSM(
        {"form": "switching", "prior": [0.7, 0.3], "T": [[0.9, 0.2], [0.1, 0.8]],
         "A": [[[0.95, 0.1], [0.0, 0.9]], [[0.5, -0.3], [0.2, 0.6]]], "b": [[0.0, 0.1], [0.5, -0.2]],
         "Q": [[[0.05, 0.01], [0.01, 0.04]], [[0.2, 0.0], [0.0, 0.15]]], "mu0": [0.0, 0.0], "P0": [[0.5, 0.0], [0.0, 0.5]]},
        [{"name": "y", "dist": "normal", "h": [1.0, 0.5, 0.0, 1.5], "c": 0.0, "sd": 0.4},
         {"name": "n", "dist": "poisson", "h": [0.2, 0.0, 0.0, 1.0], "c": 0.3}])
    _, sys_ = slds.simulate(T, np.random.default_rng(6))
    deps = gen.SlotSSM(
        {"form": "affine", "A": [[0.9, 0.05], [0.0, 0.8]], "b": [0.0, 0.1], "Q": [[0.05, 0.01], [0.01, 0.04]],
         "mu0": [0.5, 0.0], "P0": [[0.3, 0.0], [0.0, 0.3]]},
        [{"name": "a", "dist": "normal", "h": [1.0, 0.0], "c": 0.0, "sd": 0.5},
         {"name": "n", "dist": "poisson", "h": [0.5, 0.2], "c": 0.1, "parents": {"a": 0.3}},
         {"name": "g", "dist": "gamma", "args": [{"link": "exp", "h": [0.2, 0.0], "c": 0.1}, 1.5],
          "parents": {"n": 0.05}}])
    _, dys = deps.simulate(T, np.random.default_rng(7))
    lg = gen.LinearGaussianSSM.benchmark(a.d)
    lgs = gen.SlotSSM({"form": "affine", "A": lg.A, "b": lg.b, "Q": lg.Q, "mu0": lg.mu0, "P0": lg.P0},
                      [{"name": "y", "dist": "mvnormal", "H": lg.H, "c": lg.c, "R": lg.R}])
    _, ys = lg.simulate(T, np.random.default_rng(2))
    fam = timed(lg, list(ys), {("chain", 1, "y"): ys[0]})
    sl = timed(lgs, [{"y": y} for y in ys], {("chain", 1, "y"): ys[0]})
    return {
        "metric": "particle-steps/sec, slot-described SSMs",
        "unit": "particle-steps/s",
        "particles": n,
        "steps": a.steps,
        "count_ssm": timed(count, [dict(y) for y in cys], {("chain", 1, k): v for k, v in cys[0].items()}),
        "switching_lds": timed(slds, [dict(y) for y in sys_], {("chain", 1, k): v for k, v in sys_[0].items()}),
        "dependent_library": timed(deps, [dict(y) for y in dys], {("chain", 1, k): v for k, v in dys[0].items()}),
        "lgssm_d%d_as_slots" % a.d: sl,
        "lgssm_d%d_family" % a.d: fam,
        "slots_vs_family": fam["ms_per_step"] / sl["ms_per_step"],
        "note": "the generic slot functor (parameters through pointers, a loop over slots) against the hand-lowered "
                "LG-SSM family on the same observations (bit-identical results, tests/test_slots.py)",
    }


def peer_probe(gen, ctx, world, dist):
    """A few always-resampling steps of a small filter on the peer transport
    (rows cross ranks every step); returns the log-ML as an exact hex string.
    The ranks line up after the set-up, so that the device-side waits of the
    first exchange do not absorb the processes' start-up skew."""
    m = gen.LinearGaussianSSM.benchmark(4)
    _, ys = m.simulate(5, np.random.default_rng(5))
    n = 2048 * world
    err = None
    try:
        st = gen.initialize_particle_filter(m, (1,), {("chain", 1, "y"): ys[0]}, n, seed=7, ctx=ctx)
        ctx.synchronize()
    except Exception as e:  # (still at the barrier: the ranks' collectives stay in step)
        err = e
    dist.barrier()
    if err is not None:
        raise err
    gen.run_particle_filter(st, list(ys[1:]), float(n))
    lml = float(gen.log_ml_estimate(st)).hex()
    st.close()
    return lml


def secondary_multirank_path(gen, a, c2_ms, c4_ms):
    """The multi-rank code path timed on this one GPU (gh_ctx_force_multirank:
    a one-rank RCCL communicator): per step the shards' and the records'
    ncclAllGather, k_rank_a2, k_rank_b and the split step, against the one-rank
    path's ms_per_step measured above (DESIGN.md §7 projects the 8-GPU step
    from the difference)."""
    from gen_amd.transport import LocalTransport

    out = {}
    for tname, mk in (("rccl", lambda: gen.Context(device=0, force_multirank=True)),
                      # (force_multirank: a world-1 peer context otherwise takes the one-rank path —
                      # rounds 4-5 timed that by mistake as the peer path)
                      ("peer", lambda: gen.Context(device=0, transport=LocalTransport(), peer=True,
                                                   force_multirank=True))):
        ctx = mk()
        try:
            for name, model, n, d, base in (("C2", gen.LinearGaussianSSM.benchmark(a.d), a.particles, a.d, c2_ms),
                                            ("C4", gen.KitagawaSSM(10.0, 1.0), 1 << 21, 1, c4_ms)):
                r = pf_run(gen, ctx, None, 1, a, model, n, "", lambda n_res, d=d: 16 * d + 16)
                ms = r["dt"] * 1e3 / a.steps
                out[f"{name}_{tname}" if tname != "rccl" else name] = {
                    "ms_per_step": ms, "one_rank_ms_per_step": base,
                    "extra_us_per_step": None if base is None else round((ms - base) * 1e3, 2),
                    "resample_steps_timed": r["n_res"], "log_ml": r["lml"]}
        finally:
            ctx.close()
    out["note"] = ("world = 1 on the multi-rank path: C2 / C4 over RCCL (the collectives are one-rank copies), "
                   "C2_peer / C4_peer over the peer transport (the maxima and records through the rank's own "
                   "mailbox inside the fused k_rank_ab, no collective launch); no rows move, so the extra time "
                   "is the path's launches, mailbox round trips and host plan, not xGMI")
    return out


def secondary_call_by_call(gen, ctx, a, c2_ms):
    """C2 through the reference's own caller loop instead of gh_pf_run: per
    step gh_pf_maybe_resample then gh_pf_step, each one C-ABI call from the
    host (ctypes here, a ccall in the Julia shim).  "with_decision" asks for
    the Bool that maybe_resample! returns (the host waits for k_resample1 to
    post it to a host-mapped mailbox, not for the stream); "no_decision"
    passes NULL."""
    model = gen.LinearGaussianSSM.benchmark(a.d)
    out = {}
    for name, loop in (("with_decision", "cbc"), ("no_decision", "cbc_async")):
        r = pf_run(gen, ctx, None, 1, a, model, a.particles, "", lambda n_res: 16 * a.d + 16, loop=loop)
        ms = r["dt"] * 1e3 / a.steps
        out[name] = {"ms_per_step": ms, "vs_gh_pf_run": None if not c2_ms else round(ms / c2_ms, 4),
                     "resample_steps_timed": r["n_res"], "log_ml": r["lml"]}
    out["gh_pf_run_ms_per_step"] = c2_ms
    return out


def secondary_c3(gen, ctx, a):
    """C3: coal change-point RJMCMC, 2^20 independent chains x 1000 mcmc_steps
    (BASELINE.json configs[2])."""
    from gen_amd.coal import CoalChains
    from oracle import oracle as O

    ev = np.array(json.load(open(os.path.join(ROOT, "tests", "golden", "coal_events.json")))["events"])
    chains, steps = 1 << 20, 1000
    ch = CoalChains(ev, chains, seed=42, ctx=ctx)
    ch.run(0, accepts=False)  # generate (the start from the prior), untimed
    ctx.synchronize()
    t0 = time.perf_counter()
    ch.run(steps, accepts=False)  # chains resident on the device: the timed call moves no state
    ctx.synchronize()
    dt = time.perf_counter() - t0
    ks = np.bincount(ch.k, minlength=10)[:10] / chains
    kms = ch.kernel_ms
    ch.close()
    pmc = pmc_profile("pmc_k_coal.json")
    out = {
        "metric": "coal RJMCMC chain-steps/s (C3)",
        "value": chains * steps / dt,
        "unit": "chain-steps/s",
        "config": {"workload": "C3: examples/coal RJMCMC (rate, position, birth/death moves), 190 events",
                   "chains": chains, "steps": steps},
        "kernel_ms": kms,
        "k_posterior": [round(float(x), 4) for x in ks],
        "roofline": {"bound": "valu", "kernel": "k_coal",
                     "hbm_bytes_per_launch": pmc.get("hbm_bytes_per_launch") if pmc else None,
                     "valu_frac": pmc.get("valu_frac") if pmc else None,
                     "source": pmc.get("source") if pmc else None,
                     "note": ("an 8-change-point window of each chain in LDS for the launch (four waves per "
                              "SIMD), the rest of a longer chain's row in place in HBM; VALU-bound "
                              "(valu_frac from the PMC profile in source); HBM is one pass over the windows")},
    }
    if not a.no_cpu_baseline:
        def make(threads):
            nc = 512 * max(1, threads)

            def sample():
                t = time.perf_counter()
                O.coal_run(ev, nc, 200, seed=42)
                return nc * 200, time.perf_counter() - t
            return sample
        out["cpu_baseline"] = cpu_pair(make, "chain-steps/s", "orc_coal_run, 512 chains per thread x 200 steps")
    return out


def secondary_c5(gen, ctx, a):
    """C5: PMMH, 2^16 outer chains x 256 inner particles, T = 100
    (BASELINE.json configs[4]; one GPU's share is replicas only)."""
    from gen_amd.pmmh import PMMHChains
    from oracle import oracle as O

    T, chains, inner, iters = 100, 1 << 16, 256, 2
    _, ys = gen.KitagawaSSM(4.0, 1.0, 0.0, 5.0).simulate(T, np.random.default_rng(3))
    ch = PMMHChains(ys, chains, inner, seed=42, ctx=ctx)
    ch.run(0)  # generate: the start from the prior, one filter per chain (untimed)
    t0 = time.perf_counter()
    ch.run(iters)
    dt = time.perf_counter() - t0
    units = chains * iters * 4 * T * inner
    pmc = pmc_profile("pmc_k_pmmh.json")
    out = {
        "metric": "PMMH inner particle-steps/s (C5)",
        "value": units / dt,
        "unit": "particle-steps/s",
        "config": {"workload": "C5: examples/pmmh PMMH (4 MH moves per iteration, each an inner PF of T=100)",
                   "chains": chains, "inner": inner, "T": T, "iterations": iters},
        "kernel_ms": ch.kernel_ms,
        "accept_rate": [round(float(x), 4) for x in ch.accepts.sum(axis=0) / (chains * iters)],
        "roofline": {"bound": "valu", "kernel": "k_pmmh",
                     "valu_frac": pmc.get("valu_frac") if pmc else None,
                     "hbm_bytes_per_launch": pmc.get("hbm_bytes_per_launch") if pmc else None,
                     "source": pmc.get("source") if pmc else None},
    }
    if not a.no_cpu_baseline:
        def make(threads):
            nc = 4 * max(1, threads)

            def sample():
                t = time.perf_counter()
                O.pmmh_run(ys, nc, inner, 1, seed=42)  # generate + 1 iteration = 5 filters per chain
                return nc * 5 * T * inner, time.perf_counter() - t
            return sample
        out["cpu_baseline"] = cpu_pair(make, "particle-steps/s", "orc_pmmh_run, 4 chains per thread x (generate + 1 iteration)")
    return out


# ------------------------------------------------------------------- main
_KEEP = []


def main(argv=None):
    a = parse(argv)
    if a.time_every is None:
        # every k-th step-kernel launch, at least 5 in the timed region (the
        # driver's 20 steps: every 4th); events on every launch cost 1.0 us
        # per step against every 10th (A/B at 20 steps, round 5)
        a.time_every = max(1, min(10, a.steps // 5))
    import gen_amd as gen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        ctx = None
        if a.transport == "gloo":
            import torch

            from gen_amd.transport import GlooTransport

            ctx = gen.Context(device=local % max(1, torch.cuda.device_count()), transport=GlooTransport())
        elif a.transport == "peer":
            import torch

            from gen_amd.transport import GlooTransport

            try:  # (ranks may share a GPU: the one-GPU rehearsal)
                ctx = gen.Context(device=local % max(1, torch.cuda.device_count()), transport=GlooTransport(),
                                  peer=True)
                ok = 1
            except Exception as e:  # (no IPC mapping between these GPUs)
                print(f"rank {rank}: peer transport unavailable ({e}); RCCL instead", file=sys.stderr, flush=True)
                ok = 0
            oks = [None] * world
            dist.all_gather_object(oks, ok)
            if all(oks):
                # a short filter over the mapped mailboxes (every wait on the
                # device is bounded, so a mapping that does not carry stores
                # between these GPUs errors out instead of hanging): the ranks
                # must finish and agree on the log-ML bit for bit
                probe = None
                try:
                    probe = peer_probe(gen, ctx, world, dist)
                except Exception as e:
                    print(f"rank {rank}: peer transport probe failed ({e}); RCCL instead", file=sys.stderr, flush=True)
                probes = [None] * world
                dist.all_gather_object(probes, probe)
                oks = [p is not None and p == probes[0] for p in probes]
            if not all(oks):
                # (a rank whose peer context exists keeps it open: its destroy
                # would wait for the ranks that have none)
                _KEEP.append(ctx)
                ctx = None
                a.transport = "rccl"
        if ctx is None:
            uid = [gen.Context.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            ctx = gen.Context(device=local, rank=rank, world=world, unique_id=uid[0])
    elif a.force_multirank and a.transport == "peer":
        # the peer transport's multi-rank kernels at world 1 (the rank's own mailbox)
        from gen_amd.transport import LocalTransport

        ctx = gen.Context(device=0, transport=LocalTransport(), peer=True, force_multirank=True)
    else:
        ctx = gen.Context(device=0, force_multirank=a.force_multirank)
    gen.set_default_context(ctx)

    if a.model == "lgssm":
        model = gen.LinearGaussianSSM.benchmark(a.d)
        d = a.d
        kname = f"k_step<LGOptModel<{a.d}>,false>" if a.proposal == "optimal" else f"k_step<LGModel<{a.d},3>,false>"
    else:
        model = gen.KitagawaSSM(10.0, 1.0)  # examples/pmmh/run.jl:69 (var_x = 10, var_y = 1)
        d = 1
        # (the pair kernel on every rank whose first particle is a multiple of 128)
        kname = "k_step_pairs<KitModel,false>" if a.particles % 128 == 0 else "k_step<KitModel,false>"
    r = pf_run(gen, ctx, dist, world, a, model, a.particles, kname,
               lambda n_res: 16 * d + 16)
    # PMC HBM bytes per step-kernel launch of the profiled configs (tools/pmc_json.py)
    pmc = None
    if a.model == "lgssm" and a.d == 10 and a.particles == 1 << 20 and r["prop"] is None:
        pmc = pmc_profile("pmc_k_step.json")
    elif a.model == "kitagawa" and a.particles == 1 << 21:
        pmc = pmc_profile("pmc_k_step_kitagawa.json")
    set_traffic(r["roofline"], pmc)

    ys, n_global, lml = r["ys"], r["n_global"], r["lml"]
    log_ml_error = None
    if a.model == "lgssm":
        exact = model.kalman_log_marginal(ys[: 1 + a.warmup + a.steps])
        log_ml_error = {"reference": "Kalman filter (exact)", "exact": exact,
                        "abs": abs(lml - exact), "rel": abs(lml - exact) / abs(exact)}
    out = {
        "metric": ("particle-steps/sec (whole node) + log-ML error vs CPU ref, 1M-particle SSM" if a.model == "lgssm"
                   else "particle-steps/sec (whole node), nonlinear SSM (C4)"),
        "value": n_global * a.steps / r["dt"],
        "unit": "particle-steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": r["dt"] * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic (observations simulated from the model, numpy seed {2 if a.model == 'lgssm' else 3})",
        "config": {
            "workload": (f"C2: {a.d}-dim linear-Gaussian SSM " + ("optimal-proposal PF" if r["prop"] else "bootstrap PF")
                         if a.model == "lgssm" else
                         "C4: Kitagawa nonlinear SSM bootstrap PF") + f", {a.particles} particles/GPU, "
                        f"systematic resampling at ESS<N/2, record_history={not a.no_history}",
            "particles_global": n_global,
            "d": d,
            "resampler": a.resampler,
            "parallelism": f"particle-dp{world}",
            "transport": a.transport if world > 1 else (f"{a.transport} (forced multi-rank)" if a.force_multirank else "none"),
            "resample_steps_timed": r["n_res"],
            "log_ml": lml,
        },
        # log-ML error against the exact answer of the CPU reference's target
        # (Kalman filter over the same observations; C2 only).  The estimate's
        # Monte-Carlo error at this N dominates it; parity with the CPU
        # restatement of Gen's filter at equal seeds is 1e-9 (tests/).
        "log_ml_error": log_ml_error,
        "roofline": r["roofline"],
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = pf_cpu_baseline(model, ys, a.cpu_seconds)
        # the headline configuration itself (N = the bench's particles, every
        # step of the run, same seed and observations): GPU vs the CPU restatement
        # at least the C2 configuration's T = 100 (BASELINE.json configs[1])
        ys_par = ys if len(ys) >= 100 else model.simulate(100, np.random.default_rng(2))[1]
        par = cpu_parity(model, ys_par, a.particles, a.resampler, a.proposal)
        out["cpu_baseline"]["parity"] = par
        if out["log_ml_error"] is not None:
            out["log_ml_error"]["vs_cpu_reference_same_seed"] = {"particles": par["particles"], "rel": par["rel"]}
    if rank == 0 and world == 1 and not a.no_secondary and a.model == "lgssm":
        c4 = secondary_c4(gen, ctx, a)
        out["secondary"] = {"C4": c4, "C3": secondary_c3(gen, ctx, a), "C5": secondary_c5(gen, ctx, a),
                            "slots": secondary_slots(gen, ctx, a)}
        if a.proposal == "default":
            out["secondary"]["call_by_call"] = secondary_call_by_call(gen, ctx, a, out["ms_per_step"])
        if a.proposal == "default":  # (world 1: both transports, whatever --transport says)
            out["secondary"]["multirank_path"] = secondary_multirank_path(gen, a, out["ms_per_step"],
                                                                          c4["ms_per_step"])
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
