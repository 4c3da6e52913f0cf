"""Multi-rank particle-filter worker (launched by tests/test_multirank.py).

One process per rank (torch.distributed.run).  Every rank holds a shard of
one filter; the ranks talk through the host-staged gloo transport (several
ranks may share one GPU) or RCCL (one GPU per rank).  Each rank saves its
shard of the final states, log-weights, parents and the log-ML estimate.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build_model(name):
    import gen_amd as gen

    if name == "lg4":
        return gen.LinearGaussianSSM.benchmark(4)
    if name == "lg10":
        return gen.LinearGaussianSSM.benchmark(10)
    if name == "kit":
        return gen.KitagawaSSM(10.0, 1.0)
    if name == "kit_sharp":  # peaked weights: one particle (one rank) holds nearly all of them
        return gen.KitagawaSSM(10.0, 0.01)
    if name == "count":  # the slot-described family: Poisson, normal, Bernoulli, categorical addresses
        from tests.test_slots import count_model

        return count_model()
    if name == "switch":  # a slot model with a categorical (one-hot) latent
        from tests.test_slots import switching_model

        return switching_model()
    if name == "slds":  # two latent addresses (regime, state): the extended slot instantiations
        from tests.test_slots import slds_model

        return slds_model()
    if name == "deps":  # dependent observed addresses incl. a library (gamma) slot
        from tests.test_slots import dep_model

        return dep_model()
    raise ValueError(name)


def obs_at(m, y, t):
    """The step-t constraints: a slot model's dict of observed slots, or the
    family's one observed address."""
    if isinstance(y, dict):
        return {("chain", t, k): v for k, v in y.items()}
    return {m.obs_address(t): y}


def changed_model(name):
    """The Unfold of `name` with other parameters (a parameter change, --params-step)."""
    import gen_amd as gen

    if name == "count":
        from tests.test_slots import changed_count_model

        return changed_count_model()
    if name.startswith("lg"):
        m = build_model(name)
        return gen.LinearGaussianSSM(0.8 * m.A, 1.5 * m.Q, m.H, 0.7 * m.R, m.mu0 + 0.1, m.P0, b=m.b + 0.05, c=m.c - 0.1)
    return gen.KitagawaSSM(6.0, 2.0)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="lg4")
    p.add_argument("--n", type=int, default=3001)
    p.add_argument("--T", type=int, default=8)
    p.add_argument("--thr", type=float, default=None, help="ESS threshold (default: N/2)")
    p.add_argument("--seed", type=int, default=9)
    p.add_argument("--transport", default="gloo", help="gloo (host-staged), peer (device mailboxes, IPC handles "
                   "swapped over gloo), rccl, or rccl1: one rank forced onto the multi-rank path over a one-rank "
                   "RCCL communicator (gh_ctx_force_multirank)")
    p.add_argument("--batched", action="store_true", help="steps 2..T through run_particle_filter (gh_pf_run: "
                   "max-only steps, the resample's sums in k_rank_a2)")
    p.add_argument("--rejuv", type=int, default=0, help="rejuvenation moves after init and every step")
    p.add_argument("--device", type=int, default=None, help="GPU of every rank (default: LOCAL_RANK)")
    p.add_argument("--params-step", type=int, default=0, help="step whose particle_filter_step changes the Unfold's "
                   "parameters (new_args = (t, model'): every particle re-scored along its genealogy)")
    p.add_argument("--mid-query", action="store_true", help="genealogy queries between maybe_resample and the step "
                   "at t = 4 (the step then reads materialised ancestors naming received rows)")
    p.add_argument("--genealogy", action="store_true", help="also save trajectories at t = 1, 5, T, the score "
                   "columns and 500 sample_unweighted_traces indices (collective queries)")
    p.add_argument("--resampler", default="systematic", help="systematic or multinomial")
    p.add_argument("--csmc", action="store_true", help="conditional SMC (multinomial): particle 0 pinned to the "
                   "reference trajectory 0.9 x (the simulated latents)")
    p.add_argument("--sleep", default=None, help="rank:step:seconds — that rank sleeps before that call-by-call step "
                   "(a slow peer: the others' device waits must wait for it, not fail)")
    p.add_argument("--peer-timeout", type=float, default=None, help="gh_ctx_set_peer_timeout (seconds)")
    p.add_argument("--corrupt", type=int, default=None, help="after the run, rank 0 overwrites particle 0's "
                   "ancestor record of step T with this value (gh_debug_set_ancestor); every rank then runs the "
                   "collective get_traces queries and saves the errors they raise")
    p.add_argument("--out", required=True)
    a = p.parse_args()

    import torch.distributed as dist

    import gen_amd as gen
    from gen_amd.transport import GlooTransport

    import datetime

    # (bounded: a collective that one rank never joins fails the test instead of hanging it)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
    rank, world = dist.get_rank(), dist.get_world_size()
    if a.transport in ("gloo", "peer"):
        tr = GlooTransport()
        ctx = gen.Context(device=0, transport=tr, peer=a.transport == "peer")
    elif a.transport == "rccl1":
        assert world == 1
        ctx = gen.Context(device=a.device or 0, force_multirank=True)
    else:
        uid = [gen.Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        dev = a.device if a.device is not None else int(os.environ.get("LOCAL_RANK", "0"))
        ctx = gen.Context(device=dev, rank=rank, world=world, unique_id=uid[0])
    if a.peer_timeout is not None:
        ctx.set_peer_timeout(a.peer_timeout)
    gen.set_default_context(ctx)
    sleep_rank, sleep_step, sleep_s = (int(v) if i < 2 else float(v) for i, v in
                                       enumerate(a.sleep.split(":"))) if a.sleep else (-1, -1, 0.0)
    m = build_model(a.model)
    xs, ys = m.simulate(a.T, np.random.default_rng(5))
    ref = np.asarray(xs, dtype=np.float64).reshape(len(ys), -1) * 0.9
    if a.csmc:
        st = gen.initialize_conditional_particle_filter(m, (1,), obs_at(m, ys[0], 1), a.n, ref[0], seed=a.seed)
    else:
        st = gen.initialize_particle_filter(m, (1,), obs_at(m, ys[0], 1), a.n, seed=a.seed, resampler=a.resampler)
    if a.rejuv:
        gen.rejuvenate(st, a.rejuv)
    did = []
    if a.batched:
        gen.run_particle_filter(st, list(ys[1 : a.T]), a.thr)
    m2 = changed_model(a.model) if a.params_step else None
    for t in range(2, a.T + 1) if not a.batched else ():
        if rank == sleep_rank and t == sleep_step:
            import time

            time.sleep(sleep_s)
        did.append(gen.maybe_resample(st, a.thr))
        if a.mid_query and t == 4:
            st.states(2)
            gen.get_traces(st).scores()
        if a.csmc:
            gen.conditional_particle_filter_step(st, (t,), (gen.UnknownChange(),), obs_at(m, ys[t - 1], t), ref[t - 1])
        elif t == a.params_step:
            gen.particle_filter_step(st, (t, m2), (gen.UnknownChange(), gen.UnknownChange()), obs_at(m, ys[t - 1], t))
        else:
            gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), obs_at(m, ys[t - 1], t))
        if a.rejuv:
            gen.rejuvenate(st, a.rejuv)
    lml = gen.log_ml_estimate(st)
    if a.corrupt is not None:
        from gen_amd import _lib

        if rank == 0:
            _lib.check(_lib.load().gh_debug_set_ancestor(st.h, a.T, 0, a.corrupt))
        errs = {}
        for name, q in (("traj", lambda: st.states(1)), ("scores", lambda: gen.get_traces(st).scores())):
            try:
                q()
                errs[name] = ""
            except Exception as e:  # (the query must fail, not return a wrong trajectory)
                errs[name] = f"{type(e).__name__}: {e}"
        np.savez(f"{a.out}.rank{rank}.npz", **{f"err_{k}": np.array(v) for k, v in errs.items()})
        dist.barrier()
        dist.destroy_process_group()
        return
    extra = {}
    if a.genealogy:
        for t in sorted({1, min(5, a.T), a.T}):
            extra[f"traj{t}"] = st.states(t)
        tot, ps = gen.get_traces(st).scores(per_step=True)
        extra["score_tot"], extra["score_ps"] = tot, ps
        _, extra["samp"] = gen.sample_unweighted_traces(st, 500, seed=3)
    np.savez(
        f"{a.out}.rank{rank}.npz",
        states=st.states(),
        logw=gen.get_log_weights(st),
        parents=st.parents,
        lml=lml,
        did=np.array(did, dtype=np.int64),
        lo=st.first,
        **extra,
    )
    st.close()
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
