"""C5 measurement: PMMH with 2^16 chains x 256 inner particles, T = 100.

python tools/bench_pmmh.py [--chains N] [--inner P] [--iters K]
Prints one JSON line: inner particle-steps/s (4 filters per iteration, each
T x P particle-steps, per chain), the kernel's event time, and the oracle's
CPU rate on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--chains", type=int, default=1 << 16)
    p.add_argument("--inner", type=int, default=256)
    p.add_argument("--iters", type=int, default=2)
    p.add_argument("--T", type=int, default=100)
    p.add_argument("--cpu-chains", type=int, default=2)
    a = p.parse_args()
    import gen_amd as gen
    from gen_amd.pmmh import PMMHChains
    from oracle import oracle as O

    ctx = gen.Context(device=0)
    _, ys = gen.KitagawaSSM(4.0, 1.0, 0.0, 5.0).simulate(a.T, np.random.default_rng(3))
    warm = PMMHChains(ys, 256, a.inner, seed=1, ctx=ctx)
    warm.run(1)
    ch = PMMHChains(ys, a.chains, a.inner, seed=42, ctx=ctx)
    t0 = time.perf_counter()
    ch.run(a.iters)
    dt = time.perf_counter() - t0
    # the first call also runs the initial generate (one extra filter per chain)
    filters = a.iters * 4 + 1
    units = a.chains * filters * a.T * a.inner
    t1 = time.perf_counter()
    O.pmmh_run(ys, a.cpu_chains, a.inner, 1, seed=42)
    cpu_dt = time.perf_counter() - t1
    cpu_units = a.cpu_chains * 5 * a.T * a.inner
    print(json.dumps({
        "metric": "PMMH inner particle-steps/s (C5)",
        "value": units / dt,
        "kernel_value": units / (ch.kernel_ms * 1e-3),
        "unit": "particle-steps/s",
        "config": {"chains": a.chains, "inner": a.inner, "T": a.T, "iterations": a.iters, "filters_per_chain": filters},
        "kernel_ms": ch.kernel_ms,
        "wall_s": dt,
        "accept_rate": (ch.accepts.sum(axis=0) / (a.chains * a.iters)).tolist(),
        "cpu_baseline": {"value": cpu_units / cpu_dt, "unit": "particle-steps/s", "cores": 1, "kind": "port",
                         "sample": f"oracle orc_pmmh_run, {a.cpu_chains} chains x 1 iteration + generate"},
    }), flush=True)


if __name__ == "__main__":
    main()
