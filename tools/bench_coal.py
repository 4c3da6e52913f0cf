"""C3 measurement: 2^20 coal RJMCMC chains x K steps (one thread per chain).

python tools/bench_coal.py [--chains N] [--steps K]
Prints one JSON line: chain-steps/s (one mcmc_step = rate, position, birth/death
move), the kernel's event time, and the oracle's CPU rate on a bounded sample.
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
    p.add_argument("--chains", type=int, default=1 << 20)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--cpu-chains", type=int, default=64)
    a = p.parse_args()
    import gen_amd as gen
    from gen_amd.coal import CoalChains
    from oracle import oracle as O

    ev = np.array(json.load(open(os.path.join(ROOT, "tests", "golden", "coal_events.json")))["events"])
    ctx = gen.Context(device=0)
    w = CoalChains(ev, 4096, seed=1, ctx=ctx)
    w.run(5)
    ch = CoalChains(ev, a.chains, seed=42, ctx=ctx)
    ch.run(0)  # generate (the start from the prior), untimed
    t0 = time.perf_counter()
    ch.run(a.steps)  # chains resident in HBM: the timed call moves no state (12 MB of counts back)
    dt = time.perf_counter() - t0

    units = a.chains * a.steps
    t1 = time.perf_counter()
    O.coal_run(ev, a.cpu_chains, 200, seed=42)
    cpu = a.cpu_chains * 200 / (time.perf_counter() - t1)
    ks = np.bincount(ch.k, minlength=10)[:10] / a.chains
    print(json.dumps({
        "metric": "coal RJMCMC chain-steps/s (C3)",
        "value": units / dt,
        "kernel_value": units / (ch.kernel_ms * 1e-3),
        "unit": "chain-steps/s",
        "config": {"chains": a.chains, "steps": a.steps, "events": int(ev.size)},
        "kernel_ms": ch.kernel_ms,
        "wall_s": dt,
        "accept_rate": (ch.accepts.sum(axis=0) / units).tolist(),
        "k_distribution": ks.tolist(),
        "cpu_baseline": {"value": cpu, "unit": "chain-steps/s", "cores": 1, "kind": "port",
                         "sample": f"oracle orc_coal_run, {a.cpu_chains} chains x 200 steps"},
    }), flush=True)


if __name__ == "__main__":
    main()
