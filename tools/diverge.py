"""Debug tool: GPU filter vs the oracle on the bench's C2 observations at a
given N, step by step; prints the first step whose parents / log-ML differ."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import gen_amd as gen  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
T = int(sys.argv[2]) if len(sys.argv) > 2 else 40
gen.set_default_context(gen.Context(device=0))
m = gen.LinearGaussianSSM.benchmark(10)
_, ys = m.simulate(111, np.random.default_rng(2))
st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, n, seed=42)
orc = O.OraclePF(m, n, 42)
orc.init(ys[0])
for t in range(2, T + 1):
    did = gen.maybe_resample(st)
    odid, oess = orc.maybe_resample()
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    par_ok = np.array_equal(st.parents, orc.parents())
    print(t, did, odid, a, b, par_ok, flush=True)
    if did != odid or not par_ok or abs(a - b) > 1e-9 * abs(b):
        p, q = st.parents, orc.parents()
        bad = np.nonzero(p != q)[0]
        print("first mismatch slots", bad[:10], p[bad[:10]], q[bad[:10]], "count", bad.size)
        break
    gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {m.obs_address(t): ys[t - 1]})
    orc.step(ys[t - 1])
