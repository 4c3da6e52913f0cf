"""Per-block clocks of the step kernel (variant build with tools/kstep_stamps.patch):
when each 256-particle block starts and retires, where it ran, and what the
launch's occupancy over time was — the launch's ramp and tail.

python tools/kstep_stamps.py [log2 N]   (on the GPU box, after
`python tools/variants.py build kstep_stamps`)
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GEN_HIP_LIB", os.path.join(ROOT, "gen_amd", "variants", "kstep_stamps.so"))
import gen_amd as gen  # noqa: E402
from gen_amd import _lib  # noqa: E402

ctx = gen.Context(device=0)
gen.set_default_context(ctx)
name = "lg10"
n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 20)
m = gen.LinearGaussianSSM.benchmark(10) if name == "lg10" else gen.KitagawaSSM(10.0, 1.0)
_, ys = m.simulate(30, np.random.default_rng(2))
st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, n, seed=42, history_capacity=32)
gen.run_particle_filter(st, list(ys[1:26]))
ctx.synchronize()
nb = (n + 255) // 256 if name == "lg10" else (n + 511) // 512
lib = _lib.load()
buf = (ctypes.c_uint64 * (nb * 4))()
lib.gh_debug_ks_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lib.check(lib.gh_debug_ks_stamps(buf, nb))
a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 4).astype(np.int64)
t0 = a[:, 0].min()
s = (a[:, 0] - t0) * 0.01  # 100 MHz -> us
e = (a[:, 1] - t0) * 0.01
life = e - s
span = e.max()
grid = np.arange(0.0, span + 0.25, 0.25)
active = np.array([np.count_nonzero((s <= g) & (e > g)) for g in grid])
peak = active.max()
lost = float(np.sum(peak - active) * 0.25 / peak)
order = np.argsort(s)
out = {
    "model": name, "n": n, "blocks": nb, "span_us": round(float(span), 2),
    "peak_active_blocks": int(peak), "lost_block_us_over_peak": round(lost, 2),
    "last_block_start_us": round(float(s.max()), 2),
    "lifetime_us": {q: round(float(np.percentile(life, p)), 2) for q, p in (("p10", 10), ("p50", 50), ("p90", 90))},
    "lifetime_first_wave_us": round(float(np.median(life[order[: peak]])), 2),
    "lifetime_last_wave_us": round(float(np.median(life[order[-peak:]])), 2),
    "active_over_time": [int(x) for x in active[:: 4]],  # every 1 us
    "per_xcc_blocks": np.bincount(a[:, 3] & 0xF, minlength=8).tolist(),
}
print(json.dumps(out))
