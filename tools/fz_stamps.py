"""Per-phase clocks of the fused resample + step launch (gh_fused.h; variant
build with GH_RS_STAMPS).  Blocks [0, G) are the resample role, the next
ones step blocks (start, wait done, end).

python tools/fz_stamps.py [lg10|kit] [log2 N] [lib.so]   (on the GPU box)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GEN_HIP_LIB", sys.argv[3] if len(sys.argv) > 3 else
                      os.path.join(ROOT, "gen_amd", "variants", "fz_stamps.so"))
import gen_amd as gen  # noqa: E402
from gen_amd import _lib  # noqa: E402

ctx = gen.Context(device=0)
gen.set_default_context(ctx)
name = sys.argv[1] if len(sys.argv) > 1 else "lg10"
n = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 20)
m = gen.LinearGaussianSSM.benchmark(10) if name == "lg10" else gen.KitagawaSSM(10.0, 1.0)
_, ys = m.simulate(12, np.random.default_rng(2))
st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, n, seed=42, record_history=False)
gen.run_particle_filter(st, list(ys[1:10]))
ctx.synchronize()
lib = _lib.load()
buf = (ctypes.c_uint64 * (1024 * 8))()
lib.gh_debug_rs_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lib.check(lib.gh_debug_rs_stamps(buf, 1024 * 8))
G = -(-n // 4096)
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.int64)
t0 = a[:G, 0].min()
rel = (a - t0) * 0.01  # wall_clock64 ticks at 100 MHz -> us
print(f"{name} n={n} G={G}")
names = {0: "start", 7: "max", 1: "decided", 2: "quantised", 3: "barrier", 4: "offsets", 5: "marks", 6: "signalled"}
for k, nm in names.items():
    r = rel[:G, k]
    print(f"rs  {nm:10s} min {r.min():7.2f} med {np.median(r):7.2f} max {r.max():7.2f} us")
sb = rel[G:1024]
for k, nm in {0: "start", 2: "wait done", 6: "end"}.items():
    r = sb[:, k]
    print(f"stp {nm:10s} min {r.min():7.2f} med {np.median(r):7.2f} max {r.max():7.2f} us   (blocks G..1023)")
