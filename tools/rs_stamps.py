"""Per-phase clocks of k_resample1 (variant build with GH_RS_STAMPS).

python tools/rs_stamps.py [lg10|kit] [log2 N]   (on the GPU box, after
`python tools/variants.py build rs_stamps`)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GEN_HIP_LIB", os.path.join(ROOT, "gen_amd", "variants", "rs_stamps.so"))
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
buf = (ctypes.c_uint64 * (1024 * 16))()
lib.gh_debug_rs_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lib.check(lib.gh_debug_rs_stamps(buf, 1024 * 16))
grid = -(-n // (1024 * 4))  # IT = 4 (two blocks per CU at 2^21)
allraw = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.int64)
if grid < 1024 and allraw[grid, 0] != 0:  # the decider block (no tile) ran too
    grid += 1
print(f"{name} n={n} grid={grid}")
raw = allraw[:grid]
a = raw[:, :8]
waves = None
if hasattr(lib, "gh_debug_rs_waves"):  # (the probe variants have no per-wave clocks)
    wbuf = (ctypes.c_uint64 * (1024 * 16 * 4))()
    lib.gh_debug_rs_waves.argtypes = [ctypes.c_void_p, ctypes.c_int]
    _lib.check(lib.gh_debug_rs_waves(wbuf, 1024 * 16 * 4))
    waves = np.frombuffer(wbuf, dtype=np.uint64).reshape(1024, 16, 4)[:grid].astype(np.int64)
if os.environ.get("GH_STAMPS_SAVE"):  # raw per-block clocks (and per-wave marks clocks) for offline analysis
    np.save(os.environ["GH_STAMPS_SAVE"], raw)
    if waves is not None:
        np.save(os.environ["GH_STAMPS_SAVE"].replace(".npy", "_waves.npy"), waves)
t0 = a[:, 0].min()
rel = (a - t0) * 0.01  # wall_clock64 ticks at 100 MHz -> us
names = {0: "start", 7: "max", 1: "decided", 2: "quantised", 3: "barrier", 4: "offsets", 5: "marks", 6: "end"}
for k, nm in names.items():
    print(f"{nm:10s} min {rel[:, k].min():7.2f} med {np.median(rel[:, k]):7.2f} max {rel[:, k].max():7.2f} us")
# the slowest blocks of the late phases, and each phase's own duration
for k in (4, 5, 6):
    top = np.argsort(rel[:, k])[::-1][:4]
    print(f"{names[k]:10s} latest blocks " + ", ".join(f"{b} ({rel[b, k]:.2f})" for b in top))
order = [0, 7, 1, 2, 3, 4, 5, 6]
for a_, b_ in zip(order, order[1:]):
    d = rel[:, b_] - rel[:, a_]
    print(f"{names[a_]:>9s}->{names[b_]:10s} med {np.median(d):6.2f} max {d.max():6.2f} (block {int(d.argmax())}) us")
if waves is not None:  # the marks phase per wave: the latest blocks against the median block
    wd = (waves[:, :, 1] - waves[:, :, 0]) * 0.01
    car = waves[:, :, 3]
    near = waves[:, :, 2] >> 32
    waves[:, :, 2] &= 0xFFFFFFFF
    print("marks per wave index (median over blocks): " + " ".join(f"{x:.2f}" for x in np.median(wd, axis=0)) + " us")
    print(f"exact slot counts: {int(near.sum())} in {int((near > 0).sum())} waves; marks of those waves median "
          f"{np.median(wd[near > 0]) if (near > 0).any() else 0:.2f} us, of the others {np.median(wd[near == 0]):.2f} us")
    print(f"marks per wave: median {np.median(wd):.2f} us, carries median {np.median(car):.0f}, "
          f"blocks with a wave-wide carry loop {int((waves[:, :, 2].sum(axis=1) > 0).sum())} of {grid}")
    for b in np.argsort(rel[:, 5])[::-1][:4]:
        print(f"  block {b}: marks waves {' '.join(f'{x:.1f}' for x in wd[b])} us; "
              f"wave-wide loops {' '.join(str(int(x)) for x in waves[b, :, 2])}; carries {' '.join(str(int(x)) for x in car[b])}; "
              f"exact counts {' '.join(str(int(x)) for x in near[b])}")
