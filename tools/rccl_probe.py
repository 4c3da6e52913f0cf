import os, sys, subprocess
sys.path.insert(0, os.getcwd())
from tests.test_multirank import _run_workers, ROOT
import numpy as np
out = "gpurun_out/rccl/g"
os.makedirs("gpurun_out/rccl", exist_ok=True)
try:
    outs = _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", "lg4", "--n", "20011", "--T", "8",
                         "--thr", "1e9", "--seed", "9", "--transport", "rccl", "--device", "0", "--out", out], 2, timeout=100)
    print("OK")
    from oracle import oracle as O
    from tests.mr_worker import build_model
    m = build_model("lg4")
    _, ys = m.simulate(8, np.random.default_rng(5))
    ref = O.run_pf(m, ys, 20011, 9, thr=1e9)
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(2)]
    states = np.concatenate([p["states"] for p in parts], axis=0)
    print("states equal:", np.array_equal(states.T, ref.state()))
    print("parents equal:", np.array_equal(np.concatenate([p["parents"] for p in parts]), ref.parents()))
    print("lml", float(parts[0]["lml"]), ref.log_ml_estimate())
except Exception as e:
    print("FAILED", type(e).__name__, str(e)[-3000:])
