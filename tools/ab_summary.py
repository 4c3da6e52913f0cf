"""Mean ms/step and k_step ms of variants in a tools/variants.py run log."""
import ast
import sys
from collections import defaultdict

import numpy as np

for path in sys.argv[1:]:
    acc = defaultdict(list)
    for line in open(path):
        name, rest = line.split(" ", 1)
        d = ast.literal_eval(rest)
        if "ms_per_step" in d:
            acc[name].append((d["ms_per_step"] * 1e3, d["k_step_ms"] * 1e3))
    for name, v in acc.items():
        v = np.array(v)
        print(f"{path}: {name:8s} n={len(v)} ms/step {v[:, 0].mean():6.2f} (min {v[:, 0].min():6.2f})  "
              f"k_step {v[:, 1].mean():6.2f}")
