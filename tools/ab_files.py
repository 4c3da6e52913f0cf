"""Summarise gpurun_out/ab/{new,prev}_*.json (tools/gpu_abfile.sh)."""
import glob
import json

for tag in ("new", "prev"):
    rows = []
    for f in sorted(glob.glob(f"gpurun_out/ab/{tag}_*.json")):
        d = json.load(open(f))
        rows.append((f.rsplit("/", 1)[1], d["ms_per_step"] * 1e3, d["roofline"]["kernel_avg_ms"] * 1e3, d["value"]))
    for r in rows:
        print(f"{tag:5s} {r[0]:16s} step {r[1]:6.2f} us  k_step {r[2]:6.2f} us  {r[3]:.3e}")
