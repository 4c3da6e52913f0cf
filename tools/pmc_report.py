"""Summarise rocprofv3 PMC csv passes: mean counter value per kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
filt = sys.argv[2:] or ["k_step"]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if any(x in k for x in filt):
        print(k[:80])
        for c, v in sorted(d.items()):
            print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
