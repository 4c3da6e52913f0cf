"""Turn rocprofv3 output directories into the committed profile files.

  python tools/pmc_json.py c2 gpurun_out/prof3 profiles/round3
  python tools/pmc_json.py c345 gpurun_out/prof3_345 profiles/round3

c2 (tools/gpu_profile.sh): <prefix>_kernel_stats.csv, <prefix>_pmc.txt,
profiles/pmc_k_step.json.  c345 (tools/gpu_profile_c345.sh):
<prefix>_c{4,3,5}_kernel_stats.csv / _pmc.txt and profiles/pmc_k_step_kitagawa.json,
pmc_k_coal.json, pmc_k_pmmh.json — read by bench.py as roofline.traffic and
the secondaries' valu_frac.

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
come from separate --pmc passes, are reported in KiB, and FETCH_SIZE counts
half the bytes of a streaming read on gfx950 (doubled here).
valu_frac = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the
fraction of the kernel's SIMD-cycles with a VALU instruction in flight
(SQ_* count quad-cycles summed over the chip; GRBM_GUI_ACTIVE is summed over
the 8 XCDs) — the gfx94x VALUBusy formula, which ROCm 7.2 falls back to on
gfx950.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def counters(src_glob):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(src_glob)):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def mean(v):
    return sum(v) / len(v)


def write_pmc_txt(agg, path):
    lines = []
    for k, d in agg.items():
        lines.append(k)
        for c, v in sorted(d.items()):
            lines.append(f"   {c:32s} {mean(v):18.1f}  (launches={len(v)})")
    open(path, "w").write("\n".join(lines) + "\n")


def kernel_avg_ns(stats_csv, match):
    for r in csv.DictReader(open(stats_csv)):
        if match(r["Name"]):
            return float(r["AverageNs"]), int(r["Calls"])
    return None, 0


def summary(agg, match, stats_csv, source, config):
    hits = [(k, d) for k, d in agg.items() if match(k)]
    if not hits:
        return None
    k, d = max(hits, key=lambda kd: len(kd[1].get("SQ_WAVES", [])))
    out = {"kernel": k.split("(")[0]}
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        f, w = mean(d["FETCH_SIZE"]), mean(d["WRITE_SIZE"])
        out.update(fetch_bytes_per_launch=2 * f * 1024, write_bytes_per_launch=w * 1024,
                   hbm_bytes_per_launch=2 * f * 1024 + w * 1024)
    if "SQ_ACTIVE_INST_VALU" in d and "GRBM_GUI_ACTIVE" in d:
        out["valu_frac"] = mean(d["SQ_ACTIVE_INST_VALU"]) * 4 / (1024 * mean(d["GRBM_GUI_ACTIVE"]) / 8)
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
        out["valu_insts_per_wave"] = mean(d["SQ_INSTS_VALU"]) / mean(d["SQ_WAVES"])
    avg, calls = kernel_avg_ns(stats_csv, match)
    if avg is not None:
        out["avg_duration_ns"] = avg
        out["launches_traced"] = calls
    out["source"] = source
    out["method"] = ("HBM: FETCH_SIZE x 1024 x 2 (gfx950 half-count) + WRITE_SIZE x 1024, separate --pmc passes; "
                     "valu_frac: SQ_ACTIVE_INST_VALU x 4 / (1024 x GRBM_GUI_ACTIVE / 8)")
    out["config"] = config
    return out


def main():
    mode, src, prefix = sys.argv[1], sys.argv[2], sys.argv[3]
    os.makedirs(os.path.dirname(prefix), exist_ok=True)
    jobs = []
    if mode == "c2":
        jobs.append(("", os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(src, "pmc*", "run_counter_collection.csv"),
                     lambda k: "k_step<" in k and ", false>" in k, "profiles/pmc_k_step.json",
                     "bench.py default workload (C2, d=10, 2^20 particles, systematic, resample every step)"))
    else:
        jobs.append(("_c4", os.path.join(src, "c4.trace", "run_kernel_stats.csv"),
                     os.path.join(src, "c4.pmc*", "run_counter_collection.csv"),
                     lambda k: ("k_step_pairs<" in k or "k_step<" in k) and "KitModel, false" in k,
                     "profiles/pmc_k_step_kitagawa.json",
                     "bench.py --model kitagawa --particles 2097152 (C4 per GPU, systematic, resample every step)"))
        jobs.append(("_c3", os.path.join(src, "c3.trace", "run_kernel_stats.csv"),
                     os.path.join(src, "c3.pmc*", "run_counter_collection.csv"), lambda k: k.startswith("gh::k_coal("),
                     "profiles/pmc_k_coal.json", "tools/bench_coal.py (C3: 2^20 chains x 1000 RJ-MCMC iterations)"))
        jobs.append(("_c5", os.path.join(src, "c5.trace", "run_kernel_stats.csv"),
                     os.path.join(src, "c5.pmc*", "run_counter_collection.csv"), lambda k: k.startswith("gh::k_pmmh("),
                     "profiles/pmc_k_pmmh.json", "tools/bench_pmmh.py (C5: 2^16 chains x 256 inner particles)"))
    for tag, stats, pmc_glob, match, out_json, config in jobs:
        if not os.path.exists(stats):  # (a partial profile run: that configuration only)
            continue
        shutil.copy(stats, f"{prefix}{tag}_kernel_stats.csv")
        agg = counters(pmc_glob)
        write_pmc_txt(agg, f"{prefix}{tag}_pmc.txt")
        s = summary(agg, match, stats, f"{prefix}{tag}_pmc.txt", config)
        if s is not None:
            json.dump(s, open(out_json, "w"), indent=1)
            print(out_json, json.dumps(s, indent=1))


if __name__ == "__main__":
    main()
