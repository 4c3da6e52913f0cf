"""Timing-only ablation variants of libgen_hip.so (never the product).

build:  python tools/variants.py build
run:    python tools/variants.py run   (on the GPU box; one process per variant)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = {
    "base": [],
    "occ8": ["GH_LG10_WAVES=8"],
    "occ6": ["GH_LG10_WAVES=6"],
    "philox1": ["GH_PHILOX_ROUNDS=1"],
    "philox7": ["GH_PHILOX_ROUNDS=7"],
    "coal_w10": ["GH_COAL_WIN=10"],
    "coal_w7": ["GH_COAL_WIN=7"],
    "coal_w6": ["GH_COAL_WIN=6"],
    "coal_w5": ["GH_COAL_WIN=5"],
    "coal_w4": ["GH_COAL_WIN=4"],
    "coal_b64": ["GH_COAL_BLOCK=64"],
    "coal_b256w7": ["GH_COAL_BLOCK=256", "GH_COAL_WIN=7"],
    "coal_b256w6": ["GH_COAL_BLOCK=256", "GH_COAL_WIN=6"],
    "coal_b256w8": ["GH_COAL_BLOCK=256", "GH_COAL_WIN=8"],
    "coal_b512w6": ["GH_COAL_BLOCK=512", "GH_COAL_WIN=6"],
    "coal_b512w7": ["GH_COAL_BLOCK=512", "GH_COAL_WIN=7"],
    "coal_b64w10": ["GH_COAL_BLOCK=64", "GH_COAL_WIN=10"],
    "nospec": ["GH_SPEC_STREAK=0xffffffffu"],
    "fmaplain": ["GH_FMA_C_PLAIN"],
    "div20plain": ["GH_DIV20_PLAIN"],
    "mathplain": ["GH_FMA_C_PLAIN", "GH_DIV20_PLAIN"],
    "prev": [],  # A/B: a library built from an earlier commit and copied in by hand
}
# instrumented builds (not timed by `run`)
EXTRA = {"rs_stamps": ["GH_RS_STAMPS"], "kstep_stamps": []}
# variants whose hooks are not in the product sources: a patch applied to a copy
PATCHES = {"rs_stamps": os.path.join(ROOT, "tools", "rs_stamps.patch"),
           "kstep_stamps": os.path.join(ROOT, "tools", "kstep_stamps.patch"),
}
BENCH_ARGS = os.environ.get("GH_VARIANT_ARGS", "--steps 50").split()
# GH_VARIANT_SCRIPT=tools/bench_pmmh.py times another workload with the same variants
BENCH_SCRIPT = os.environ.get("GH_VARIANT_SCRIPT", "bench.py")


def main():
    if sys.argv[1] == "build":
        from gen_amd import build as gb

        for name, defs in {**VARIANTS, **EXTRA}.items():
            if len(sys.argv) > 2 and name not in sys.argv[2:]:
                continue
            gb.build_variant(name, defs, PATCHES.get(name))
            print("built", name, flush=True)
    else:
        out = {}
        for name in [v for v in VARIANTS if len(sys.argv) < 3 or v in sys.argv[2:]]:
            lib = os.path.join(ROOT, "gen_amd", "variants", f"{name}.so")
            env = dict(os.environ, GEN_HIP_LIB=lib)
            r = subprocess.run([sys.executable, os.path.join(ROOT, BENCH_SCRIPT)] +
                               (["--no-cpu-baseline"] if BENCH_SCRIPT == "bench.py" else []) + BENCH_ARGS,
                               env=env, capture_output=True, text=True, timeout=300)
            try:
                d = json.loads(r.stdout.strip().splitlines()[-1])
                out[name] = ({"ms_per_step": d["ms_per_step"], "k_step_ms": d["roofline"]["kernel_avg_ms"],
                              "value": d["value"]} if "roofline" in d else {"value": d["value"]})
            except Exception:
                out[name] = {"error": r.stderr[-500:]}
            print(name, out[name], flush=True)
        json.dump(out, open(os.path.join(ROOT, "gpurun_out", "variants.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
