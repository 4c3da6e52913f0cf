"""Build libgen_hip.so (gfx950) in-tree with hipcc.

The library is plain C-ABI (include/gen_hip.h); no torch headers are involved.
-ffp-contract=off is part of the numeric specification: the
kernels spell every fused multiply-add as fma() and must not get extra ones.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgen_hip.so")
SOURCES = [os.path.join(CSRC, "gh_api.hip")]
HEADERS = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "gen_hip.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GH_OFFLOAD_ARCH", "gfx950")


def hipcc_cmd(out: str = LIB, extra: list[str] | None = None) -> list[str]:
    return [
        HIPCC,
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-ffp-contract=off",
        "-fno-fast-math",
        # keep constant materialisation next to its uses inside the persistent
        # loops (hoisted fp64 polynomial constants otherwise spill)
        "-mllvm",
        "-disable-machine-licm",
        "-fPIC",
        "-shared",
        "-Wall",
        "-Wno-unused-function",
        "-Wno-unused-value",
        "-I" + os.path.join(ROOT, "include"),
        *(extra or []),
        *SOURCES,
        "-o",
        out,
        "-L/opt/rocm/lib",
        "-lrccl",
        "-Wl,-rpath,/opt/rocm/lib",
    ]


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(s) <= t for s in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return LIB
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    tmp = LIB + ".tmp"
    cmd = hipcc_cmd(out=tmp)
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


def build_variant(name: str, defines: list[str]) -> str:
    """Timing-only variant (e.g. -DGH_PHILOX_ROUNDS=7) at gen_amd/variants/<name>.so;
    never the product, never used by the parity tests."""
    out_dir = os.path.join(HERE, "variants")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"{name}.so")
    subprocess.run(hipcc_cmd(out=out, extra=[f"-D{d}" for d in defines]), check=True)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":
        build_variant(sys.argv[2], sys.argv[3:])
    else:
        build(force="--force" in sys.argv)
