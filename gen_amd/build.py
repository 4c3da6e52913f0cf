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
SOURCES = [os.path.join(CSRC, "gh_api.hip")] + sorted(glob.glob(os.path.join(CSRC, "gh_inst_*.hip")))
HEADERS = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "gen_hip.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GH_OFFLOAD_ARCH", "gfx950")
JOBS = int(os.environ.get("GH_BUILD_JOBS", str(min(16, os.cpu_count() or 4))))

FLAGS = [
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
    "-Wall",
    "-Wno-unused-function",
    "-Wno-unused-value",
    "-I" + os.path.join(ROOT, "include"),
]


def compile_cmd(src: str, obj: str, extra: list[str] | None = None) -> list[str]:
    return [HIPCC, *FLAGS, *(extra or []), "-c", src, "-o", obj]


def _sources(csrc: str) -> list[str]:
    return [os.path.join(csrc, "gh_api.hip")] + sorted(glob.glob(os.path.join(csrc, "gh_inst_*.hip")))


def link_cmd(objs: list[str], out: str) -> list[str]:
    return [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", *objs, "-o", out, "-L/opt/rocm/lib", "-lrccl",
            "-Wl,-rpath,/opt/rocm/lib"]


def hipcc_cmd(out: str = LIB, extra: list[str] | None = None) -> list[str]:
    """One-shot command (all sources in one hipcc call); kept for tools that
    print or reuse the flags."""
    return [HIPCC, *FLAGS, "-shared", *(extra or []), *SOURCES, "-o", out, "-L/opt/rocm/lib", "-lrccl",
            "-Wl,-rpath,/opt/rocm/lib"]


def _compile_all(out: str, obj_dir: str, extra: list[str] | None, verbose: bool, sources: list[str] | None = None) -> None:
    """Every translation unit to an object in parallel, then one link."""
    os.makedirs(obj_dir, exist_ok=True)
    sources = sources or SOURCES
    objs = [os.path.join(obj_dir, os.path.basename(s).replace(".hip", ".o")) for s in sources]
    cmds = [compile_cmd(s, o, extra) for s, o in zip(sources, objs)]
    if verbose:
        print(" ".join(cmds[0]), f"(+{len(cmds) - 1} units, {JOBS} jobs)", flush=True)
    from concurrent.futures import ThreadPoolExecutor

    def run(cmd):
        return subprocess.run(cmd, capture_output=True, text=True)

    # the biggest unit (gh_api.hip) first
    with ThreadPoolExecutor(max_workers=JOBS) as ex:
        results = list(ex.map(run, cmds))
    failed = [(c, r) for c, r in zip(cmds, results) if r.returncode != 0]
    for c, r in failed:
        sys.stderr.write(r.stdout + r.stderr)
    if failed:
        raise subprocess.CalledProcessError(failed[0][1].returncode, failed[0][0])
    subprocess.run(link_cmd(objs, out), check=True)


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
    _compile_all(tmp, os.path.join(HERE, "build_obj"), None, verbose)
    os.replace(tmp, LIB)
    return LIB


def build_variant(name: str, defines: list[str], patch: str | None = None) -> str:
    """Timing-only variant (e.g. -DGH_PHILOX_ROUNDS=7) at gen_amd/variants/<name>.so;
    never the product, never used by the parity tests.  `patch`: a unified
    diff against gen_amd/csrc (e.g. tools/rs_stamps.patch, the resample's
    phase clocks), applied to a copy of the sources for this build only."""
    out_dir = os.path.join(HERE, "variants")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"{name}.so")
    sources = None
    if patch:
        src = os.path.join(out_dir, f"src_{name}")
        shutil.rmtree(src, ignore_errors=True)
        shutil.copytree(CSRC, os.path.join(src, "gen_amd", "csrc"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(src, "include"))
        with open(patch) as f:
            subprocess.run(["patch", "-s", "-p1", "-d", os.path.join(src, "gen_amd", "csrc")], stdin=f, check=True)
        sources = _sources(os.path.join(src, "gen_amd", "csrc"))
    _compile_all(out, os.path.join(out_dir, f"obj_{name}"), [f"-D{d}" for d in defines], True, sources)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":
        build_variant(sys.argv[2], sys.argv[3:])
    else:
        build(force="--force" in sys.argv)
