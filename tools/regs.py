"""Print per-kernel register/occupancy usage of libgen_hip's device code.

python tools/regs.py [substring-filter ...]   (GH_REGS_SRC=gh_inst_lg2.hip: another unit)
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       f"-I{ROOT}/include", "--cuda-device-only", "-c", f"{ROOT}/gen_amd/csrc/" + __import__("os").environ.get("GH_REGS_SRC", "gh_api.hip"), "-o", "/tmp/_regs.o",
       "-Rpass-analysis=kernel-resource-usage", "-mllvm", "-disable-machine-licm"] + [x for a in sys.argv[1:] if a.startswith("-mllvm=") for x in ("-mllvm", a[7:])] + [a for a in sys.argv[1:] if a.startswith("-D")]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
filt = [a for a in sys.argv[1:] if not a.startswith(("-D", "-mllvm="))]
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if filt and not any(f in r["name"] for f in filt):
        continue
    print(f"{r['name'][:70]:70s} vgpr={r.get('VGPRs')} sgpr={r.get('TotalSGPRs')} occ={r.get('Occupancy [waves/SIMD]')} "
          f"vspill={r.get('VGPRs Spill')} scratch={r.get('ScratchSize [bytes/lane]')}")
