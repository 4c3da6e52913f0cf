#!/bin/bash
# GPU tests, then the C4 (Kitagawa) bench A/B over k_step_multi's virtual
# blocks per workgroup (GH_STEP_TPW = 1 is the one-block k_step), the C2
# bench line and a kernel-trace profile.
set -e
OUT=gpurun_out/tpw
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
for r in 1 2; do
  for t in 1 2 4 8; do
    GH_STEP_TPW=$t timeout -k 10 120 python bench.py --model kitagawa --particles 2097152 --no-cpu-baseline > $OUT/c4_tpw$t.r$r.json 2> $OUT/c4_tpw$t.r$r.err
  done
done
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
GH_PROF_STEPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/profile_run.py > $OUT/trace.log 2>&1
timeout -k 10 200 python tools/rccl_probe.py > $OUT/rccl.log 2>&1
