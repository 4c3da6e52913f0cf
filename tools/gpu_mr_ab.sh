#!/bin/bash
# The multi-rank path over the peer transport forced onto the one GPU of a box:
# its GPU tests, the fused resample (k_rank_ab) against the two-kernel path
# (GH_NO_FUSED_RANK) at C2 and C4, and kernel traces of both configurations.
#   gpurun -- 'bash tools/gpu_mr_ab.sh gpurun_out/<dir>'
set -e
O=${1:-gpurun_out/mr_ab}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multirank.py -m gpu -k peer -x -v --timeout 300 --timeout-method thread > "$O/gputest.log" 2>&1
for v in "c2|" "c4|--model kitagawa --particles 2097152"; do
  name=${v%%|*}; args=${v#*|}
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 --force-multirank --transport peer $args > "$O/$name.fused.json" 2> "$O/$name.fused.err"
  GH_NO_FUSED_RANK=1 timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 --force-multirank --transport peer $args > "$O/$name.split.json" 2> "$O/$name.split.err"
done
for v in "c4mr_peer|--model kitagawa --particles 2097152 --force-multirank --transport peer" "c2mr_peer|--force-multirank --transport peer"; do
  name=${v%%|*}; args=${v#*|}
  GH_PROF_STEPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- python3 tools/profile_run.py $args > "$O/$name.log" 2>&1
done
