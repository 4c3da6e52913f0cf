#!/bin/bash
# One GPU session at a round's end: parity tests, the default bench line (with
# the CPU baseline), C4/C5/C3 measurements, then the rocprofv3 passes
# (kernel trace + stats, then one PMC counter group per run).
set -e
OUT=${1:-gpurun_out/round}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python bench.py --model kitagawa --particles 2097152 --no-cpu-baseline > $OUT/bench_kitagawa.json 2> $OUT/bench_kitagawa.err
timeout -k 10 300 python tools/bench_pmmh.py > $OUT/bench_pmmh.json 2> $OUT/bench_pmmh.err
timeout -k 10 300 python tools/bench_coal.py > $OUT/bench_coal.json 2> $OUT/bench_coal.err
bash tools/gpu_profile.sh $OUT/prof
