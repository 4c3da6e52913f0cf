#!/bin/bash
# Phase and block clocks of the step and resample kernels (instrumented
# variant libraries built from tools/*_stamps.patch), C2 and C4 sizes; plus
# the GPU tests named in $1 (if any) against the product library.
set -e
O=gpurun_out/stamps
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest $1 -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  tail -2 $O/pytest.log
fi
timeout -k 10 120 python tools/kstep_stamps.py lg10 20 > $O/kstep_lg10.json 2> $O/kstep_lg10.err
timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $O/rs_lg10.txt 2>&1
timeout -k 10 120 python tools/rs_stamps.py kit 21 > $O/rs_kit.txt 2>&1
cat $O/kstep_lg10.json $O/rs_lg10.txt $O/rs_kit.txt
