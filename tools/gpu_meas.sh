#!/bin/bash
# Measurement pass: the C2 bench with the per-launch kernel events (fence-free
# timing events) at several densities against no events, at the default size
# and at the driver's --steps 20 --warmup 5.
set -e
OUT=gpurun_out/meas2
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --time-every 10 > $OUT/c2_ev10.r$r.json 2> $OUT/c2_ev10.r$r.err
  timeout -k 10 120 python bench.py --no-cpu-baseline > $OUT/c2_def.r$r.json 2> $OUT/c2_def.r$r.err
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-kernel-timing > $OUT/c2_noev.r$r.json 2> $OUT/c2_noev.r$r.err
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/c2_s20.r$r.json 2> $OUT/c2_s20.r$r.err
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --no-kernel-timing > $OUT/c2_s20noev.r$r.json 2> $OUT/c2_s20noev.r$r.err
done
