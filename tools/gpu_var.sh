#!/bin/bash
set -e
mkdir -p gpurun_out/var
export TMPDIR=/tmp
timeout -k 10 600 python tools/variants.py run base occ8 occ6 > gpurun_out/var/variants.txt 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline --no-kernel-timing > gpurun_out/var/bench_notime.json 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/var/bench_time.json 2>&1
