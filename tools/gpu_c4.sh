#!/bin/bash
set -e
mkdir -p gpurun_out/c4
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --model kitagawa --particles 2097152 --no-cpu-baseline > gpurun_out/c4/bench_c4.json 2> gpurun_out/c4/bench_c4.err
timeout -k 10 300 python bench.py --no-cpu-baseline --no-history > gpurun_out/c4/bench_c2_nohist.json 2> gpurun_out/c4/bench_c2_nohist.err
