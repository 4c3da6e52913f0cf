#!/bin/bash
set -e
mkdir -p gpurun_out/rs
export TMPDIR=/tmp
timeout -k 10 120 python tools/rs_stamps.py > gpurun_out/rs/stamps.txt 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/rs/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/rs/bench.json 2> gpurun_out/rs/bench.err
GH_PROF_STEPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/rs/trace -o run --output-format csv -- python3 tools/profile_run.py > gpurun_out/rs/trace.log 2>&1
