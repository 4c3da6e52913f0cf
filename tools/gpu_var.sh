#!/bin/bash
# Timing variants (tools/variants.py run) after the GPU parity tests, then the
# resample phase clocks.  Variants: pass names as arguments.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 900 python tools/variants.py run "$@" > gpurun_out/variants.log 2>&1
timeout -k 10 900 python tools/variants.py run "$@" >> gpurun_out/variants.log 2>&1
if [ -f gen_amd/variants/rs_stamps.so ]; then timeout -k 10 120 python tools/rs_stamps.py > gpurun_out/rs_stamps.txt 2>&1; fi
