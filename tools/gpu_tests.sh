#!/bin/bash
# the GPU test suite only
set -e
mkdir -p gpurun_out/tests
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests/pytest_gpu.log 2>&1
