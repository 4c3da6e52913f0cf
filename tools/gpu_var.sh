#!/bin/bash
set -e
mkdir -p gpurun_out/var
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/var/pytest_gpu.log 2>&1
timeout -k 10 600 python tools/variants.py run base philox1 > gpurun_out/var/variants.txt 2>&1
