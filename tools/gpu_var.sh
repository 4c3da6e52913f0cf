#!/bin/bash
# Interleaved A/B of timing-only variants on one box (C2): tools/gpu_var.sh v1 v2 ...
set -e
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python tools/variants.py run "$@" >> gpurun_out/var/c2.log 2>&1
done
