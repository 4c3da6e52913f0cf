#!/bin/bash
# base vs prev, C2, four alternations
set -e
mkdir -p gpurun_out/ab4
export TMPDIR=/tmp
for i in 1 2 3 4; do
  timeout -k 10 300 python tools/variants.py run base prev >> gpurun_out/ab4/c2.log 2>&1
done
