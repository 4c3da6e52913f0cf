#!/bin/bash
# LG-SSM, Kitagawa and PMMH timings of the built variants (GPU box).
mkdir -p gpurun_out/var3
export TMPDIR=/tmp
V="$*"
timeout -k 10 300 python tools/variants.py run $V > gpurun_out/var3/lg.txt 2>&1 || exit 1
GH_VARIANT_ARGS="--steps 50 --model kitagawa --particles 2097152" timeout -k 10 300 python tools/variants.py run $V > gpurun_out/var3/kit.txt 2>&1 || exit 1
GH_VARIANT_SCRIPT=tools/bench_pmmh.py GH_VARIANT_ARGS="--cpu-chains 1" timeout -k 10 400 python tools/variants.py run $V > gpurun_out/var3/pmmh.txt 2>&1 || exit 1
