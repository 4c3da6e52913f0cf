#!/bin/bash
# four interleaved rocprofv3 rounds of timing-only variants (C2 bench config)
set -e
OUT=gpurun_out/varprof4
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3 4; do
  for v in "$@"; do
    GEN_HIP_LIB=gen_amd/variants/$v.so GH_PROF_STEPS=60 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$v.$i -o run --output-format csv -- python3 tools/profile_run.py > $OUT/$v.$i.log 2>&1
  done
done
