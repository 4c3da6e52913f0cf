#!/bin/bash
# rocprofv3 kernel-trace A/B of timing-only variants (C2 bench config):
# tools/gpu_var_prof.sh v1 v2 ...  -> per-kernel averages per variant and round
set -e
OUT=gpurun_out/varprof
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in "$@"; do
    GEN_HIP_LIB=gen_amd/variants/$v.so GH_PROF_STEPS=40 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$v.$i -o run --output-format csv -- python3 tools/profile_run.py > $OUT/$v.$i.log 2>&1
  done
done
