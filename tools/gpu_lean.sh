#!/bin/bash
# C4 (2^21 particles) with and without the lean two-blocks-per-CU resample:
# rocprofv3 kernel stats and bench lines, alternating
set -e
OUT=gpurun_out/lean
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for v in base no_lean; do
    GEN_HIP_LIB=gen_amd/variants/$v.so GH_PROF_STEPS=40 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$v.$i -o run --output-format csv -- python3 tools/profile_run.py --model kitagawa --particles 2097152 > $OUT/$v.$i.log 2>&1
    GEN_HIP_LIB=gen_amd/variants/$v.so timeout -k 10 120 python bench.py --model kitagawa --particles 2097152 --no-cpu-baseline > $OUT/$v.$i.json 2> $OUT/$v.$i.err
  done
done
