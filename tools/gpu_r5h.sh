#!/bin/bash
# Round-5 GPU pass H: resample phase clocks, product vs the exact slot count
# out of line (rs_noinl: a smaller marks loop), C2 and C4, twice each.
set -e
OUT=$PWD/gpurun_out/r5h
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in rs_stamps rs_noinl; do
    GH_STAMPS_SAVE=$OUT/${v}_lg10_$rep.npy GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $OUT/${v}_lg10_$rep.txt 2>&1
    GH_STAMPS_SAVE=$OUT/${v}_kit_$rep.npy GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python tools/rs_stamps.py kit 21 > $OUT/${v}_kit_$rep.txt 2>&1
  done
done
for f in $OUT/*.txt; do echo "== $f"; grep -E "^(quantised|barrier|offsets|marks|end) " $f; done
