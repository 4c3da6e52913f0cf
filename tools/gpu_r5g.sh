#!/bin/bash
# Round-5 GPU pass G: raw per-block resample clocks (C2, C4; product and
# no-stores probe) saved for offline analysis, plus the hardware placement
# of each block (XCC / SE / CU ids from the hardware registers).
set -e
OUT=$PWD/gpurun_out/r5g
mkdir -p $OUT
export TMPDIR=/tmp
for v in rs_stamps rs_nomarks; do
  GH_STAMPS_SAVE=$OUT/${v}_lg10.npy GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $OUT/${v}_lg10.txt 2>&1
  GH_STAMPS_SAVE=$OUT/${v}_kit.npy GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python tools/rs_stamps.py kit 21 > $OUT/${v}_kit.txt 2>&1
done
