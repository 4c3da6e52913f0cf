#!/bin/bash
# Round-5 GPU pass I: resample phase clocks with per-wave marks-phase clocks
# (C2, C4), saved for offline analysis.
set -e
OUT=$PWD/gpurun_out/r5i
mkdir -p $OUT
export TMPDIR=/tmp
GH_STAMPS_SAVE=$OUT/lg10.npy GEN_HIP_LIB=$PWD/gen_amd/variants/rs_stamps.so timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $OUT/lg10.txt 2>&1
GH_STAMPS_SAVE=$OUT/kit.npy GEN_HIP_LIB=$PWD/gen_amd/variants/rs_stamps.so timeout -k 10 120 python tools/rs_stamps.py kit 21 > $OUT/kit.txt 2>&1
