#!/bin/bash
# Round-5 GPU pass F: the resample's phase clocks with the marks' stores
# skipped and with the exact slot-count fallback skipped (timing-only probes,
# tools/rs_probe.patch), beside the plain clocks, C2 and C4, twice each.
set -e
OUT=$PWD/gpurun_out/r5f
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in rs_stamps rs_nomarks rs_noexact; do
    GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $OUT/${v}_lg10_$rep.txt 2>&1
    GEN_HIP_LIB=$PWD/gen_amd/variants/$v.so timeout -k 10 120 python tools/rs_stamps.py kit 21 > $OUT/${v}_kit_$rep.txt 2>&1
  done
done
for f in $OUT/*_1.txt $OUT/*_2.txt; do echo "== $f"; grep -E "^(end|marks|offsets) |offsets->marks|barrier->offsets" $f; done
