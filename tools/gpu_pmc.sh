#!/bin/bash
# PMC passes (one counter group per run) for the bench config; kernel-trace only.
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
export GH_PROF_STEPS=${GH_PROF_STEPS:-10}
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctrs -d "$OUT/p$i" -o run --output-format csv -- python3 tools/profile_run.py > "$OUT/p$i.log" 2>&1
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_SMEM
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
FETCH_SIZE
WRITE_SIZE
LIST
