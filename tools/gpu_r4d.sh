# coal window 8 / 256-thread blocks: coal GPU tests, C3 bench, C3 PMC (VALU busy, HBM)
set -e
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_coal.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/coal_tests.log 2>&1
timeout -k 10 120 python tools/bench_coal.py --cpu-chains 1 > $O/coal.json 2> $O/coal.err
export TMPDIR=/tmp
C3="tools/bench_coal.py --cpu-chains 1"
i=0
GH_PROF_STEPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c3.trace -o run --output-format csv -- python3 $C3 > $O/c3.trace.log 2>&1
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctrs -d $O/c3.pmc$i -o run --output-format csv -- python3 $C3 > $O/c3.pmc$i.log 2>&1
done
