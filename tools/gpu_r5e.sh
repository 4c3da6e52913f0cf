#!/bin/bash
# Round-5 GPU pass E: the GPU suite on 32-bit range marks, then an interleaved
# A/B against the previous commit's library (gen_amd/variants/prev.so, 64-bit
# marks) at C2 and C4, and the resample's phase clocks.
set -e
OUT=$PWD/gpurun_out/r5e
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -3 $OUT/pytest.log
for rep in 1 2 3 4; do
  for m in "c2|" "c4|--model kitagawa --particles 2097152"; do
    name=${m%%|*}; args=${m#*|}
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 $args > $OUT/${name}_head_$rep.json 2>$OUT/${name}_head_$rep.err
    GEN_HIP_LIB=$PWD/gen_amd/variants/prev.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 $args > $OUT/${name}_prev_$rep.json 2>$OUT/${name}_prev_$rep.err
    GEN_HIP_LIB=$PWD/gen_amd/variants/ld16.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 5 $args > $OUT/${name}_ld16_$rep.json 2>$OUT/${name}_ld16_$rep.err
  done
done
GEN_HIP_LIB=$PWD/gen_amd/variants/rs_stamps.so timeout -k 10 120 python tools/rs_stamps.py lg10 20 > $OUT/rs_stamps_lg10.txt 2>&1
GEN_HIP_LIB=$PWD/gen_amd/variants/rs_stamps.so timeout -k 10 120 python tools/rs_stamps.py kit 21 > $OUT/rs_stamps_kit.txt 2>&1
python - $OUT <<'PY'
import json, sys, statistics as st
out = sys.argv[1]
for name in ("c2", "c4"):
    for v in ("head", "prev", "ld16"):
        us, ks = [], []
        for r in range(1, 5):
            s = open(f"{out}/{name}_{v}_{r}.json").read()
            j = json.loads(s[s.index('{"metric"'):])
            us.append(j["ms_per_step"] * 1e3)
            ks.append(j["roofline"]["kernel_avg_ms"] * 1e3)
        print(name, v, " ".join(f"{u:.2f}" for u in us), f"median {st.median(us):.2f}", f"kernel {st.median(ks):.2f}")
PY
tail -n 9 $OUT/rs_stamps_lg10.txt $OUT/rs_stamps_kit.txt
