#!/bin/bash
# End-of-round GPU pass (run on the GPU box from the repo root):
#   whole -m gpu suite, smoke(), the default bench line, rocprofv3 stats + PMC
#   for C2 (tools/gpu_profile.sh) and C4/C3/C5 (tools/gpu_profile_c345.sh),
#   kernel traces of the multi-rank path forced onto the one GPU (C2, C4).
# Then, here: python tools/pmc_json.py c2 OUT/prof profiles/roundN
#             python tools/pmc_json.py c345 OUT/prof345 profiles/roundN
set -e
O=${1:-gpurun_out/round}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gputest.log" 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
bash tools/gpu_profile.sh "$O/prof"
bash tools/gpu_profile_c345.sh "$O/prof345"
for v in "c2mr|--force-multirank --transport rccl" "c4mr|--model kitagawa --particles 2097152 --force-multirank --transport rccl" \
         "c2mr_peer|--force-multirank --transport peer" "c4mr_peer|--model kitagawa --particles 2097152 --force-multirank --transport peer"; do
  name=${v%%|*}; args=${v#*|}
  GH_PROF_STEPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- python3 tools/profile_run.py $args > "$O/$name.log" 2>&1
done
