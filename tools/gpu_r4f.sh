# whole GPU suite, bench line, forced multi-rank traces
set -e
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
export TMPDIR=/tmp
for v in "c2mr|--force-multirank" "c4mr|--model kitagawa --particles 2097152 --force-multirank"; do
  name=${v%%|*}; args=${v#*|}
  GH_PROF_STEPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python3 tools/profile_run.py $args > $O/$name.log 2>&1
done
