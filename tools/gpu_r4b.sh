# round-4 GPU pass: whole GPU suite, smoke, default bench line, C2 rocprofv3 stats + PMC
set -e
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
bash tools/gpu_profile.sh $O/prof
