# round-4 GPU check: new multi-rank paths first, then the whole GPU suite and the bench
mkdir -p gpurun_out/r4a
timeout -k 10 600 python -u -m pytest tests/test_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4a/mr.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/gputest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r4a/bench.log 2>&1
