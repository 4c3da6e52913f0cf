mkdir -p gpurun_out/r4a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/gputest.log 2>&1 && timeout -k 10 300 python bench.py > gpurun_out/r4a/bench.log 2>&1
