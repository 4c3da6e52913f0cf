# round-4 GPU check: new tests first, then the whole GPU suite, the bench, bound-path A/B, C3 window variants
mkdir -p gpurun_out/r4a
timeout -k 10 600 python -u -m pytest tests/test_coal.py tests/test_unfold_kats_device.py tests/test_step_params.py tests/test_lg_linear_proposal.py tests/test_lg_optimal.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4a/mr.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/gputest.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r4a/bench.log 2>&1 && \
bash tools/gpu_bench_rep.sh gpurun_out/r4a/ab 3 "--no-secondary" "--no-secondary --exact-quantisation" "--no-secondary --model kitagawa --particles 2097152" "--no-secondary --model kitagawa --particles 2097152 --exact-quantisation" > gpurun_out/r4a/ab.log 2>&1 && \
for v in base coal_w10 coal_w7; do
  lib=gen_amd/libgen_hip.so; [ $v != base ] && lib=gen_amd/variants/$v.so
  GEN_HIP_LIB=$lib timeout -k 10 120 python tools/bench_coal.py --steps 300 > gpurun_out/r4a/coal_$v.json 2>&1 || exit 1
done
