# multi-rank GPU tests, the 2-rank torchrun rehearsal of bench.py, the bench line (forced multi-rank secondary)
set -e
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multirank.py -m gpu -q --timeout 300 --timeout-method thread > $O/mr_tests.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --transport gloo --particles 262144 > $O/tr2.json 2> $O/tr2.err
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
bash tools/gpu_bench_rep.sh $O/ab 3 "--no-secondary --model kitagawa --particles 2097152" "gen_amd/variants/pairshards.so|--no-secondary --model kitagawa --particles 2097152" > $O/ab.log 2>&1
