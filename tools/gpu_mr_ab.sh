# multi-rank GPU tests, then a same-box A/B of the forced multi-rank path: the tree's library against
# gen_amd/variants/prev.so (an earlier build), C2 and C4, 3 reps
set -e
O=gpurun_out/mr_ab2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multirank.py -m gpu -q --timeout 300 --timeout-method thread > $O/mr_tests.log 2>&1
bash tools/gpu_bench_rep.sh $O/ab 3 "--no-secondary --force-multirank" "gen_amd/variants/prev.so|--no-secondary --force-multirank" "--no-secondary --force-multirank --model kitagawa --particles 2097152" "gen_amd/variants/prev.so|--no-secondary --force-multirank --model kitagawa --particles 2097152" > $O/ab.log 2>&1
