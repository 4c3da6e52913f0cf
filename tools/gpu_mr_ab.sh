# forced multi-rank A/B on one box: the previous build (prev.so) against the tree's library, C2 and C4, 3 reps
set -e
O=gpurun_out/mr_ab
mkdir -p $O
bash tools/gpu_bench_rep.sh $O/ab 3 "--no-secondary --force-multirank" "gen_amd/variants/prev.so|--no-secondary --force-multirank" "--no-secondary --force-multirank --model kitagawa --particles 2097152" "gen_amd/variants/prev.so|--no-secondary --force-multirank --model kitagawa --particles 2097152" "--no-secondary" > $O/ab.log 2>&1
