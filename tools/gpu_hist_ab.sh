# does the step kernel slow down with the history footprint or with the run length? (one box, 2 reps)
set -e
O=gpurun_out/hist
mkdir -p $O
bash tools/gpu_bench_rep.sh $O/ab 2 "--no-secondary --steps 100" "--no-secondary --steps 100 --no-history" "--no-secondary --steps 20 --warmup 5" "--no-secondary --steps 400" > $O/ab.log 2>&1
