set -e
O=gpurun_out/te
mkdir -p $O
bash tools/gpu_bench_rep.sh $O/ab 3 "--no-secondary --steps 100" "--no-secondary --steps 100 --time-every 10" "--no-secondary --steps 100 --time-every 1" "--no-secondary --steps 100 --no-kernel-timing" > $O/ab.log 2>&1
