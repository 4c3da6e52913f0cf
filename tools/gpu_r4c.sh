# round-4 profiles: C2 (stats + PMC), C4/C3/C5 (stats + PMC); C4 resample tile A/B (IT=4 vs IT=8)
set -e
O=gpurun_out/r4c
mkdir -p $O
bash tools/gpu_profile.sh $O/prof
bash tools/gpu_profile_c345.sh $O/prof345
bash tools/gpu_bench_rep.sh $O/ab 3 "--no-secondary --model kitagawa --particles 2097152" "gen_amd/variants/rsit8.so|--no-secondary --model kitagawa --particles 2097152" > $O/ab.log 2>&1
