set -e
mkdir -p gpurun_out/rsprof
export TMPDIR=/tmp
for rep in 1 2; do
for v in base wave; do
  lib=gen_amd/libgen_hip.so; [ $v = wave ] && lib=gen_amd/variants/wave.so
  for m in "--model lgssm" "--model kitagawa --particles 2097152"; do
    tag=$(echo $m | tr -d ' -' | cut -c1-20)
    GEN_HIP_LIB=$lib GH_PROF_STEPS=30 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rsprof/${v}_${tag}_$rep -o run --output-format csv -- python3 tools/profile_run.py $m > gpurun_out/rsprof/${v}_${tag}_$rep.log 2>&1
  done
done
done
