set -e
mkdir -p gpurun_out/cmp
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/cmp/new.json 2> gpurun_out/cmp/new.err
GEN_HIP_LIB=$PWD/prev_lib.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/cmp/prev.json 2> gpurun_out/cmp/prev.err
