# C3 layout A/B on one box: LDS window (change points kept in LDS) and block size; 2 rounds
set -e
O=gpurun_out/coal_ab3
mkdir -p $O
for r in 1 2; do
  for v in coal_b256w7 coal_b256w6 coal_b256w8 coal_b512w6 coal_b512w7; do
    lib=gen_amd/libgen_hip.so; [ $v != base ] && lib=gen_amd/variants/$v.so
    GEN_HIP_LIB=$lib timeout -k 10 120 python tools/bench_coal.py --cpu-chains 1 > $O/${v}_$r.json 2> $O/${v}_$r.err
  done
done
