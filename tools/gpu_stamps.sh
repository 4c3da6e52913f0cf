# k_resample1 phase clocks (GH_RS_STAMPS variant, `python tools/variants.py build rs_stamps`), C2 and C4
set -e
O=gpurun_out/stamps
mkdir -p $O
for args in "lg10 20" "kit 21"; do
  timeout -k 10 120 python tools/rs_stamps.py $args >> $O/stamps.txt 2>&1
done
