# the multi-rank GPU tests (host transport 2..4 ranks on one GPU, forced RCCL world 1) and the 2-rank torchrun rehearsal
set -e
O=${1:-gpurun_out/mr}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multirank.py -m gpu -q --timeout 300 --timeout-method thread > $O/mr_tests.log 2>&1
bash tools/gpu_torchrun2.sh
