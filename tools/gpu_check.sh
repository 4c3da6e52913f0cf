# the whole -m gpu suite and smoke() (a pre-commit check on the GPU box)
set -e
O=${1:-gpurun_out/check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
