# round 5: the in-library node-sharded TaintToleration cycle in the two-pass form (census all-gather,
# picks, uint64 MAX reduce-scatter, slice finals) — loopback world > 1, sharded, taint suites
set -o pipefail
T=${1:-r05ac}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_loopback.py tests/test_gpu_sharded.py tests/test_gpu_taint.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
MINISCHED_TT=v1 timeout -k 10 600 python -u -m pytest tests/test_gpu_loopback.py -m gpu -x -q --timeout 300 --timeout-method thread -k "taint or tt or 3" > gpurun_out/${T}_v1_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_v1_tests.log; [ $rc -eq 0 ] || exit $rc
