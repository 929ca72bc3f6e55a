# round 5: multi-term NodeAffinity parity (new plugin set 4), the sequential suite with the
# in-step merge as the default, then the unstamped per-workgroup timeline of config E
set -o pipefail
T=${1:-r05h}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nam.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_nam_tests.log 2>&1; rc=$?; tail -4 gpurun_out/${T}_nam_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sequential or config_e or resource or seq or merge" > gpurun_out/${T}_e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_e_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r05g.sh ${T}
