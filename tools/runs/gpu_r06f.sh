# round 6: NAM rescale multiply-high: NAM suite + NAM timing + kernel stats
set -o pipefail
T=${1:-r06f}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nam.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_namprof -o run --output-format csv -- python tools/bench_nam.py > gpurun_out/${T}_namprof.log 2>&1 || { tail gpurun_out/${T}_namprof.log; exit 1; }
grep median_ms gpurun_out/${T}_namprof.log
