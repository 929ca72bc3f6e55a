# round 5: two-pass TaintToleration over node shards (census, pick, final entry points): parity, timing
set -o pipefail
T=${1:-r05ab}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "tt or taint" > gpurun_out/${T}_tt_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tt_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python tools/bench_tt.py --reps 5 2>/dev/null | tail -1 | tee -a gpurun_out/${T}_tt.txt || exit 1; done
