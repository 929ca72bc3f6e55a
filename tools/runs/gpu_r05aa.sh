# round 5: multi-term NodeAffinity keys in name-digit lane order with hash skipping, seg early exit — parity, timing
set -o pipefail
T=${1:-r05aa}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "nam" > gpurun_out/${T}_nam_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_nam_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python tools/bench_nam.py --reps 5 2>/dev/null | tail -1 | tee -a gpurun_out/${T}_nam.txt || exit 1; done
