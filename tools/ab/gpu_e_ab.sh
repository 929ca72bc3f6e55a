#!/bin/bash
# config E: parity subset, then the default engine vs MINISCHED_SEQ_MERGE=launch (A/B)
set -o pipefail
TAG=${1:-r03i}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "resource or sequential or config_e" > gpurun_out/$TAG/e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/e_tests.log; [ $rc -eq 0 ] || exit $rc
$T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/$TAG/e_default.jsonl 2> gpurun_out/$TAG/e1.err || exit 1
MINISCHED_SEQ_MERGE=launch $T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/$TAG/e_launch.jsonl 2> gpurun_out/$TAG/e2.err || exit 1
cut -c1-300 gpurun_out/$TAG/e_default.jsonl gpurun_out/$TAG/e_launch.jsonl
