#!/bin/bash
# compact host-array cycle: zero-copy single launch (default) vs staged copies + widen/narrow (MINISCHED_COMPACT_ZC=0)
set -o pipefail
TAG=${1:-r03zm}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "compact or nunn or pp or parity or config_c" > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0 1 0; do
  MINISCHED_COMPACT_ZC=$v $T 120 python -u tools/probe_compact.py >> gpurun_out/$TAG/probe.jsonl 2>> gpurun_out/$TAG/probe.err || exit 1
  tail -1 gpurun_out/$TAG/probe.jsonl
done
