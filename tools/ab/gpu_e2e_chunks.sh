#!/bin/bash
# host-API e2e (ms_schedule_batch_compact / ms_schedule_batch at config C) with 1 / 2 / 3 / 4 chunks; compact parity first
set -o pipefail
TAG=${1:-r03t}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "compact or schedule" > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2 3 4 2 1; do
  MINISCHED_E2E_CHUNKS=$k $T 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs > gpurun_out/$TAG/b$k.json 2> gpurun_out/$TAG/b$k.err || exit 1
  echo chunks=$k $(python -c "import json; d=json.loads(open('gpurun_out/$TAG/b$k.json').read().strip().split(chr(10))[-1]); print('compact', round(d['e2e_compact']['ms_median'],4), [round(x,3) for x in d['e2e_compact']['runs']], 'full', round(d['e2e']['ms_median'],4))")
done
