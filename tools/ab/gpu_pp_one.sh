#!/bin/bash
# K1 pp one-pod-at-a-time small-shard form (MINISCHED_PP_ONE=1): parity, then the G=8/4 shard probe A/B
set -o pipefail
TAG=${1:-r03q}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
MINISCHED_PP_ONE=1 $T 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/one_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/one_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MINISCHED_PP_ONE=$v PROBE_G=8 PROBE_STREAMS=1 PROBE_STEPS=100 $T 120 python -u tools/step_probe_lib.py > gpurun_out/$TAG/probe_$v.json 2> gpurun_out/$TAG/probe_$v.err || exit 1
  echo one=$v $(tail -n 1 gpurun_out/$TAG/probe_$v.json)
done
for c in 16 32; do
  MINISCHED_PP_ONE=1 MINISCHED_PP_CHUNK=$c PROBE_G=8 PROBE_STREAMS=1 PROBE_STEPS=100 $T 120 python -u tools/step_probe_lib.py > gpurun_out/$TAG/probe_c$c.json 2> gpurun_out/$TAG/probe_c$c.err || exit 1
  echo one=1 chunk=$c $(tail -n 1 gpurun_out/$TAG/probe_c$c.json)
done
