#!/bin/bash
# config E: in-step merge (default) vs MINISCHED_SEQ_MERGE=launch, parity subset first, then phase stamps
set -o pipefail
TAG=${1:-r03l}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
L=$PWD/mini-kube-scheduler_amd/minisched_amd
$T 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "resource or sequential or config_e" > gpurun_out/$TAG/e_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/e_tests.log; [ $rc -eq 0 ] || exit $rc
for m in step launch step launch; do
  MINISCHED_SEQ_MERGE=$m $T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/$TAG/e_$m.jsonl 2> gpurun_out/$TAG/e_$m.err || exit 1
  echo $m $(python -c "import json; d=json.loads(open('gpurun_out/$TAG/e_$m.jsonl').read().split(chr(10))[0]); print(round(d['median_s']*1e3,2), d.get('parity_vs_oracle_prefix'), d.get('fit_errors'), d.get('seq_counters_all_runs'))")
done
MINISCHED_LIB=$L/libminisched_gpu_vst.so $T 200 python -u tools/bench_configs.py --configs E --reps 1 > gpurun_out/$TAG/e_vst.jsonl 2> gpurun_out/$TAG/e_vst.err || exit 1
grep MS_VSTAMPS gpurun_out/$TAG/e_vst.err | tail -1
