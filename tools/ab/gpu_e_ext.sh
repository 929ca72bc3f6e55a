#!/bin/bash
# config E: certified ranks 4..7 for the validator's slow pods (default) vs top-4 only (MINISCHED_SEQ_EXT=0)
set -o pipefail
TAG=${1:-r03v}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "resource or sequential or config_e" > gpurun_out/$TAG/e_tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/e_tests.log; [ $rc -eq 0 ] || exit $rc
MINISCHED_SEQ_EXT=0 $T 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "config_e or sequential_batch_sizes" > gpurun_out/$TAG/e_tests0.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/e_tests0.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  MINISCHED_SEQ_EXT=$v $T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/$TAG/e_$v.jsonl 2> gpurun_out/$TAG/e_$v.err || exit 1
  echo ext=$v $(python -c "import json; d=json.loads(open('gpurun_out/$TAG/e_$v.jsonl').read().split(chr(10))[0]); print(round(d['median_s']*1e3,2), d['codes'], d['seq_counters_all_reps'])")
done
MINISCHED_LIB=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_vstamps.so $T 200 python -u tools/bench_configs.py --configs E --reps 1 > gpurun_out/$TAG/e_vst.jsonl 2> gpurun_out/$TAG/e_vst.err || exit 1
grep MS_VSTAMPS gpurun_out/$TAG/e_vst.err | tail -1
