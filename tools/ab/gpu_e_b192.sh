#!/bin/bash
# config E: 192-pod speculative batches (MS_SEQ_BATCH=192 build) vs the default 128: parity of both, then timing
set -o pipefail
TAG=${1:-r03p}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for v in default b192; do
  if [ $v = default ]; then LIB=$L/libminisched_gpu.so; else LIB=$L/libminisched_gpu_$v.so; fi
  MINISCHED_LIB=$LIB $T 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "resource or sequential or config_e" > gpurun_out/$TAG/e_tests_$v.log 2>&1
  rc=$?; echo $v $(tail -1 gpurun_out/$TAG/e_tests_$v.log); [ $rc -eq 0 ] || exit $rc
done
for v in default b192 default b192; do
  if [ $v = default ]; then LIB=$L/libminisched_gpu.so; else LIB=$L/libminisched_gpu_$v.so; fi
  MINISCHED_LIB=$LIB $T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/$TAG/e_$v.jsonl 2> gpurun_out/$TAG/e_$v.err || exit 1
  echo $v $(python -c "import json; d=json.loads(open('gpurun_out/$TAG/e_$v.jsonl').read().split(chr(10))[0]); print(round(d['median_s']*1e3,2), d['codes'], d['seq_counters_all_reps'])")
done
