#!/bin/bash
# config E A/B: the default build against variant builds (tools/build_variants.sh), with phase stamps
# usage: tools/gpu_e_walk.sh TAG "v1 v2 ..." "vst1 vst2 ..."
set -o pipefail
TAG=${1:-r03k}; VARS=${2:-"default w65"}; VSTS=${3-"vw17 vw65"}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
L=$PWD/mini-kube-scheduler_amd/minisched_amd
$T 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "resource or sequential or config_e" > gpurun_out/$TAG/e_tests.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/e_tests.log; [ $rc -eq 0 ] || exit $rc
for v in $VARS $VARS; do
  if [ $v = default ]; then LIB=$L/libminisched_gpu.so; else LIB=$L/libminisched_gpu_$v.so; fi
  MINISCHED_LIB=$LIB $T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/$TAG/e_$v.jsonl 2> gpurun_out/$TAG/e_$v.err || exit 1
  echo $v $(python -c "import json; d=json.loads(open('gpurun_out/$TAG/e_$v.jsonl').read().split(chr(10))[0]); print(round(d['median_s']*1e3,2), d.get('parity_vs_oracle_prefix'), d.get('fit_errors'))")
done
for v in $VSTS; do
  MINISCHED_LIB=$L/libminisched_gpu_$v.so $T 200 python -u tools/bench_configs.py --configs E --reps 1 > gpurun_out/$TAG/e_$v.jsonl 2> gpurun_out/$TAG/e_$v.err || exit 1
  grep MS_VSTAMPS gpurun_out/$TAG/e_$v.err | tail -1
done
