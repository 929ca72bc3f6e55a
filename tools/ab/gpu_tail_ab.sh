#!/bin/bash
# K1 pp last partial word: full word (t0), packed on one wave (t1), packed over 4 waves (default), alternating
set -o pipefail
TAG=${1:-r03zg}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp PROBE_ROWS=100000,99840,50010 PROBE_STEPS=200
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for r in 1 2 3; do
  for v in t0 t1 t4; do
    lib=$L/libminisched_gpu_$v.so; [ $v = t4 ] && lib=$L/libminisched_gpu.so
    MINISCHED_LIB=$lib timeout -k 10 200 python -u tools/probe_tail.py > gpurun_out/$TAG/$v.$r.json 2>&1 || exit 1
    echo $v $(tail -1 gpurun_out/$TAG/$v.$r.json)
  done
done
