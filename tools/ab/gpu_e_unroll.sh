#!/bin/bash
# config E: rows unrolled per block in the transposed batch sweep (MS_TP_UNROLL 1 / 2 default / 4), alternating
set -o pipefail
TAG=${1:-r03zs}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for r in 1 2; do
  for v in u2 u1 u4; do
    lib=$L/libminisched_gpu_$v.so; [ $v = u2 ] && lib=$L/libminisched_gpu.so
    MINISCHED_LIB=$lib timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/$TAG/e_$v.$r.jsonl 2> gpurun_out/$TAG/e_$v.$r.err || exit 1
    echo $v $(python -c "import json; d=json.loads(open('gpurun_out/$TAG/e_$v.$r.jsonl').read().split(chr(10))[0]); print(round(d['median_s']*1e3,2), d['codes'], d['seq_counters_all_reps'])")
  done
done
