#!/bin/bash
# config E A/B over env settings, each with validator phase stamps (diagnostic build)
# usage: bash tools/gpu_pipe.sh "MINISCHED_SEQ_PIPE=1" "MINISCHED_SEQ_PIPE=0 MINISCHED_SEQ_BATCH=256" ...
set -o pipefail
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python tools/bench_configs.py --configs E --reps 2 > gpurun_out/pipe_$i.jsonl 2>/dev/null || exit 1
  echo "[$cfg]: $(python3 -c "import json;d=json.load(open('gpurun_out/pipe_$i.jsonl'));print(round(d['median_s'],4), d['seq_counters_all_reps'])")"
  env $cfg MINISCHED_LIB=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_vstamps.so timeout -k 10 120 python tools/bench_configs.py --configs E --reps 1 2>&1 >/dev/null | grep MS_VSTAMPS || exit 1
done
