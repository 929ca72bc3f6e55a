#!/bin/bash
# config E: pipelined vs serial batches, plus validator phase stamps (diagnostic build)
set -o pipefail
mkdir -p gpurun_out
for p in 1 0; do
  MINISCHED_SEQ_PIPE=$p timeout -k 10 120 python tools/bench_configs.py --configs E --reps 2 > gpurun_out/pipe_$p.jsonl 2>/dev/null || exit 1
  echo "pipe $p: $(python3 -c "import json;d=json.load(open('gpurun_out/pipe_$p.jsonl'));print(round(d['median_s'],4), d['seq_counters_all_reps'])")"
  MINISCHED_SEQ_PIPE=$p MINISCHED_LIB=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_vstamps.so timeout -k 10 120 python tools/bench_configs.py --configs E --reps 1 2>&1 >/dev/null | grep MS_VSTAMPS || exit 1
done
