#!/bin/bash
# N = 1 bench forms, interleaved twice: per-step timing events on/off, grouped decodes on/off.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/n1_ab.jsonl
for rep in 1 2; do
for cfg in "1 0" "0 0" "1 1" "0 1"; do
  set -- $cfg
  MINISCHED_BENCH_STEP_EVENTS=$1 MINISCHED_BENCH_PIPE1=$2 timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu-baseline \
      > gpurun_out/n1.json 2> gpurun_out/n1.err || { tail gpurun_out/n1.err; exit 1; }
  python -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/n1.json') if l.startswith('{')][0])
print(json.dumps({'rep': $rep, 'step_events': $1, 'pipe1': $2, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'pods_scheduled': d['pods_scheduled']}))" | tee -a gpurun_out/n1_ab.jsonl
done
done
