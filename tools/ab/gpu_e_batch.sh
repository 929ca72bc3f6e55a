#!/bin/bash
# config E: speculative batch size (MINISCHED_SEQ_BATCH <= 128) on the fused single-stream engine
set -o pipefail
TAG=${1:-r03o}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for b in 128 96 112 80 64 128; do
  MINISCHED_SEQ_BATCH=$b timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 3 > gpurun_out/$TAG/e_b$b.jsonl 2> gpurun_out/$TAG/e_b$b.err || exit 1
  echo b$b $(python -c "import json; d=json.loads(open('gpurun_out/$TAG/e_b$b.jsonl').read().split(chr(10))[0]); print(round(d['median_s']*1e3,2), d.get('fit_errors'))")
done
