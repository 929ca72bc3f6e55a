#!/bin/bash
# config E time vs the speculative sweep's pods-per-wave chunk
set -o pipefail
mkdir -p gpurun_out
for c in 4 8 16 32; do
  MINISCHED_SEQ_CHUNK=$c timeout -k 10 120 python tools/bench_configs.py --configs E --reps 2 > gpurun_out/chunk_$c.jsonl 2>/dev/null || exit 1
  echo "chunk $c: $(python3 -c "import json;d=json.load(open('gpurun_out/chunk_$c.jsonl'));print(round(d['median_s'],4))")"
done
