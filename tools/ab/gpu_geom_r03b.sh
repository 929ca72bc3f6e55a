#!/bin/bash
# K1 pp 8-word single-wave form vs the 4-word form at strong-scaling shards
set -o pipefail
mkdir -p gpurun_out/geom_r03b
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
V="kw8:;kw4:MINISCHED_PP_WORDS=4;kw4w2:MINISCHED_PP_WAVES=2;kw8c16:MINISCHED_PP_CHUNK=16;kw8c48:MINISCHED_PP_CHUNK=48;kw8c64:MINISCHED_PP_CHUNK=64;kw8c128:MINISCHED_PP_CHUNK=128"
for G in 8 16; do
  N=$((100000 / G)); B=$((100000 - N))
  for MODE in sweep; do
  AB_NODES=$N AB_NODE_BASE=$B AB_PODS=100000 AB_MODE=$MODE AB_ROUNDS=12 AB_VARIANTS="$V" timeout -k 10 200 python -u tools/ab_pp.py > gpurun_out/geom_r03b/g$G$MODE.json 2> gpurun_out/geom_r03b/g$G.err || { tail -5 gpurun_out/geom_r03b/g$G.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/geom_r03b/g$G$MODE.json'))
print('G=$G $MODE', {k: round(v['median_ms']*1e3,1) for k,v in d.items() if isinstance(v, dict)}, d['identical'])"
  done
done
AB_NODES=12500 AB_NODE_BASE=87500 AB_PODS=800000 AB_MODE=sweep AB_ROUNDS=8 AB_VARIANTS="kw8:;kw4:MINISCHED_PP_WORDS=4" timeout -k 10 200 python -u tools/ab_pp.py > gpurun_out/geom_r03b/weak.json 2>/dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/geom_r03b/weak.json')); print('weak 12.5k x 800k', {k: round(v['median_ms']*1e3,1) for k,v in d.items() if isinstance(v, dict)}, d['identical'])"
for V2 in 8 4; do
  MINISCHED_PP_WORDS=$V2 AB_NODES=12500 AB_NODE_BASE=87500 AB_PODS=100000 AB_MODE=sweep AB_ROUNDS=5 AB_VARIANTS="x:" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/geom_r03b/prof_$V2 -o run --output-format csv -- python tools/ab_pp.py > /dev/null 2> gpurun_out/geom_r03b/prof_$V2.err || { tail -3 gpurun_out/geom_r03b/prof_$V2.err; exit 1; }
  grep k_sweep_nunn_pp gpurun_out/geom_r03b/prof_$V2/run_kernel_stats.csv | cut -d, -f1,2,4 | sed 's/(unsigned.*)"/"/'
done
