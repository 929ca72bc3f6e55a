#!/bin/bash
# K1 pp geometry at the strong-scaling shard shapes (config C over G = 2/4/8):
# interleaved A/B of waves per workgroup and pods per workgroup, sweep only.
set -o pipefail
mkdir -p gpurun_out/geom_r03
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
V="def:;w1:MINISCHED_PP_WAVES=1;w2:MINISCHED_PP_WAVES=2;w8:MINISCHED_PP_WAVES=8;w16:MINISCHED_PP_WAVES=16;c48:MINISCHED_PP_CHUNK=48;c200:MINISCHED_PP_CHUNK=200;c400:MINISCHED_PP_CHUNK=400;w2c200:MINISCHED_PP_WAVES=2,MINISCHED_PP_CHUNK=200;w2c400:MINISCHED_PP_WAVES=2,MINISCHED_PP_CHUNK=400;w1c100:MINISCHED_PP_WAVES=1,MINISCHED_PP_CHUNK=100;w1c200:MINISCHED_PP_WAVES=1,MINISCHED_PP_CHUNK=200"
for G in 8 4 2; do
  N=$((100000 / G)); B=$((100000 - N))
  AB_NODES=$N AB_NODE_BASE=$B AB_PODS=100000 AB_MODE=sweep AB_ROUNDS=10 AB_VARIANTS="$V" timeout -k 10 200 python -u tools/ab_pp.py > gpurun_out/geom_r03/g$G.json 2> gpurun_out/geom_r03/g$G.err || { tail -5 gpurun_out/geom_r03/g$G.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/geom_r03/g$G.json'))
print('G=$G', {k: round(v['median_ms']*1e3,1) for k,v in d.items() if isinstance(v, dict)}, d['identical'])"
done
# fixed cost: the same shard with few pods
for P in 1000 10000; do
  AB_NODES=12500 AB_NODE_BASE=87500 AB_PODS=$P AB_MODE=sweep AB_ROUNDS=10 AB_VARIANTS="def:" timeout -k 10 100 python -u tools/ab_pp.py > gpurun_out/geom_r03/p$P.json 2>/dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/geom_r03/p$P.json')); print('12.5k x $P', round(d['def']['median_ms']*1e3,1), 'us')"
done
AB_NODES=12500 AB_NODE_BASE=87500 AB_PODS=100000 AB_MODE=sweep AB_VARIANTS="def:" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/geom_r03/prof -o run --output-format csv -- python tools/ab_pp.py > /dev/null 2> gpurun_out/geom_r03/prof.err || { tail -3 gpurun_out/geom_r03/prof.err; exit 1; }
find gpurun_out/geom_r03/prof -name "*kernel_stats.csv" -exec head -4 {} \;
