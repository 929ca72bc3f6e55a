#!/bin/bash
# K1 parity + waves-per-workgroup A/B at several shard sizes, launches back to back (one GPU call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1; rc=$?; tail -2 gpurun_out/par.log; [ $rc -eq 0 ] || { grep -m3 -B10 "Error\|assert" gpurun_out/par.log | head -50; exit $rc; }
GEOM_REPS=10 GEOM_SHARDS=100000,50000,25000,12500 GEOM_RPL=30 GEOM_CHUNK=${GEOM_CHUNK:-0} GEOM_WAVES=${GEOM_WAVES:-1,2,4} GEOM_K1=${GEOM_K1:-v7} timeout -k 10 300 python tools/k1_geom.py > gpurun_out/geom2.jsonl 2> gpurun_out/geom2.err || { tail gpurun_out/geom2.err; exit 1; }
cat gpurun_out/geom2.jsonl
