#!/bin/bash
# K1 geometry sweep + SQ counters of the production K1 (one GPU call).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-geom}
timeout -k 10 300 python tools/k1_geom.py > gpurun_out/geom_${TAG}.jsonl 2> gpurun_out/geom_${TAG}.err || { echo geom failed; tail gpurun_out/geom_${TAG}.err; exit 1; }
cat gpurun_out/geom_${TAG}.jsonl
bash tools/pmc_k1.sh v7
