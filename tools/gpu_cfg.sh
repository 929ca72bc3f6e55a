#!/bin/bash
# Secondary config timings only (tools/bench_configs.py), e.g. bash tools/gpu_cfg.sh E,B tag
set -o pipefail
mkdir -p gpurun_out
CFG=${1:-B,C,D,E}
TAG=${2:-cfg}
timeout -k 10 300 python tools/bench_configs.py --configs $CFG > gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}.err || { echo configs failed; tail -5 gpurun_out/${TAG}.err; exit 1; }
cat gpurun_out/${TAG}.jsonl
