#!/bin/bash
# rocprofv3 kernel stats of one secondary config run: bash tools/prof_cfg.sh E tag
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-E}
TAG=${2:-profcfg}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG} -o run --output-format csv -- python tools/bench_configs.py --configs $CFG --reps 2 > gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}.err || { echo prof failed; tail -5 gpurun_out/${TAG}.err; exit 1; }
cut -c1-160 gpurun_out/${TAG}/run_kernel_stats.csv | head -8
