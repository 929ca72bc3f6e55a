#!/bin/bash
# kernel trace of the strong-scaling step probe at G = 8 (coalesced pairs and
# single launches): per-dispatch K1 durations by grid size.
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/prof_g8pair_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
PROBE_G=8 PROBE_STREAMS=1 PROBE_COALESCE=1,0 PROBE_STEPS=100 timeout -k 10 150 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python tools/step_probe_lib.py > $OUT/probe.json 2> $OUT/probe.err || { tail $OUT/probe.err; exit 1; }
echo ok
