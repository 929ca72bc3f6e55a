#!/bin/bash
# rocprofv3 passes over tools/g8_shard_sweep.py (one strong-scaling shard's K1
# sweep, K launches): kernel trace + stats, then one --pmc pass (SQ counters).
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/prof_g8_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
B="python tools/g8_shard_sweep.py"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/run.json 2> $OUT/stats.err || { echo stats pass failed; tail $OUT/stats.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || { echo sq pass failed; tail $OUT/sq.err; exit 1; }
echo ok
