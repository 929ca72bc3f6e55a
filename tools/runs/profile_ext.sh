#!/bin/bash
# kernel stats + one SQ --pmc pass for the extension sweeps (tools/tt_time.py, tools/na_time.py)
# and the G = 8 strong-scaling shard (tools/g8_shard_sweep.py), for DESIGN's per-kernel table.
set -o pipefail
TAG=${1:-r04}
export TMPDIR=/tmp
for t in tt na g8; do
  case $t in tt) B="python tools/tt_time.py";; na) B="python tools/na_time.py";; g8) B="python tools/g8_shard_sweep.py";; esac
  OUT=gpurun_out/prof_ext_${TAG}/$t; mkdir -p $OUT
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/run.json 2> $OUT/stats.err || { echo $t stats failed; tail $OUT/stats.err; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || { echo $t sq failed; tail $OUT/sq.err; exit 1; }
done
echo ok
