#!/bin/bash
# Per-shard K1 counters for bench.py's N > 1 roofline: for G = 2, 4, 8 the sweep of one
# strong-scaling shard (tools/g8_shard_sweep.py: N/G rows x 100k pods, keys out), kernel
# stats + one SQ --pmc pass; summarised by tools/shard_profile_summary.py into
# profiles/<tag>_pmc_shard<rows>.json (bench.py --profile-shard-prefix).
set -o pipefail
TAG=${1:-r04}
export TMPDIR=/tmp
for G in 2 4 8; do
  OUT=gpurun_out/prof_shard_${TAG}/G$G; mkdir -p $OUT
  G=$G timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python tools/g8_shard_sweep.py > $OUT/run.json 2> $OUT/stats.err || { echo G$G stats failed; tail $OUT/stats.err; exit 1; }
  G=$G timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- python tools/g8_shard_sweep.py > /dev/null 2> $OUT/sq.err || { echo G$G sq failed; tail $OUT/sq.err; exit 1; }
done
echo ok
