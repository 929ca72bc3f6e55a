#!/bin/bash
# VALU issue rate vs waves per SIMD: the event-clock pass of
# tools/ubench/valu_rates (W = 1/2/4/8/16), then ONE --pmc pass over the same
# program (kernel trace on: durations per dispatch) with SQ_INSTS_VALU,
# SQ_ACTIVE_INST_VALU (quad-cycles summed over waves), SQ_BUSY_CYCLES, SQ_WAVES,
# SQ_WAVE_CYCLES and GRBM_GUI_ACTIVE (cycles summed over the 8 XCDs).
# Summary -> profiles/<tag>_valu_issue.json (tools/ubench/valu_pmc_summary.py).
set -o pipefail
TAG=${1:-r05b}
OUT=gpurun_out/valu_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
B=tools/ubench/valu_rates
timeout -k 10 120 $B 1 2 4 8 16 > $OUT/event_rates.txt 2> $OUT/event.err || { echo event pass failed; tail $OUT/event.err; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    -d $OUT/pmc -o run --output-format csv -- $B 1 2 4 8 16 > $OUT/pmc_stdout.txt 2> $OUT/pmc.err || { echo pmc pass failed; tail $OUT/pmc.err; exit 1; }
python tools/ubench/valu_pmc_summary.py $OUT $TAG
