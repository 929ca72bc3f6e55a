#!/bin/bash
# rocprofv3 passes for the headline kernel: kernel stats, then one --pmc pass
# per TCC counter group (never combined with tracing domains), then SQ counters.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/bench_stats.json 2> $OUT/stats.err || { echo stats pass failed; tail $OUT/stats.err; exit 1; }
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > /dev/null 2> $OUT/fetch.err || { echo fetch pass failed; tail $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > /dev/null 2> $OUT/write.err || { echo write pass failed; tail $OUT/write.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || { echo sq pass failed; tail $OUT/sq.err; }
ls -R $OUT | head -40
