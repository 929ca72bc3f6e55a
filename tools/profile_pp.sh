#!/bin/bash
# rocprofv3 passes over bench.py's timed kernel (K1 pp, config C, N = 1):
# kernel trace + stats, then one --pmc pass per counter group (never combined
# with tracing domains): SQ issue counters, FETCH_SIZE, WRITE_SIZE.
# Summary -> profiles/<tag>_pmc_C.json (read by bench.py's roofline) and
# profiles/<tag>_kernel_stats.csv.
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras --profile-json /dev/null"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/bench_stats.json 2> $OUT/stats.err || { echo stats pass failed; tail $OUT/stats.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || { echo sq pass failed; tail $OUT/sq.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > /dev/null 2> $OUT/fetch.err || { echo fetch pass failed; tail $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > /dev/null 2> $OUT/write.err || { echo write pass failed; tail $OUT/write.err; exit 1; }
python tools/pp_profile_summary.py $OUT $TAG
