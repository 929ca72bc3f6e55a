#!/bin/bash
# rocprofv3 passes over config E (50k nodes x 200k pods, exact sequential):
# kernel trace + stats, one --pmc pass per counter group (never combined with
# tracing domains), and the validator's wave durations from the MS_VSTAMPS
# diagnostic build (`make -C mini-kube-scheduler_amd vstamps`, built in-tree
# beforehand). Summary -> profiles/<tag>_pmc_E.json (read by bench.py's config
# E roofline) and profiles/<tag>_e_kernel_stats.csv (the box keeps only
# gpurun_out/: rerun the summary here on the merged gpurun_out/prof_e_<tag>).
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/prof_e_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
B="python tools/bench_configs.py --configs E --reps 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/bench_stats.jsonl 2> $OUT/stats.err || { echo stats pass failed; tail $OUT/stats.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || { echo sq pass failed; tail $OUT/sq.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > /dev/null 2> $OUT/fetch.err || { echo fetch pass failed; tail $OUT/fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > /dev/null 2> $OUT/write.err || { echo write pass failed; tail $OUT/write.err; exit 1; }
MINISCHED_LIB=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_vstamps.so timeout -k 10 200 $B > $OUT/vst.jsonl 2> $OUT/vst.err || { echo vstamps run failed; tail $OUT/vst.err; exit 1; }
python tools/e_profile_summary.py $OUT $TAG
