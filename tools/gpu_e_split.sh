# config E kernel durations with the validator and the sweep in separate launches (MINISCHED_SEQ_PIPE=0)
set -o pipefail
TAG=${1:-r02n}
OUT=gpurun_out/e_split_${TAG}; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MINISCHED_SEQ_PIPE=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python -u tools/bench_configs.py --configs E --reps 1 > $OUT/e.jsonl 2> $OUT/e.err || exit 1
find $OUT -name '*kernel_stats.csv' | xargs cat
