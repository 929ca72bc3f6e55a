# validator cost with one vs two stale batches (two-stream modes, kernel stats)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for p in 1 2; do
OUT=gpurun_out/e_pipe$p; rm -rf $OUT; mkdir -p $OUT
MINISCHED_SEQ_PIPE=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python -u tools/bench_configs.py --configs E --reps 1 > $OUT/e.jsonl 2> $OUT/e.err || exit 1
echo pipe=$p $(cut -c1-200 $OUT/e.jsonl)
grep -E "validate_seq|tp_topk|topk_merge" $OUT/run_kernel_stats.csv | cut -c1-160
done
