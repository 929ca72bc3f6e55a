set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/e_prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python tools/bench_configs.py --configs E --reps 1 > $OUT/bench.jsonl 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
f=$(find $OUT -name "*kernel_trace.csv" | head -1); s=$(find $OUT -name "*kernel_stats.csv" | head -1)
python tools/e_timeline.py $f | tee $OUT/timeline.json
cp $s $OUT/kernel_stats.csv; rm -f $f
