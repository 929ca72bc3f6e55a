# config E: the top-4 merge inside the step (default) vs its own launch (MINISCHED_SEQ_MERGE=kernel)
set -o pipefail
TAG=${1:-r02ze}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resource or config_e or chunked or commit or sequential" > gpurun_out/${TAG}_e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_e_tests.log; [ $rc -eq 0 ] || exit $rc
for m in step kernel step kernel; do
MINISCHED_SEQ_MERGE=$m timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/${TAG}_e_$m.jsonl 2> gpurun_out/${TAG}_e_$m.err || exit 1
echo merge=$m; cut -c1-200 gpurun_out/${TAG}_e_$m.jsonl
done
OUT=gpurun_out/e_merge_${TAG}; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python -u tools/bench_configs.py --configs E --reps 1 > $OUT/e.jsonl 2> $OUT/e.err || exit 1
grep -E "seq_step|topk_merge|tp_topk" $OUT/run_kernel_stats.csv | cut -c1-200
