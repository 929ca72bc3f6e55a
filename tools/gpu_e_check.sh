# config E: parity subset (resource-aware / sequential / full-size E), E timing, kernel trace of the steps
set -o pipefail
TAG=${1:-r02zf}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resource or config_e or chunked or commit or sequential" > gpurun_out/${TAG}_e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/${TAG}_e.jsonl 2> gpurun_out/${TAG}_e.err || exit 1
cut -c1-260 gpurun_out/${TAG}_e.jsonl
OUT=gpurun_out/e_${TAG}; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python -u tools/bench_configs.py --configs E --reps 1 > $OUT/e.jsonl 2> $OUT/e.err || exit 1
grep -E "seq_step|topk_merge|tp_topk" $OUT/run_kernel_stats.csv | cut -c1-220
