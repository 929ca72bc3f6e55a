# config E: parity of the sweep forms + A/B timing of the binary64 LeastAllocated form
set -o pipefail
TAG=${1:-r02o}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resource or config_e or chunked or commit" > gpurun_out/${TAG}_e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_e_tests.log; [ $rc -eq 0 ] || exit $rc
for f in 0 1; do
MINISCHED_SEQ_FAST=$f timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 3 > gpurun_out/${TAG}_e_fast$f.jsonl 2> gpurun_out/${TAG}_e_fast$f.err || exit 1
echo fast=$f; cut -c1-260 gpurun_out/${TAG}_e_fast$f.jsonl
done
bash tools/gpu_e_split.sh ${TAG} | grep -E "sweep_full_topk|validate_seq|topk_merge" | cut -c1-200
OUT=gpurun_out/e_fused_${TAG}; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python -u tools/bench_configs.py --configs E --reps 1 > $OUT/e.jsonl 2> $OUT/e.err || exit 1
grep -E "seq_step|topk_merge|tp_topk" $OUT/run_kernel_stats.csv | cut -c1-200
