# config E evidence: kernel trace of the default fused steps + PMC of the transposed sweep
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/e_fused_r02y; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python -u tools/bench_configs.py --configs E --reps 1 > $OUT/e.jsonl 2> $OUT/e.err || exit 1
grep -E "seq_step|topk_merge|tp_topk|build_drows" $OUT/run_kernel_stats.csv | cut -c1-180
bash tools/pmc_e_sweep.sh || exit 1
