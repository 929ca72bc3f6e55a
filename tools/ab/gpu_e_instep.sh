#!/bin/bash
# config E: batch k+1's top-4 merge inside step k by the sweep workgroups (default) vs a
# k_topk_merge launch after each step (MINISCHED_SEQ_MERGE=launch); the validator's fallback
# (MINISCHED_SEQ_MERGE=fallback: workers skip, the validator merges every pod) for parity only
set -o pipefail
TAG=${1:-r03za}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "resource or sequential or config_e" > gpurun_out/$TAG/e_tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/e_tests.log; [ $rc -eq 0 ] || exit $rc
MINISCHED_SEQ_MERGE=fallback $T 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "config_e or sequential_batch_sizes or fuzz_resource_sequential" > gpurun_out/$TAG/e_tests_fb.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/e_tests_fb.log; [ $rc -eq 0 ] || exit $rc
for v in instep launch instep launch; do
  MINISCHED_SEQ_MERGE=$v $T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/$TAG/e_$v.jsonl 2> gpurun_out/$TAG/e_$v.err || exit 1
  echo merge=$v $(python -c "import json; d=json.loads(open('gpurun_out/$TAG/e_$v.jsonl').read().split(chr(10))[0]); print(round(d['median_s']*1e3,2), d['codes'], d['seq_counters_all_reps'])")
done
cd /tmp && $T 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs E --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find gpurun_out/$TAG/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/$TAG/kernel_stats.csv
head -6 gpurun_out/$TAG/kernel_stats.csv | cut -c1-220
MINISCHED_LIB=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_vstamps.so $T 200 python -u tools/bench_configs.py --configs E --reps 1 > gpurun_out/$TAG/e_vst.jsonl 2> gpurun_out/$TAG/e_vst.err || exit 1
grep MS_VSTAMPS gpurun_out/$TAG/e_vst.err | tail -1
