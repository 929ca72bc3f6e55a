# round 6: the merge's lanes combining their sorted top-8 by a 6-stage butterfly (MS_MERGE_SORTED=2, main)
# vs 8 rounds of wave max + shift (s1): GPU suite, E A/B, the timeline build
set -o pipefail
T=${1:-r06af}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in main s1; do
    LIB=$L/libminisched_gpu_$v.so; [ $v = main ] && LIB=$L/libminisched_gpu.so
    MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes']['success'])" gpurun_out/${T}_E$v$i.jsonl $v
  done
done
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('tl build E', round(d['median_s']*1e3,2), 'ms', d['codes']['success'])" gpurun_out/${T}_tl.jsonl
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_e_wg_timeline_run.json | tail -2
rm -f gpurun_out/${T}_tl.bin
