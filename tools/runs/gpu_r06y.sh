# round 6: the write-back with its rows loaded and derived together (MS_WB_ILP=1, main) vs row after row (ilp0):
# GPU suite, then E A/B and the validator's phase stamps for both
set -o pipefail
T=${1:-r06y}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in main ilp0; do
    LIB=$L/libminisched_gpu_$v.so; [ $v = main ] && LIB=$L/libminisched_gpu.so
    MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes']['success'])" gpurun_out/${T}_E$v$i.jsonl $v
  done
done
for v in vstamps vstilp0; do
  MINISCHED_LIB=$L/libminisched_gpu_$v.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_$v.jsonl 2> gpurun_out/${T}_$v.err || { tail gpurun_out/${T}_$v.err; exit 1; }
  echo "$v: $(grep MS_VSTAMPS gpurun_out/${T}_$v.err | tail -1 | cut -c1-700)"
done
