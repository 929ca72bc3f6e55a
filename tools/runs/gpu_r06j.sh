# round 6: config E after the ranks-4..7 walk: warm-up size (0 / 4096 / 8192 pods in batches of 64),
# validator phase stamps (vstamps build)
set -o pipefail
T=${1:-r06j}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
e() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['seq_counters_all_reps'], d['codes'])" $1 $2; }
for i in 1 2; do
  for v in main w0 w4k; do
    LIB=$L/libminisched_gpu_$v.so; [ $v = main ] && LIB=$L/libminisched_gpu.so
    MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    e gpurun_out/${T}_E$v$i.jsonl $v
  done
done
MINISCHED_LIB=$L/libminisched_gpu_vstamps.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_vst.jsonl 2> gpurun_out/${T}_vst.err || { tail gpurun_out/${T}_vst.err; exit 1; }
grep MS_VSTAMPS gpurun_out/${T}_vst.err | tail -1 | cut -c1-700
