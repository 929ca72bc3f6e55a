# round 6: config E micro A/Bs on the closing kernel: merge poll sleep 1 / 4 (default 2), warm-up
# 3,072 / 5,120 pods (default 4,096)
set -o pipefail
T=${1:-r06aj}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for i in 1 2; do
  for v in main sl1 sl4 w3k w5k; do
    LIB=$L/libminisched_gpu_$v.so; [ $v = main ] && LIB=$L/libminisched_gpu.so
    MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes']['success'])" gpurun_out/${T}_E$v$i.jsonl $v
  done
done
