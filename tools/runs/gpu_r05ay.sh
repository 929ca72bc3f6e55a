# round 5: config E with the sweep's 4-row blocks unrolled twice (MS_TP_UNROLL=2) vs once, same box
set -o pipefail
T=${1:-r05ay}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for v in unr2 main unr2 main; do
  if [ $v = main ]; then LIB=$L/libminisched_gpu.so; else LIB=$L/libminisched_gpu_$v.so; fi
  MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E_$v.jsonl 2> gpurun_out/${T}_E_$v.err || { tail gpurun_out/${T}_E_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes'])" gpurun_out/${T}_E_$v.jsonl $v
done
