# round 6: config E A/B: the node table's columns in one 2 MB-rounded allocation (main, MS_TABLE_ONE_ALLOC=1)
# vs one allocation per column (oa0); the validator phase stamps of both after the E runs
set -o pipefail
T=${1:-r06ae}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -m gpu -k "config_e_full" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2 3; do
  for v in main oa0; do
    LIB=$L/libminisched_gpu_$v.so; [ $v = main ] && LIB=$L/libminisched_gpu.so
    MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes']['success'])" gpurun_out/${T}_E$v$i.jsonl $v
  done
done
for v in vstamps vstoa0; do
  MINISCHED_LIB=$L/libminisched_gpu_$v.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_$v.jsonl 2> gpurun_out/${T}_$v.err || { tail gpurun_out/${T}_$v.err; exit 1; }
  echo "$v: $(grep MS_VSTAMPS gpurun_out/${T}_$v.err | tail -1 | sed -E 's/.*(epilogue parts: [^|]*).*/\1/')"
done
