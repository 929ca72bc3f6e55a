# round 6: config E A/B after the sorted merge (r06ab): the merge rounds' wave max by the unique-high-word form (wu,
# MS_MERGE_WMAX=wave_max_u64_unique) vs two 32-bit reductions (main); the config E full-size tests on main first
set -o pipefail
T=${1:-r06ac}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -m gpu -k "config_e_full" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2 3; do
  for v in main wu; do
    LIB=$L/libminisched_gpu_$v.so; [ $v = main ] && LIB=$L/libminisched_gpu.so
    MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes']['success'])" gpurun_out/${T}_E$v$i.jsonl $v
  done
done
