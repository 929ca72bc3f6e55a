# round 5: config E sweep unroll 2 as the default: E parity suites, then unroll 1 / 2 (main) / 4 on one box
set -o pipefail
T=${1:-r05az}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py tests/test_golden.py tests/test_gpu_loopback.py > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for v in unr1 main unr4 unr1 main unr4; do
  if [ $v = main ]; then LIB=$L/libminisched_gpu.so; else LIB=$L/libminisched_gpu_$v.so; fi
  MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E_$v.jsonl 2> gpurun_out/${T}_E_$v.err || { tail gpurun_out/${T}_E_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes'])" gpurun_out/${T}_E_$v.jsonl $v
done
