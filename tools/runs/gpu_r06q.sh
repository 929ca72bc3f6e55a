# round 6: config E with one sweep tile per CU (runtime tile height: 208 rows at 50k nodes) and 8- vs
# 12-wave step workgroups -- parity (main build and w8), then a same-run A/B against the round's HEAD build
set -o pipefail
T=${1:-r06q}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -k "config_e or seq or sequential or fuzz or golden or chunked" > gpurun_out/${T}_e_tests.log 2>&1 || { tail -30 gpurun_out/${T}_e_tests.log; exit 1; }
tail -1 gpurun_out/${T}_e_tests.log
MINISCHED_LIB=$L/libminisched_gpu_w8.so timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -k "config_e or seq or sequential or chunked" > gpurun_out/${T}_e_tests_w8.log 2>&1 || { tail -30 gpurun_out/${T}_e_tests_w8.log; exit 1; }
tail -1 gpurun_out/${T}_e_tests_w8.log
for i in 1 2; do
  for v in head main w8 w8t256; do
    LIB=$L/libminisched_gpu_$v.so; [ $v = main ] && LIB=$L/libminisched_gpu.so
    MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes'], d['seq_counters_all_reps']['recomputes'])" gpurun_out/${T}_E$v$i.jsonl $v
  done
done
