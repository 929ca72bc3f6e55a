# config E: batch k+1's merge inside step k (MINISCHED_SEQ_MERGE=instep) vs a merge launch
# after each step (launch, the default): sequential parity first, then timing
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r04zk}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resource or config_e or sequential or commit or chunked" > gpurun_out/${T}_e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_e_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_e_tests.log | head -20; exit $rc; }
for i in 1 2; do
  for m in instep launch; do
    ms=$(MINISCHED_SEQ_MERGE=$m timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3), d['seq_counters_all_reps'])") || exit 1
    echo "merge=$m E_ms=$ms" >> gpurun_out/${T}_e_instep.txt
  done
done
cat gpurun_out/${T}_e_instep.txt
