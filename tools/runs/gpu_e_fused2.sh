# config E: depth-2 fused pipeline (default) vs depth 1 (MINISCHED_SEQ_PIPE=fused): parity first, then timing
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resource or config_e or sequential or commit or chunked" > gpurun_out/r04w_e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04w_e_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r04w_e_tests.log | head -20; exit $rc; }
for i in 1 2; do
  for m in fused2 fused; do
    ms=$(MINISCHED_SEQ_PIPE=$m timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3), d['seq_counters_all_reps'])") || exit 1
    echo "$m E_ms=$ms" >> gpurun_out/r04w_e_fused2.txt
  done
done
cat gpurun_out/r04w_e_fused2.txt
