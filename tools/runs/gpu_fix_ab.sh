# K1 fixed-slot form: GPU suite, then config C bench with MINISCHED_PP_FIX=1/0 alternating, G=8 probe
set -o pipefail
TAG=${1:-r04j}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    echo "FIX=$f $(MINISCHED_PP_FIX=$f timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-extras --no-cpu-baseline 2>/dev/null | tail -1 | cut -c1-200)" >> gpurun_out/${TAG}_fix_ab.txt || exit 1
  done
done
cat gpurun_out/${TAG}_fix_ab.txt
for f in 1 0; do
  echo "FIX=$f $(MINISCHED_PP_FIX=$f PROBE_G=8,4,2 PROBE_STREAMS=1 timeout -k 10 200 python tools/step_probe_lib.py 2>/dev/null | tail -1)" >> gpurun_out/${TAG}_fix_ab.txt || exit 1
done
tail -2 gpurun_out/${TAG}_fix_ab.txt
