# round 5: k_nam_keys four rows per step with one rescale ballot: NAM parity suite, A/B at 50k x 100k
set -o pipefail
T=${1:-r05au}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nam.py > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for v in namhead main namhead main; do
  if [ $v = main ]; then LIB=$L/libminisched_gpu.so; else LIB=$L/libminisched_gpu_$v.so; fi
  MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_nam.py --reps 5 > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || { tail gpurun_out/${T}_$v.err; exit 1; }
  echo $v $(tail -1 gpurun_out/${T}_$v.json | cut -c1-120)
done
