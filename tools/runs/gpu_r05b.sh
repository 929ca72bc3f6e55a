# round 5: config E with binary64 tile keys in the sweep's sort network — sequential parity,
# same-run A/B against the u64 network (libminisched_gpu_f64off.so), E kernel trace; VALU issue ubench
set -o pipefail
T=${1:-r05b}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sequential or config_e or resource or seq" > gpurun_out/${T}_e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_e_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in f64off new; do
    if [ $v = new ]; then lib=$L/libminisched_gpu.so; else lib=$L/libminisched_gpu_$v.so; fi
    ms=$(MINISCHED_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3))") || exit 1
    echo "$v E_ms=$ms" | tee -a gpurun_out/${T}_e_ab.txt
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_etrace -o run --output-format csv -- python tools/bench_configs.py --configs E --reps 1 > /dev/null 2> gpurun_out/${T}_etrace.err || { echo trace failed; tail gpurun_out/${T}_etrace.err; exit 1; }
python tools/e_batches.py gpurun_out/${T}_etrace/run_kernel_trace.csv > gpurun_out/${T}_e_batches.json || exit 1
head -c 1500 gpurun_out/${T}_e_batches.json
bash tools/ubench/valu_pmc.sh ${T} > gpurun_out/${T}_valu.log 2>&1 || { tail gpurun_out/${T}_valu.log; exit 1; }
cat gpurun_out/${T}_valu.log
