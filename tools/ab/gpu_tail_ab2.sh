#!/bin/bash
# K1 pp last partial word packed where it lowers the busiest SIMD (default) vs never (t0): parity, then alternating timings
set -o pipefail
TAG=${1:-r03zh}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "nunn or pp or fuzz or config_c or sharded or parity" > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
export PROBE_ROWS=100000,25000,25020,6250,50000 PROBE_STEPS=200
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for r in 1 2; do
  for v in t0 def; do
    lib=$L/libminisched_gpu_$v.so; [ $v = def ] && lib=$L/libminisched_gpu.so
    MINISCHED_LIB=$lib $T 200 python -u tools/probe_tail.py > gpurun_out/$TAG/$v.$r.json 2>&1 || exit 1
    echo $v $(tail -1 gpurun_out/$TAG/$v.$r.json)
  done
done
$T 300 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-configs > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/$TAG/bench.json').read().strip().split(chr(10))[-1]); print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'])"
