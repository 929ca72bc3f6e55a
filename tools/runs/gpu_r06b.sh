# round 6: the changed suites (NAM label 255, TT final shard plans, host mirror) + the driver-shape bench
set -o pipefail
T=${1:-r06b}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nam.py tests/test_gpu_taint.py tests/test_host_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['device_ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel_ms_blocks']); print({k: v.get('ms') for k, v in d['configs'].items()})"
