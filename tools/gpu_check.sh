#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_${TAG}.log
[ $rc -eq 0 ] || { echo "pytest gpu failed rc=$rc"; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke_${TAG}.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo bench failed; tail gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/prof_${TAG}.err || { echo rocprof failed; tail gpurun_out/prof_${TAG}.err; exit 1; }
find gpurun_out/prof_${TAG} -name '*stats*' | head
