# round 6: timed-region one-off: per-step events + a kernel trace
# of exactly the driver's bench shape (--steps 20 --warmup 5)
set -o pipefail
T=${1:-r06a}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 240 python -u tools/probe_timed_region.py > gpurun_out/${T}_timed.jsonl 2> gpurun_out/${T}_timed.err || { tail gpurun_out/${T}_timed.err; exit 1; }
cut -c1-400 gpurun_out/${T}_timed.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/${T}_trace_bench.json 2> gpurun_out/${T}_trace.err || { tail gpurun_out/${T}_trace.err; exit 1; }
cut -c1-300 gpurun_out/${T}_trace_bench.json
timeout -k 10 300 python -u -m pytest tests/test_host_cpp.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_host_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_host_tests.log; exit $rc
