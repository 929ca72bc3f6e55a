# round 6: NAM (parallel classes / row-part pick) suite + bench; the solo-rank loopback test and
# the honest per-rank probe
set -o pipefail
T=${1:-r06e}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nam.py "tests/test_gpu_loopback.py::test_solo_rank_probe_mode" -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_probe_rank.py > gpurun_out/${T}_probe_rank.jsonl 2> gpurun_out/${T}_probe_rank.err || { tail gpurun_out/${T}_probe_rank.err; exit 1; }
cat gpurun_out/${T}_probe_rank.jsonl
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_namprof -o run --output-format csv -- python tools/bench_nam.py > gpurun_out/${T}_namprof.log 2>&1 || { tail gpurun_out/${T}_namprof.log; exit 1; }
tail -2 gpurun_out/${T}_namprof.log
