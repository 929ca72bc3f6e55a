#!/bin/bash
# round-3 check: new GPU tests, bench (with configs B/D/E), naming probe, config-E profile
set -o pipefail
mkdir -p gpurun_out/r03b
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py tests/test_host_cpp.py -v --timeout 300 --timeout-method thread -k "library or node_sharded_full or weak_shard or four_contexts or large_call or readme or compact or replay" > gpurun_out/r03b/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r03b/tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err || { tail -5 gpurun_out/r03b/bench.err; exit 1; }
cut -c1-700 gpurun_out/r03b/bench.json
timeout -k 10 240 python -u tools/probe_naming.py > gpurun_out/r03b/naming.log 2>&1 || { tail -5 gpurun_out/r03b/naming.log; exit 1; }
grep -v "^{" gpurun_out/r03b/naming.log | tail -5
bash tools/profile_e.sh r03 > gpurun_out/r03b/prof_e.log 2>&1 || { tail -5 gpurun_out/r03b/prof_e.log; exit 1; }
tail -30 gpurun_out/r03b/prof_e.log
