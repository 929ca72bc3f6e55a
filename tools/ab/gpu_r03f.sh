#!/bin/bash
# full GPU suite + library step probe (host phases) + bench
set -o pipefail
mkdir -p gpurun_out/r03f
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03f/tests.log; grep -E "FAILED|Error" gpurun_out/r03f/tests.log | head -5; [ $rc -eq 0 ] || exit $rc
MINISCHED_HOST_PROF=1 PROBE_G=8,4,2 PROBE_STREAMS=2,1 timeout -k 10 150 python -u tools/step_probe_lib.py > gpurun_out/r03f/step.json 2>&1 || { tail -3 gpurun_out/r03f/step.json; exit 1; }
grep -E "MS_HOST" gpurun_out/r03f/step.json | head -3; tail -n 1 gpurun_out/r03f/step.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03f/bench.json 2> gpurun_out/r03f/bench.err || { tail -5 gpurun_out/r03f/bench.err; exit 1; }
cut -c1-400 gpurun_out/r03f/bench.json
