#!/bin/bash
# r03h: config E with the sweep-merged top-4 (default) vs a merge launch per batch;
# K1 pt (pod per lane) parity + A/B against pp at config C and at the G=8 shard;
# then the round-end rehearsal (tools/gpu_round.sh).
set -o pipefail
mkdir -p gpurun_out/r03h
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "resource or sequential or config_e" > gpurun_out/r03h/e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03h/e_tests.log; [ $rc -eq 0 ] || exit $rc
$T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/r03h/e_sweepmerge.jsonl 2> gpurun_out/r03h/e1.err || exit 1
MINISCHED_SEQ_MERGE=launch $T 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/r03h/e_launch.jsonl 2> gpurun_out/r03h/e2.err || exit 1
cut -c1-300 gpurun_out/r03h/e_sweepmerge.jsonl gpurun_out/r03h/e_launch.jsonl
MINISCHED_K1_FORM=pt $T 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h/pt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03h/pt_tests.log; [ $rc -eq 0 ] || exit $rc
for f in pp pt; do MINISCHED_K1_FORM=$f $T 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/r03h/bench_$f.json 2> gpurun_out/r03h/bench_$f.err || exit 1; cut -c1-250 gpurun_out/r03h/bench_$f.json; done
for f in pp pt; do MINISCHED_K1_FORM=$f PROBE_G=8,4,2 PROBE_STREAMS=1 PROBE_STEPS=50 $T 150 python -u tools/step_probe_lib.py > gpurun_out/r03h/step_$f.json 2>&1 || exit 1; tail -n 1 gpurun_out/r03h/step_$f.json; done
bash tools/gpu_round.sh r03h
