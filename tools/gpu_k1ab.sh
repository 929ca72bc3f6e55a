#!/bin/bash
# K1 variant parity + interleaved A/B (one GPU call)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-k1ab}
if [ -x tools/ubench/valu_rates ]; then timeout -k 10 60 tools/ubench/valu_rates > gpurun_out/valu_rates.txt 2>&1 && cat gpurun_out/valu_rates.txt || exit 1; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${TAG}.log
[ $rc -eq 0 ] || { echo "parity failed rc=$rc"; grep -m5 -B5 "Error\|assert" gpurun_out/pytest_${TAG}.log; exit $rc; }
AB_VARIANTS=${AB_VARIANTS:-v7,v0} AB_ROUNDS=10 timeout -k 10 180 python tools/ab_k1.py \
    > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err || { echo ab failed; tail gpurun_out/ab_${TAG}.err; exit 1; }
cat gpurun_out/ab_${TAG}.json
