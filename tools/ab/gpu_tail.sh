#!/bin/bash
# K1 pp packed last word: parity (NU+NN paths), sweep time near word boundaries, configs C and D
set -o pipefail
TAG=${1:-r03ze}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "nunn or pp or fuzz or config_c or config_d or sharded or smoke or parity" > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
$T 240 python -u tools/probe_tail.py > gpurun_out/$TAG/tail.json 2>&1 || exit 1
tail -1 gpurun_out/$TAG/tail.json
$T 300 python -u tools/bench_configs.py --configs C,D --reps 5 > gpurun_out/$TAG/cd.jsonl 2> gpurun_out/$TAG/cd.err || exit 1
python -c "
import json
for l in open('gpurun_out/$TAG/cd.jsonl'):
    d=json.loads(l); print(d.get('config'), round(d['median_s']*1e3,4))"
