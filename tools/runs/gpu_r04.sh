#!/bin/bash
# round-4 rehearsal: tools/gpu_round.sh (GPU suite, smoke, configs B-E, bench + CPU baseline, rocprof stats +
# PMC of K1 pp, weak probe, 2-rank gloo), config E profile, strong-scaling per-rank probe
set -o pipefail
TAG=${1:-r04}
bash tools/gpu_round.sh $TAG || exit $?
bash tools/profile_e.sh $TAG > gpurun_out/${TAG}_profile_e.log 2>&1 || { echo profile_e failed; tail gpurun_out/${TAG}_profile_e.log; exit 1; }
PROBE_G=8,4,2 PROBE_STREAMS=1 PROBE_STEPS=100 timeout -k 10 150 python -u tools/step_probe_lib.py > gpurun_out/${TAG}_step_probe.json 2> gpurun_out/${TAG}_step_probe.err || exit 1
tail -n 1 gpurun_out/${TAG}_step_probe.json
