#!/bin/bash
# Full round-end rehearsal: GPU tests, smoke, bench (+ CPU baseline), rocprof stats + PMC passes.
set -o pipefail
TAG=${1:-r01}
bash tools/gpu_check.sh ${TAG} && bash tools/profile.sh ${TAG}
