#!/bin/bash
# cross-stream hand-off latency: event, event(release-to-device), wait-value
set -o pipefail
mkdir -p gpurun_out/xs
export TMPDIR=/tmp
for m in 0 1 2 3; do
  timeout -k 10 60 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/xs/m$m -o run -- ./tools/ubench/xstream $m > gpurun_out/xs/m$m.log 2>&1 || { echo mode $m failed; tail -3 gpurun_out/xs/m$m.log; exit 1; }
  echo "mode $m:"; python3 tools/ubench/xstream.py gpurun_out/xs/m$m/run_kernel_trace.csv
done
