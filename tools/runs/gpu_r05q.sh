# round 5: the strong-scaling per-rank step (tools/step_probe_lib.py) at G = 1/2/4/8 on the current
# tree, and a kernel trace of the G = 8 probe
set -o pipefail
T=${1:-r05q}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PROBE_G=1,2,4,8 PROBE_STREAMS=2 PROBE_REPEAT=2 timeout -k 10 300 python -u tools/step_probe_lib.py > gpurun_out/${T}_step_probe.jsonl 2> gpurun_out/${T}_step_probe.err || { tail gpurun_out/${T}_step_probe.err; exit 1; }
tail -1 gpurun_out/${T}_step_probe.jsonl
PROBE_G=8 PROBE_STREAMS=2 PROBE_STEPS=100 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_g8trace -o run --output-format csv -- python tools/step_probe_lib.py > gpurun_out/${T}_g8trace.json 2> gpurun_out/${T}_g8trace.err || { tail gpurun_out/${T}_g8trace.err; exit 1; }
cut -c1-150 gpurun_out/${T}_g8trace/run_kernel_stats.csv | head -8
