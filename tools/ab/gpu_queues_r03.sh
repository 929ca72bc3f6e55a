#!/bin/bash
# Which hardware queues do the library's two sweep streams land on, and does
# the overlap appear? step_probe_lib at G = 8, 4 under: default; high-priority
# sweep streams; GPU_MAX_HW_QUEUES=8. Then one kernel trace per variant.
set -o pipefail
mkdir -p gpurun_out/queues_r03
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for V in def prio q8; do
  case $V in
    def) P=0; Q=4 ;;
    prio) P=1; Q=4 ;;
    q8) P=0; Q=8 ;;
  esac
  MINISCHED_SWEEP_PRIO=$P GPU_MAX_HW_QUEUES=$Q PROBE_G=8,4 PROBE_STREAMS=2,1 timeout -k 10 120 python -u tools/step_probe_lib.py > gpurun_out/queues_r03/$V.json 2>&1 || { tail -3 gpurun_out/queues_r03/$V.json; exit 1; }
  echo "$V $(tail -n 1 gpurun_out/queues_r03/$V.json)"
done
for V in prio q8; do
  case $V in
    prio) P=1; Q=4 ;;
    q8) P=0; Q=8 ;;
  esac
  MINISCHED_SWEEP_PRIO=$P GPU_MAX_HW_QUEUES=$Q PROBE_G=8 PROBE_STREAMS=2 PROBE_STEPS=20 timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/queues_r03/prof_$V -o run --output-format csv -- python tools/step_probe_lib.py > /dev/null 2>&1 || { echo trace $V failed; exit 1; }
  python3 - $V <<'PY'
import csv, sys, collections
v = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/queues_r03/prof_{v}/run_kernel_trace.csv")))
q = collections.Counter((r["Queue_Id"], "sweep" if "sweep" in r["Kernel_Name"] else r["Kernel_Name"][:24]) for r in rows)
print(v, dict(q))
PY
done
