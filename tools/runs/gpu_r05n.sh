# config E parity under warm-up batches / merge forms (the r05m full-size failure)
set -o pipefail
T=${1:-r05n}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "8192:64 instep" "0:0 instep" "8192:64 launch" "8192:64 fallback" "4096:64 instep" "8192:32 instep"; do
  set -- $cfg
  MINISCHED_SEQ_WARM=$1 MINISCHED_SEQ_MERGE=$2 timeout -k 10 120 python -u tools/e_parity_probe.py >> gpurun_out/${T}_probe.txt 2>&1 || { tail gpurun_out/${T}_probe.txt; exit 1; }
done
cat gpurun_out/${T}_probe.txt
