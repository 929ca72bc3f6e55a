# round 5: balanced K1 shard split (MINISCHED_PP_BALANCE) — sharded parity, step probe A/B at G = 2/4/8
set -o pipefail
T=${1:-r05s}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "shard or loopback or pp or nunn" > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 1 0 1 0; do
  MINISCHED_PP_BALANCE=$b PROBE_G=2,4,8 PROBE_STREAMS=1 timeout -k 10 300 python -u tools/step_probe_lib.py > gpurun_out/${T}_probe_b$b.jsonl 2>> gpurun_out/${T}_probe.err || { tail gpurun_out/${T}_probe.err; exit 1; }
  echo "balance=$b $(tail -1 gpurun_out/${T}_probe_b$b.jsonl)" | tee -a gpurun_out/${T}_balance_ab.txt
done
