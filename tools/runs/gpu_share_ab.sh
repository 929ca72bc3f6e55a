# K1 shared last word (MINISCHED_PP_SHARE, default on) vs off: full GPU suite, then
# single-launch shard sweeps (G = 8 / 16, and the coalesced pair) and the pipelined step at G = 8 / 4 / 2
set -o pipefail
T=${TAG:-r04zm}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_gpu_tests.log | head -20; exit $rc; }
O=gpurun_out/${T}_share_ab.txt
for i in 1 2; do
  for sh in 1 0; do
    echo "share=$sh G8 $(MINISCHED_PP_SHARE=$sh G=8 K=200 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1)" >> $O || exit 1
    echo "share=$sh G8pair $(MINISCHED_PP_SHARE=$sh PAIR=1 G=8 K=100 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1)" >> $O || exit 1
    echo "share=$sh step $(MINISCHED_PP_SHARE=$sh PROBE_G=8,4,2 PROBE_STREAMS=1 timeout -k 10 200 python tools/step_probe_lib.py 2>/dev/null | tail -1)" >> $O || exit 1
  done
done
cat $O
