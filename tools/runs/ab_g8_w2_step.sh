# G = 8 pipelined step (coalesced submits): MINISCHED_PP_WAVES=2 vs the default geometry
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  echo "default $(PROBE_G=8 PROBE_STREAMS=1 timeout -k 10 120 python tools/step_probe_lib.py 2>/dev/null | tail -1)" >> gpurun_out/r04t_g8_w2.txt || exit 1
  echo "waves2 $(MINISCHED_PP_WAVES=2 PROBE_G=8 PROBE_STREAMS=1 timeout -k 10 120 python tools/step_probe_lib.py 2>/dev/null | tail -1)" >> gpurun_out/r04t_g8_w2.txt || exit 1
done
cat gpurun_out/r04t_g8_w2.txt
