set -e
mkdir -p gpurun_out
for w in 2 4 7 8 16; do
  echo "W=$w $(MINISCHED_PP_WAVES=$w PROBE_G=8 PROBE_STREAMS=1 PROBE_COALESCE=1 timeout -k 10 120 python -u tools/step_probe_lib.py 2>>gpurun_out/r04f_w.err | tail -1)" >> gpurun_out/r04f_wsweep.txt
done
for c in 64 96 128 192 256; do
  echo "chunk=$c $(MINISCHED_PP_CHUNK=$c PROBE_G=8 PROBE_STREAMS=1 PROBE_COALESCE=1 timeout -k 10 120 python -u tools/step_probe_lib.py 2>>gpurun_out/r04f_w.err | tail -1)" >> gpurun_out/r04f_wsweep.txt
done
