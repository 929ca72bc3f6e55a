# config E batch size A/B (MINISCHED_SEQ_BATCH <= the build's 128)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for b in 128 120 112; do
    ms=$(MINISCHED_SEQ_BATCH=$b timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3))") || exit 1
    echo "B=$b E_ms=$ms" >> gpurun_out/r04za_e_batch.txt
  done
done
cat gpurun_out/r04za_e_batch.txt
