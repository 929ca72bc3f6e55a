# host-array calls (bench.py e2e / e2e_compact): zero-copy pipeline parts 1 / 2 / 3 for 100k pods
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for p in 1 2 3; do
    v=$(MINISCHED_ZC_PARTS=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['e2e_compact']['ms_median'],4), round(d['e2e']['ms_median'],4))") || exit 1
    echo "parts=$p e2e_compact/e2e ms: $v" >> gpurun_out/r04zb_zc_parts.txt
  done
done
cat gpurun_out/r04zb_zc_parts.txt
