# config E: depth-2 fused pipeline at smaller batches vs depth 1 at 128
set -o pipefail
mkdir -p gpurun_out
for cfg in "fused2 64" "fused2 96" "fused 128" "fused2 80"; do
  set -- $cfg
  ms=$(MINISCHED_SEQ_PIPE=$1 MINISCHED_SEQ_BATCH=$2 timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3), d['seq_counters_all_reps'])") || exit 1
  echo "$1 B=$2 E_ms=$ms" >> gpurun_out/r04w_e_fused2_b.txt
done
cat gpurun_out/r04w_e_fused2_b.txt
