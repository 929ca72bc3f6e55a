# round 5: config E warm-up batch sweep (MINISCHED_SEQ_WARM=<pods>:<batch>) on the current kernels
set -o pipefail
T=${1:-r05an}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for w in 8192:64 0:0 4096:64 16384:64 8192:32 8192:64; do
  MINISCHED_SEQ_WARM=$w timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E_$w.jsonl 2> gpurun_out/${T}_E_$w.err || { tail gpurun_out/${T}_E_$w.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['codes'])" gpurun_out/${T}_E_$w.jsonl $w
done
