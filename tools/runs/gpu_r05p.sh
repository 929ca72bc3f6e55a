# round 5: bit-sliced two-pass TaintToleration (census / plan / pick / final) — parity, A/B vs the
# per-pair summary sweep (MINISCHED_TT=v1), kernel trace of the TT config
set -o pipefail
T=${1:-r05p}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
true
for v in v2 v1 v2 v1; do
  ms=$(MINISCHED_TT=$v timeout -k 10 200 python tools/bench_tt.py --reps 5 2>/dev/null | tail -1) || exit 1
  echo "$v TT_ms=$ms" | tee -a gpurun_out/${T}_tt_ab.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ttprof -o run --output-format csv -- python tools/bench_tt.py --reps 3 > gpurun_out/${T}_ttprof.jsonl 2> gpurun_out/${T}_ttprof.err || { tail gpurun_out/${T}_ttprof.err; exit 1; }
cut -c1-160 gpurun_out/${T}_ttprof/run_kernel_stats.csv | head -8
