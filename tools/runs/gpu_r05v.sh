# round 5: host-copy helper threads for single-shard host-array calls (MINISCHED_COPY_THREADS) — parity, e2e A/B
set -o pipefail
T=${1:-r05v}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "compact or zc or chunk or host or e2e or batch" > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for t in 3 0 7; do
    MINISCHED_COPY_THREADS=$t timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline > gpurun_out/${T}_b$t.json 2>/dev/null || exit 1
    python - "$t" gpurun_out/${T}_b$t.json <<'PY' | tee -a gpurun_out/${T}_e2e_ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c, e = d["e2e_compact"], d["e2e"]
print(f"threads={sys.argv[1]} compact_ms={c['ms_median']:.4f} runs={[round(x,4) for x in c['runs']]} "
      f"stage_in={[p['stage_in'] for p in c['phases_us']]} stage_out={[p['stage_out'] for p in c['phases_us']]} "
      f"rec40_ms={e['ms_median']:.4f} step_ms={d['ms_per_step']:.4f}")
PY
  done
done
