# round 5: host-array chunk count (MINISCHED_ZC_PARTS 1/2/3) now that the host copies run on the copy pool
set -o pipefail
T=${1:-r05y}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for p in 2 1 3; do
    MINISCHED_ZC_PARTS=$p timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline > gpurun_out/${T}_p$p.json 2>/dev/null || exit 1
    python - "$p" gpurun_out/${T}_p$p.json <<'PY' | tee -a gpurun_out/${T}_parts_ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c, e = d["e2e_compact"], d["e2e"]
print(f"parts={sys.argv[1]} compact_ms={c['ms_median']:.4f} rec40_ms={e['ms_median']:.4f} step_ms={d['ms_per_step']:.4f} "
      f"wait={[p['wait'] for p in c['phases_us']]}")
PY
  done
done
