set -o pipefail
export PYTHONUNBUFFERED=1
for pg in 0 1 0 1; do  # MINISCHED_PAGEABLE: 0 pinned staging, 1 direct (default)
MINISCHED_PAGEABLE=$pg timeout -k 10 120 python -u tools/bench_configs.py --configs C --reps 9 > gpurun_out/e2e_pg$pg.jsonl 2>/dev/null || exit 1
echo pageable=$pg $(cut -c1-330 gpurun_out/e2e_pg$pg.jsonl)
done
