# ms_schedule_batch at config C: copies beside the cycle in 1 / 2 / 4 chunks (MINISCHED_E2E_CHUNKS)
set -o pipefail
export PYTHONUNBUFFERED=1
for k in 1 2 4 1 2 4; do
MINISCHED_E2E_CHUNKS=$k timeout -k 10 120 python -u tools/bench_configs.py --configs C --reps 9 > gpurun_out/e2e_k$k.jsonl 2>/dev/null || exit 1
echo chunks=$k $(cut -c1-330 gpurun_out/e2e_k$k.jsonl)
done
