# full GPU suite + E timing + bench (one call)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r02k}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --configs B,C,D,E --reps 5 > gpurun_out/${TAG}_configs.jsonl 2> gpurun_out/${TAG}_configs.err || exit 1
cat gpurun_out/${TAG}_configs.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'], d['median_s'], d.get('evals_per_s'))"
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
