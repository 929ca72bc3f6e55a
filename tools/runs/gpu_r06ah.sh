# round 6 closing rehearsal (r06ah): the full GPU suite, smoke, the default bench line (driver shape)
set -o pipefail
T=${1:-r06ah}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['device_ms_per_step'], d['roofline']['kernel_ms']); print({k: v.get('ms') for k, v in d['configs'].items()}); print(d['configs'].get('C_names'))"
python -c "import json; d=json.loads(open(\"gpurun_out/${T}_bench.json\").read().strip().splitlines()[-1]); print(json.dumps(d[\"roofline\"])[:400]); print(json.dumps(d[\"configs\"][\"E\"])[:900])"
