# round 5: final bench line (bench.py with the E step split) and smoke
set -o pipefail
T=${1:-r05ar}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/${T}_smoke.log; exit 1; }
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); print({k: v.get('ms') for k, v in d['configs'].items()}); print(d['configs']['E']['roofline']['step_split'])"
