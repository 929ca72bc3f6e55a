# round 6: NAM per-class pipeline + general terms: its GPU suite, then the bench (all configs)
set -o pipefail
T=${1:-r06d}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nam.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_nam_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${T}_nam_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step']); print({k: (v.get('ms'), v.get('parity_vs_oracle_prefix', v.get('parity_vs_oracle'))) for k, v in d['configs'].items()})"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_namprof -o run --output-format csv -- python tools/bench_nam.py > gpurun_out/${T}_namprof.log 2>&1 || { tail gpurun_out/${T}_namprof.log; exit 1; }
