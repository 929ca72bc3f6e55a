# round 6: the 8-wave / CU-sized-tile step as the default: GPU suite, timeline, E
set -o pipefail
T=${1:-r06r}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E.jsonl 2> gpurun_out/${T}_E.err || { tail gpurun_out/${T}_E.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('E', round(d['median_s']*1e3,2), 'ms')" gpurun_out/${T}_E.jsonl
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_e_wg_timeline_run.json | tail -2
rm -f gpurun_out/${T}_tl.bin
