# round 6: config E whole-run timeline with the merge workers' poll-done / ranks-merged stamps
# (timeline build only; the product kernel is unchanged)
set -o pipefail
T=${1:-r06aa}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('tl build E', round(d['median_s']*1e3,2), 'ms', d['codes']['success'])" gpurun_out/${T}_tl.jsonl
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_e_wg_timeline_run.json | tail -2
rm -f gpurun_out/${T}_tl.bin
