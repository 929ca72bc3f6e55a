# round 6: config E profiles on the closing step kernel (sorted merge, one-allocation table): bench roofline + step_split sources
set -o pipefail
T=${1:-r06ag}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
bash tools/profile_e.sh $T > gpurun_out/${T}_pe.log 2>&1 || { tail -20 gpurun_out/${T}_pe.log; exit 1; }
tail -3 gpurun_out/${T}_pe.log
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('tl build E', round(d['median_s']*1e3,2), 'ms')" gpurun_out/${T}_tl.jsonl
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_e_wg_timeline_run.json | tail -2
rm -f gpurun_out/${T}_tl.bin
