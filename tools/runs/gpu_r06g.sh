# round 6: config E diagnostics on the current sources: whole-run step timeline (tl build) and the
# validator's phase stamps (vstamps build)
set -o pipefail
T=${1:-r06g}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E_main.jsonl 2> gpurun_out/${T}_E_main.err || { tail gpurun_out/${T}_E_main.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('main', round(d['median_s']*1e3,2), 'ms')" gpurun_out/${T}_E_main.jsonl
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_tl.json | tail -3
rm -f gpurun_out/${T}_tl.bin
MINISCHED_LIB=$L/libminisched_gpu_vstamps.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_vst.jsonl 2> gpurun_out/${T}_vst.err || { tail gpurun_out/${T}_vst.err; exit 1; }
grep MS_VSTAMPS gpurun_out/${T}_vst.err | tail -1 | cut -c1-600
