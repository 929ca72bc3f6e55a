# round 5: config E validator phases: the timeline build (per-step stamps) and the
# MS_VSTAMPS build (per-phase cycle totals, printed at context teardown)
set -o pipefail
T=${1:-r05af}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$PWD/mini-kube-scheduler_amd/minisched_amd
#MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
#python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_tl.json | tail -1
MINISCHED_LIB=$L/libminisched_gpu_vstamps.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_vst.jsonl 2> gpurun_out/${T}_vst.err || { tail gpurun_out/${T}_vst.err; exit 1; }
grep MS_VSTAMPS gpurun_out/${T}_vst.err
