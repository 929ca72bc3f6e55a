# round 5: config E step timeline with the validator's phases (prologue / decisions / write-back)
set -o pipefail
T=${1:-r05ae}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$PWD/mini-kube-scheduler_amd/minisched_amd
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_tl.json | tail -1
