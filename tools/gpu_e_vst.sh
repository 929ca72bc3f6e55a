# config E wave stamps (MS_VSTAMPS build): validator vs sweep wave durations per step
set -o pipefail
TAG=${1:-r02zf}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MINISCHED_LIB=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_vstamps.so timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 1 > gpurun_out/${TAG}_e_vst.jsonl 2> gpurun_out/${TAG}_e_vst.err || exit 1
grep MS_VSTAMPS gpurun_out/${TAG}_e_vst.err
