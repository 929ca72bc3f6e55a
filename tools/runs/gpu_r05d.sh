# round 5: where the in-step merge path's time goes (MS_VSTAMPS build, per-workgroup timeline of
# steps 200-215, instep vs launch)
set -o pipefail
T=${1:-r05d}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for v in instep launch; do
  MS_TIMELINE=gpurun_out/${T}_tl_$v.bin MINISCHED_SEQ_MERGE=$v MINISCHED_LIB=$L/libminisched_gpu_vstamps.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_vst_$v.jsonl 2> gpurun_out/${T}_vst_$v.err || { tail gpurun_out/${T}_vst_$v.err; exit 1; }
  python tools/e_wg_timeline.py gpurun_out/${T}_tl_$v.bin gpurun_out/${T}_tl_$v.json | tail -4
done
