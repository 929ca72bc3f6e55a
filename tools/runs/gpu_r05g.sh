# round 5: per-workgroup timeline of config-E steps 200-215 from the MS_TIMELINE_ONLY build (plain
# timestamp stores, none of the stamped build's contended counters), instep vs launch merge
set -o pipefail
T=${1:-r05g}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for v in instep launch; do
  MS_TIMELINE=gpurun_out/${T}_tl_$v.bin MINISCHED_SEQ_MERGE=$v MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl_$v.jsonl 2> gpurun_out/${T}_tl_$v.err || { tail gpurun_out/${T}_tl_$v.err; exit 1; }
  python tools/e_wg_timeline.py gpurun_out/${T}_tl_$v.bin gpurun_out/${T}_tl_$v.json | tail -6
  tail -1 gpurun_out/${T}_tl_$v.jsonl | cut -c1-200
done
