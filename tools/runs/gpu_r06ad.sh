# round 6 diagnostic (wrong results by design): the validator's write-back phase with the derived-row (the MS_DIAG_WB_SKIP switch it builds with was removed after the run; patch: git show 29227c1)
# stores (vsk1) or the table-column stores (vsk2) left out, against the full write-back (vstamps);
# validator phase stamps, and the timeline build without derived-row stores (tlsk1)
set -o pipefail
T=${1:-r06ad}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for v in vstamps vsk1 vsk2; do
  MINISCHED_LIB=$L/libminisched_gpu_$v.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_$v.jsonl 2> gpurun_out/${T}_$v.err || { tail gpurun_out/${T}_$v.err; exit 1; }
  echo "$v: $(grep MS_VSTAMPS gpurun_out/${T}_$v.err | tail -1 | sed -E 's/.*(epilogue parts: [^|]*).*/\1/')"
done
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tlsk1.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_e_wg_timeline_run.json | tail -2
rm -f gpurun_out/${T}_tl.bin
