# round 5: in-step merge on tagged lists (default) vs the counter (ctr): the sequential suite,
# E A/B (+ warm-up batches), timeline of the tagged form
set -o pipefail
T=${1:-r05l}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sequential or config_e or resource or seq or merge" > gpurun_out/${T}_e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_e_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new ctr; do
    for w in 0:0 8192:64; do
      lib=$L/libminisched_gpu_$v.so; [ $v = new ] && lib=$L/libminisched_gpu.so
      ms=$(MINISCHED_SEQ_WARM=$w MINISCHED_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3))") || exit 1
      echo "$v warm=$w E_ms=$ms" | tee -a gpurun_out/${T}_e_ab.txt
    done
  done
done
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_tl.json | tail -1
