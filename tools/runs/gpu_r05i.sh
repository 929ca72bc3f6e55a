# round 5: config E sweep-phase timeline (tile staged / tasks done) + merge wave-max variant A/B
set -o pipefail
T=${1:-r05i}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_tl.json | tail -3
for i in 1 2; do
  for v in new mu; do
    lib=$L/libminisched_gpu_$v.so; [ $v = new ] && lib=$L/libminisched_gpu.so
    ms=$(MINISCHED_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3))") || exit 1
    echo "$v E_ms=$ms" | tee -a gpurun_out/${T}_e_ab.txt
  done
done
