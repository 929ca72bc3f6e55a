# config E: merge kernel variants (MINISCHED_LIB=...mergeold.so vs the tree's build) + merge kernel time
set -o pipefail
mkdir -p gpurun_out
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for i in 1 2; do
  for v in mergeold new; do
    if [ $v = new ]; then lib=$L/libminisched_gpu.so; else lib=$L/libminisched_gpu_$v.so; fi
    ms=$(MINISCHED_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3))") || exit 1
    echo "$v E_ms=$ms" >> gpurun_out/${TAG:-r04zd}_e_merge.txt
  done
done
cat gpurun_out/${TAG:-r04zd}_e_merge.txt
