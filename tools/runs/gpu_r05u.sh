# round 5: config E in-step merge polling flags and keys in one loop (MS_MERGE_FUSEDPOLL) — parity, A/B
set -o pipefail
T=${1:-r05u}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=$PWD/mini-kube-scheduler_amd/minisched_amd
MINISCHED_LIB=$L/libminisched_gpu_fp.so REPS=1 timeout -k 10 120 python -u tools/e_parity_probe.py > gpurun_out/${T}_fp_parity.txt 2>&1 || { tail gpurun_out/${T}_fp_parity.txt; exit 1; }
cat gpurun_out/${T}_fp_parity.txt | grep n_bad
for i in 1 2 3; do
  for v in base fp; do
    lib=$L/libminisched_gpu_$v.so; [ $v = base ] && lib=$L/libminisched_gpu.so
    ms=$(MINISCHED_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3))") || exit 1
    echo "$v E_ms=$ms" | tee -a gpurun_out/${T}_e_ab.txt
  done
done
