# config E: MS_TP_UNROLL variants of the transposed sweep (tools/build_variants.sh tpu1/tpu4/tpu8) vs default (2)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for i in 1 2; do
  for v in default tpu1 tpu4 tpu8; do
    if [ $v = default ]; then lib=$L/libminisched_gpu.so; else lib=$L/libminisched_gpu_$v.so; fi
    ms=$(MINISCHED_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;print(round(json.loads(sys.stdin.read())['median_s']*1e3,3))") || exit 1
    echo "$v E_ms=$ms" >> gpurun_out/r04s_e_unroll.txt
  done
done
cat gpurun_out/r04s_e_unroll.txt
