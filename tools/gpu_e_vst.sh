set -o pipefail
for pipe in 1 2; do
MINISCHED_SEQ_PIPE=$pipe MINISCHED_LIB=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_vstamps.so timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 1 > gpurun_out/e_vst_$pipe.jsonl 2>gpurun_out/e_vst_$pipe.err || exit 1
echo pipe=$pipe; grep MS_VSTAMPS gpurun_out/e_vst_$pipe.err
done
