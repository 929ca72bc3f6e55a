# interleaved E timing of the default library and an A/B build (MINISCHED_LIB), 3 alternations
set -o pipefail
A=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu.so
B=$PWD/mini-kube-scheduler_amd/minisched_amd/${1:-libminisched_gpu_ab.so}
for it in 1 2 3; do
  for L in $A $B; do
    echo -n "$(basename $L): "
    MINISCHED_LIB=$L timeout -k 10 120 python -u tools/bench_configs.py --configs E --reps 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['median_s'], d['codes']['success'])" || exit 1
  done
done
