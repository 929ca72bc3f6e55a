# round 5 closing: whole GPU suite, smoke, bench; then a NodeAffinity timing probe
# (k_nam_keys without the later segments' table composition, timing only: slower, 9.96 vs 9.52 ms -- composed tables die sooner and skip work; the probe switch was not kept)
set -o pipefail
bash tools/gpu_r05ad.sh r05aw || exit 1
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for v in main namprobe; do
  if [ $v = main ]; then LIB=$L/libminisched_gpu.so; else LIB=$L/libminisched_gpu_$v.so; fi
  MINISCHED_LIB=$LIB timeout -k 10 200 python tools/bench_nam.py --reps 5 > gpurun_out/r05aw_nam_$v.json 2> gpurun_out/r05aw_nam_$v.err || { tail gpurun_out/r05aw_nam_$v.err; exit 1; }
  echo $v $(tail -1 gpurun_out/r05aw_nam_$v.json | cut -c1-60)
done
