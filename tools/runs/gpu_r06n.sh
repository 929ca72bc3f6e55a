# round 6: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG) for config E's 1,600 step launches
set -o pipefail
T=${1:-r06n}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
e() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms')" $1 $2; }
for i in 1 2; do
  for v in default 1 0; do
    if [ $v = default ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
    timeout -k 10 200 python tools/bench_configs.py --configs E,B --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    python -c "import json,sys; L=[json.loads(l) for l in open(sys.argv[1])]; print(sys.argv[2], {d['config']: round(d['median_s']*1e3,4) for d in L})" gpurun_out/${T}_E$v$i.jsonl kernarg_$v
  done
done
unset HIP_FORCE_DEV_KERNARG
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for v in 1 0; do
  HIP_FORCE_DEV_KERNARG=$v MS_TIMELINE=gpurun_out/${T}_tl$v.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl$v.jsonl 2> gpurun_out/${T}_tl$v.err || { tail gpurun_out/${T}_tl$v.err; exit 1; }
  python tools/e_wg_timeline.py gpurun_out/${T}_tl$v.bin gpurun_out/${T}_tl$v.json | tail -2
  rm -f gpurun_out/${T}_tl$v.bin
done
