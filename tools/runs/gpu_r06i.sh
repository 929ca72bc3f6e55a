# round 6: ranks 4..7 walked in the validator's rounds (walk_top4<true>) -- config E A/B against the
# previous kernels (libminisched_gpu_base.so), plus the merge record prefetch (pf) and the unique-high-word
# wave max (pfu); parity suites, whole-run timeline
set -o pipefail
T=${1:-r06i}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
e() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['seq_counters_all_reps'], d['codes'])" $1 $2; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/${T}_e_tests.log 2>&1 || { tail -30 gpurun_out/${T}_e_tests.log; exit 1; }
tail -1 gpurun_out/${T}_e_tests.log
for i in 1 2; do
  MINISCHED_LIB=$L/libminisched_gpu_base.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_Ebase$i.jsonl 2> gpurun_out/${T}_Ebase$i.err || { tail gpurun_out/${T}_Ebase$i.err; exit 1; }
  e gpurun_out/${T}_Ebase$i.jsonl base
  timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_Enew$i.jsonl 2> gpurun_out/${T}_Enew$i.err || { tail gpurun_out/${T}_Enew$i.err; exit 1; }
  e gpurun_out/${T}_Enew$i.jsonl new
  for v in pf pfu; do
    MINISCHED_LIB=$L/libminisched_gpu_$v.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E$v$i.jsonl 2> gpurun_out/${T}_E$v$i.err || { tail gpurun_out/${T}_E$v$i.err; exit 1; }
    e gpurun_out/${T}_E$v$i.jsonl $v
  done
done
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_tl.json | tail -1
rm -f gpurun_out/${T}_tl.bin
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_loopback.py tests/test_gpu_sharded.py -m gpu > gpurun_out/${T}_lb_tests.log 2>&1 || { tail -30 gpurun_out/${T}_lb_tests.log; exit 1; }
tail -1 gpurun_out/${T}_lb_tests.log
