# round 5: in-step merge synchronisation variants (counter scope, poll sleep, list fences,
# fine-grained counter): parity of the fence variants, then E (instep) per variant, twice
set -o pipefail
T=${1:-r05f}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp MINISCHED_SEQ_MERGE=instep
L=$PWD/mini-kube-scheduler_amd/minisched_amd
for v in fence1 fence0; do
  MINISCHED_LIB=$L/libminisched_gpu_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "merge_forms" > gpurun_out/${T}_tests_$v.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for v in new scope1 fence1 spin0 fence0 fine; do
    lib=$L/libminisched_gpu_$v.so; fe=0
    if [ $v = new ]; then lib=$L/libminisched_gpu.so; fi
    if [ $v = fine ]; then lib=$L/libminisched_gpu.so; fe=1; fi
    ms=$(MINISCHED_CTR_FINE=$fe MINISCHED_LIB=$lib timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3))") || exit 1
    echo "$v E_ms=$ms" | tee -a gpurun_out/${T}_e_sync_ab.txt
  done
done
# K1 wave-state counters at the G = 8 shard (12.5k rows) and at G = 1 (100k rows), PAIR (coalesced) form
for g in 8 1; do
  G=$g PAIR=1 K=20 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/${T}_k1pmc_g$g -o run --output-format csv -- python tools/g8_shard_sweep.py > gpurun_out/${T}_k1pmc_g$g.json 2> gpurun_out/${T}_k1pmc_g$g.err || { echo k1 pmc g$g failed; tail gpurun_out/${T}_k1pmc_g$g.err; exit 1; }
done
echo done
