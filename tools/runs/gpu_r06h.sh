# round 6: config E at 192-pod batches (MS_SEQ_BATCH=192 build) against the 128 default, its
# whole-run timeline, and full-size E parity through the 192 build
set -o pipefail
T=r06h
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=$PWD/mini-kube-scheduler_amd/minisched_amd
e() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['median_s']*1e3,2), 'ms', d['seq_counters_all_reps'])" $1 $2; }
timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E128.jsonl 2> gpurun_out/${T}_E128.err || { tail gpurun_out/${T}_E128.err; exit 1; }
e gpurun_out/${T}_E128.jsonl b128
MINISCHED_LIB=$L/libminisched_gpu_b192.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E192.jsonl 2> gpurun_out/${T}_E192.err || { tail gpurun_out/${T}_E192.err; exit 1; }
e gpurun_out/${T}_E192.jsonl b192
MINISCHED_SEQ_BATCH=128 MINISCHED_LIB=$L/libminisched_gpu_b192.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 > gpurun_out/${T}_E192at128.jsonl 2> gpurun_out/${T}_E192at128.err || { tail gpurun_out/${T}_E192at128.err; exit 1; }
e gpurun_out/${T}_E192at128.jsonl b192_at128
MS_TIMELINE=gpurun_out/${T}_tl.bin MINISCHED_LIB=$L/libminisched_gpu_tl192.so timeout -k 10 200 python tools/bench_configs.py --configs E --reps 1 > gpurun_out/${T}_tl.jsonl 2> gpurun_out/${T}_tl.err || { tail gpurun_out/${T}_tl.err; exit 1; }
python tools/e_wg_timeline.py gpurun_out/${T}_tl.bin gpurun_out/${T}_tl.json | tail -3
rm -f gpurun_out/${T}_tl.bin
MINISCHED_LIB=$L/libminisched_gpu_b192.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -k "config_e" > gpurun_out/${T}_e192_tests.log 2>&1 || { tail -30 gpurun_out/${T}_e192_tests.log; exit 1; }
tail -2 gpurun_out/${T}_e192_tests.log
# instruction-fetch counters of config E (k_seq_step's code is ~180 KB): which exist here, then one pass
timeout -k 10 120 rocprofv3 -L > gpurun_out/${T}_counters_avail.txt 2>&1 || echo "list failed"
W=""
for c in SQ_WAVES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_BUSY_CYCLES; do
  grep -q "\b$c\b" gpurun_out/${T}_counters_avail.txt && W="$W $c"
done
echo "icache counters:$W"
if [ -n "$W" ]; then
  timeout -s KILL 200 rocprofv3 --pmc $W -d gpurun_out/${T}_ic -o run --output-format csv -- python tools/bench_configs.py --configs E --reps 1 > /dev/null 2> gpurun_out/${T}_ic.err || { echo ic pass failed; tail -5 gpurun_out/${T}_ic.err; exit 1; }
  python - gpurun_out/${T}_ic <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "seq_step" in k or "sweep_full" in k:
        print(k, {c: round(v / max(1, n[(k, c)]), 1) for c, v in d.items()})
PY
fi
