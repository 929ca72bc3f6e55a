# round 5 checkpoint: the whole GPU suite, smoke, the default bench line (configs, CPU baseline),
# a kernel trace of 20 back-to-back bench steps (kernel vs step time), the naming-layout probe
# (allocator skew fallback) and the 2-rank gloo rehearsal of the N > 1 line
set -o pipefail
T=${1:-r05o}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
REPS=1 timeout -k 10 120 python -u tools/e_parity_probe.py > gpurun_out/${T}_e_probe.txt 2>&1 && cat gpurun_out/${T}_e_probe.txt || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/${T}_smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${T}_bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_steptrace -o run --output-format csv -- python bench.py --steps 20 --warmup 10 --no-extras --no-cpu-baseline > gpurun_out/${T}_steptrace.json 2> gpurun_out/${T}_steptrace.err || { echo trace failed; tail gpurun_out/${T}_steptrace.err; exit 1; }
PROBE_LAYOUTS=cycling,iid_allocated,skew_allocated,skew_dense timeout -k 10 300 python -u tools/probe_naming.py > gpurun_out/${T}_naming.log 2>&1 || { tail gpurun_out/${T}_naming.log; exit 1; }
tail -1 gpurun_out/${T}_naming.log | cut -c1-600
MINISCHED_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-extras \
    > gpurun_out/${T}_bench2_gloo.json 2> gpurun_out/${T}_bench2_gloo.err || { echo 2-rank rehearsal failed; tail -20 gpurun_out/${T}_bench2_gloo.err; exit 1; }
echo done
