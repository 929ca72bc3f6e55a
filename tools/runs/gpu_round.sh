# Round-end rehearsal: full GPU suite, smoke, configs B-E, bench (+CPU baseline), rocprof stats + PMC of the
# timed kernel, weak-scaling per-rank probe and a 2-rank gloo rehearsal of the N > 1 bench path.
set -o pipefail
TAG=${1:-r02t}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py --configs B,C,D,E --reps 5 > gpurun_out/${TAG}_configs.jsonl 2> gpurun_out/${TAG}_configs.err || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cut -c1-400 gpurun_out/${TAG}_bench.json
timeout -k 10 200 python -u tools/weak_probe.py > gpurun_out/${TAG}_weak_probe.json 2> gpurun_out/${TAG}_weak_probe.err || exit 1
cat gpurun_out/${TAG}_weak_probe.json
bash tools/profile_pp.sh ${TAG} > gpurun_out/${TAG}_profile.log 2>&1 || { echo profile failed; tail gpurun_out/${TAG}_profile.log; exit 1; }
MINISCHED_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 \
    > gpurun_out/${TAG}_bench2_gloo.json 2> gpurun_out/${TAG}_bench2_gloo.err || { echo 2-rank rehearsal failed; tail -20 gpurun_out/${TAG}_bench2_gloo.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench2_gloo.json
