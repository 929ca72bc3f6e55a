# round 5, first GPU call: the new TT ordering tests, the loopback suite, a bench line (no configs)
# with the self-verification fields, and a 2-rank gloo rehearsal of the N > 1 line
set -o pipefail
T=${1:-r05a}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_loopback.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_loopback.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_loopback.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-configs > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail gpurun_out/${T}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${T}_bench.json
MINISCHED_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-extras \
    > gpurun_out/${T}_bench2_gloo.json 2> gpurun_out/${T}_bench2_gloo.err || { echo 2-rank rehearsal failed; tail -20 gpurun_out/${T}_bench2_gloo.err; exit 1; }
cut -c1-300 gpurun_out/${T}_bench2_gloo.json
