# full GPU suite + configs + bench + 2-rank gloo rehearsal of the (weak-scaling) multi-GPU bench
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r02n}
mkdir -p gpurun_out
bash tools/gpu_full.sh ${TAG} || exit 1
MINISCHED_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 \
    > gpurun_out/${TAG}_bench2_gloo.json 2> gpurun_out/${TAG}_bench2_gloo.err || { echo 2-rank rehearsal failed; tail -20 gpurun_out/${TAG}_bench2_gloo.err; exit 1; }
cat gpurun_out/${TAG}_bench2_gloo.json
