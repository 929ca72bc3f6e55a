set -o pipefail
mkdir -p gpurun_out
GEOM_REPS=10 GEOM_PODS=50000,100000,200000,400000 GEOM_SHARDS=100000,12500 GEOM_RPL=30 GEOM_CHUNK=0 GEOM_WAVES=4 timeout -k 10 300 python tools/k1_geom.py > gpurun_out/geom3.jsonl 2> gpurun_out/geom3.err || { tail gpurun_out/geom3.err; exit 1; }
cat gpurun_out/geom3.jsonl
