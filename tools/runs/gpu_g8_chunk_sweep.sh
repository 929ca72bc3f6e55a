# G = 8 shard: K1 chunk sizes (MINISCHED_PP_CHUNK) for the single batch and the coalesced pair,
# against the wave-per-SIMD quantisation model (tools: DESIGN §5)
set -o pipefail
T=${TAG:-r04zn}
mkdir -p gpurun_out
O=gpurun_out/${T}_g8_chunks.txt
for i in 1 2; do
  for c in default 40 48 56 64 80 96 104; do
    if [ $c = default ]; then E="X=1"; else E="MINISCHED_PP_CHUNK=$c"; fi
    echo "chunk=$c single $(env $E G=8 K=200 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1)" >> $O || exit 1
    echo "chunk=$c pair $(env $E PAIR=1 G=8 K=100 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1)" >> $O || exit 1
  done
done
cat $O
