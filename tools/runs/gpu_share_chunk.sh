# K1 at G = 8: the shared last word (MINISCHED_PP_SHARE) at chunk 104 (two waves per SIMD), single batch and pair
set -o pipefail
T=${TAG:-r04zo}
mkdir -p gpurun_out
O=gpurun_out/${T}_share_chunk.txt
for i in 1 2 3; do
  for sh in 1 0; do
    echo "share=$sh chunk=104 single $(MINISCHED_PP_SHARE=$sh MINISCHED_PP_CHUNK=104 G=8 K=200 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1)" >> $O || exit 1
    echo "share=$sh chunk=default single $(MINISCHED_PP_SHARE=$sh G=8 K=200 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1)" >> $O || exit 1
    echo "share=$sh pair $(MINISCHED_PP_SHARE=$sh PAIR=1 G=8 K=100 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1)" >> $O || exit 1
  done
done
cat $O
