# strong-scaling shard sweeps (tools/g8_shard_sweep.py, single launches): K1 waves x chunk grid per G
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${TAG:-r04n}_shapes.txt
run() { echo "G=$1 $2 $(env G=$1 $2 K=200 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1 | python -c 'import json,sys;print(round(json.loads(sys.stdin.read())["us_per_launch_wall"],2))')" >> $OUT; }
for G in 8 4 2; do
  run $G "X=0" || exit 1
  for w in 2 4 8; do
    for c in 24 40 56 80; do
      run $G "MINISCHED_PP_WAVES=$w MINISCHED_PP_CHUNK=$c" || exit 1
    done
  done
  run $G "X=0" || exit 1
done
cat $OUT
