# config D (50k rows x 1M pods) and C with MINISCHED_PP_CHUNK=56 vs default
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for c in default 56 112; do
    for cfg in D C; do
      if [ $c = default ]; then e="X=0"; else e="MINISCHED_PP_CHUNK=$c"; fi
      v=$(env $e timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --no-extras --no-cpu-baseline | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])") || exit 1
      echo "config=$cfg chunk=$c ms_per_step=$v" >> gpurun_out/r04o_d_chunk.txt
    done
  done
done
cat gpurun_out/r04o_d_chunk.txt
