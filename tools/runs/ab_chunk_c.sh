# config C chunk A/B for the fixed-slot form (MINISCHED_PP_CHUNK: pods per workgroup)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for c in default 200 136 104; do
    if [ $c = default ]; then v=$(timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-extras --no-cpu-baseline | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])") || exit 1
    else v=$(MINISCHED_PP_CHUNK=$c timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-extras --no-cpu-baseline | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'])") || exit 1; fi
    echo "chunk=$c ms_per_step=$v" >> gpurun_out/r04l_chunk_ab.txt
  done
done
cat gpurun_out/r04l_chunk_ab.txt
