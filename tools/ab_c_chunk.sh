# K1 pp fused cycle at config C (100k x 100k): pods per workgroup around the one-round default
set -o pipefail
export PYTHONUNBUFFERED=1
AB_MODE=select AB_NODES=100000 AB_PODS=100000 AB_ROUNDS=8 \
AB_VARIANTS="def:X=1;c104:MINISCHED_PP_CHUNK=104;c136:MINISCHED_PP_CHUNK=136;c264:MINISCHED_PP_CHUNK=264;c392:MINISCHED_PP_CHUNK=392;w8:MINISCHED_PP_WAVES=8" \
timeout -k 10 200 python -u tools/ab_pp.py
