# pp sweep geometry at the weak-scaling shard sizes (rows N/G, pods G x 100k): waves per workgroup
set -o pipefail
export PYTHONUNBUFFERED=1
for cfg in "12500 87500 800000" "50000 50000 200000"; do
  set -- $cfg
  AB_MODE=sweep AB_NODES=$1 AB_NODE_BASE=$2 AB_PODS=$3 AB_ROUNDS=6 \
  AB_VARIANTS="w1:MINISCHED_PP_WAVES=1;w2:MINISCHED_PP_WAVES=2;w4:MINISCHED_PP_WAVES=4;w8:MINISCHED_PP_WAVES=8;w16:MINISCHED_PP_WAVES=16;def:X=1" \
  timeout -k 10 200 python -u tools/ab_pp.py || exit 1
done
