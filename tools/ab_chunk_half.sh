# K1 pp: pods per workgroup for one resident workgroup per CU ("half": 16 waves per CU) vs the default two
set -o pipefail
export PYTHONUNBUFFERED=1
run() {  # nodes base pods mode variants
  AB_MODE=$4 AB_NODES=$1 AB_NODE_BASE=$2 AB_PODS=$3 AB_ROUNDS=8 AB_VARIANTS="$5" timeout -k 10 200 python -u tools/ab_pp.py || exit 1
}
run 100000 0 100000 select "def:X=1;c392:MINISCHED_PP_CHUNK=392;c400:MINISCHED_PP_CHUNK=400"
run 50000 50000 1000000 select "def:X=1;c1960:MINISCHED_PP_CHUNK=1960"
run 50000 50000 200000 sweep "def:X=1;c392:MINISCHED_PP_CHUNK=392"
run 25000 75000 400000 sweep "def:X=1;c392:MINISCHED_PP_CHUNK=392"
run 12500 87500 800000 sweep "def:X=1;c784:MINISCHED_PP_CHUNK=784"
