# K1 pp: 4 vs 8 30-row words per lane (MINISCHED_PP_WORDS), with pods-per-workgroup variants
set -o pipefail
export PYTHONUNBUFFERED=1
run() {  # nodes base pods mode variants
  AB_MODE=$4 AB_NODES=$1 AB_NODE_BASE=$2 AB_PODS=$3 AB_ROUNDS=8 AB_VARIANTS="$5" timeout -k 10 200 python -u tools/ab_pp.py || exit 1
}
run 100000 0 100000 select "k4:X=1;k8:MINISCHED_PP_WORDS=8;k8c392:MINISCHED_PP_WORDS=8,MINISCHED_PP_CHUNK=392;k8c104:MINISCHED_PP_WORDS=8,MINISCHED_PP_CHUNK=104"
run 12500 87500 800000 sweep "k4:X=1;k8:MINISCHED_PP_WORDS=8"
run 25000 75000 400000 sweep "k4:X=1;k8:MINISCHED_PP_WORDS=8"
run 50000 50000 1000000 select "k4:X=1;k8:MINISCHED_PP_WORDS=8"
