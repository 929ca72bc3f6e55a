# G=8 shard sweep (tools/g8_shard_sweep.py, single launches) across K1 shapes, fixed-slot form
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { echo "$1 $(env $2 K=200 timeout -k 10 120 python tools/g8_shard_sweep.py | tail -1)" >> gpurun_out/r04m_g8_forms.txt; }
for i in 1 2; do
  run default "X=1" || exit 1
  run waves2 "MINISCHED_PP_WAVES=2" || exit 1
  run words8 "MINISCHED_PP_WORDS=8" || exit 1
  run chunk56 "MINISCHED_PP_CHUNK=56" || exit 1
  run fix0 "MINISCHED_PP_FIX=0" || exit 1
done
cat gpurun_out/r04m_g8_forms.txt
