# round 5: config E rocprof passes on the final kernels (sweep unrolled twice) -> profiles/r05bc_*
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/profile_e.sh r05bc && ls gpurun_out/prof_e_r05bc
