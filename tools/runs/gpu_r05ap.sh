# round 5: config E rocprof passes on the final kernels (stats + PMC + vstamps) -> profiles/r05ap_*
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/profile_e.sh r05ap && ls gpurun_out/prof_e_r05ap
