# round 5: NodeAffinity kernel trace on the final kernels (rocprofv3 --kernel-trace --stats)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/prof_nam_r05ax
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nam_r05ax -o run --output-format csv -- python tools/bench_nam.py --reps 3 > gpurun_out/prof_nam_r05ax/bench.json 2> gpurun_out/prof_nam_r05ax/err.txt || { tail gpurun_out/prof_nam_r05ax/err.txt; exit 1; }
find gpurun_out/prof_nam_r05ax -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r05ax_nam_kernel_stats.csv
cut -d, -f1-4 gpurun_out/r05ax_nam_kernel_stats.csv | head -8
