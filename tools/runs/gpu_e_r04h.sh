set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resource or config_e or chunked or commit or sequential or cursor" > gpurun_out/r04h_e_tests.log 2>&1 || { tail -30 gpurun_out/r04h_e_tests.log; exit 1; }
tail -2 gpurun_out/r04h_e_tests.log
timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 5 > gpurun_out/r04h_e.jsonl 2> gpurun_out/r04h_e.err || exit 1
cut -c1-300 gpurun_out/r04h_e.jsonl
bash tools/profile_e.sh r04h
