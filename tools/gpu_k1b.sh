set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_par.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_par.log; [ $rc -eq 0 ] || { grep -m3 -B10 "Error\|assert" gpurun_out/pytest_par.log | head -60; exit $rc; }
GEOM_RPL=30 GEOM_CHUNK=0 GEOM_K1=v7,v7i timeout -k 10 300 python tools/k1_geom.py > gpurun_out/geom_b.jsonl 2> gpurun_out/geom_b.err || { tail gpurun_out/geom_b.err; exit 1; }
cat gpurun_out/geom_b.jsonl
