set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_check.sh r01b && AB_VARIANTS=bits32,bits32l,bits64,lazy AB_ROUNDS=10 timeout -k 10 120 python tools/ab_k1.py > gpurun_out/ab_r01b.json 2>gpurun_out/ab_r01b.err && cat gpurun_out/ab_r01b.json
