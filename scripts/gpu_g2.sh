set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -m gpu -k "conv or gemm or ip or alexnet or C3" > gpurun_out/g2/tests.txt 2>&1 || { tail -30 gpurun_out/g2/tests.txt; exit 1; }
tail -3 gpurun_out/g2/tests.txt
for v in 3 2 0; do RRAM_GEMM_V2=$v timeout -k 10 200 python scripts/kbench.py --only gemm > gpurun_out/g2/kb_$v.txt 2>&1 || exit 1; done
for v in 3 0; do RRAM_GEMM_V2=$v timeout -k 10 200 python bench.py --no-cpu-baseline --profile-layers > gpurun_out/g2/b_$v.json 2> gpurun_out/g2/b_$v.err || exit 1; done
