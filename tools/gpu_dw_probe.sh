set -o pipefail
mkdir -p gpurun_out/dw
timeout -k 10 200 python -u -m pytest tests/test_gpu_g9.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dw/g9.txt 2>&1 || { tail -30 gpurun_out/dw/g9.txt; exit 1; }
tail -5 gpurun_out/dw/g9.txt
timeout -k 10 200 python -u tools/bench_gemm.py --reps 200 > gpurun_out/dw/bench_gemm.txt 2>&1 || { tail -30 gpurun_out/dw/bench_gemm.txt; exit 1; }
cat gpurun_out/dw/bench_gemm.txt
