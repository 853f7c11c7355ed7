# tower dW probe: parity of mrec_tower_dw (+ big-tile GEMM) and its timing vs the
# generic 3-dW GEMM launch; out: gpurun_out/dw/
set -o pipefail
mkdir -p gpurun_out/dw
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -x -v --timeout 120 --timeout-method thread -k "tower_dw or big_tiles or weight_grad" > gpurun_out/dw/tests.txt 2>&1 || { tail -40 gpurun_out/dw/tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/dw/tests.txt | tail -8
timeout -k 10 200 python -u tools/bench_gemm.py --reps 200 --only dw3 > gpurun_out/dw/bench_gemm.txt 2>&1 || { tail -30 gpurun_out/dw/bench_gemm.txt; exit 1; }
timeout -k 10 200 python -u tools/bench_gemm.py --reps 200 --only tdw >> gpurun_out/dw/bench_gemm.txt 2>&1 || { tail -30 gpurun_out/dw/bench_gemm.txt; exit 1; }
cat gpurun_out/dw/bench_gemm.txt | grep -v amdgpu.ids
MREC_TDW_LDS=1 timeout -k 10 200 python -u tools/bench_gemm.py --reps 200 --only tdw > gpurun_out/dw/bench_gemm_nolds.txt 2>&1 || { tail -30 gpurun_out/dw/bench_gemm_nolds.txt; exit 1; }
echo "LDS-shared 128-blocks:"; grep tdw gpurun_out/dw/bench_gemm_nolds.txt
