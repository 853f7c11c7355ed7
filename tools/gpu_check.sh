# GEMM numerics + microbench first, then the round script.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_dense.py -x -q > gpurun_out/dense_tests.log 2>&1 || { echo DENSE_FAIL; tail -40 gpurun_out/dense_tests.log; exit 1; }
tail -1 gpurun_out/dense_tests.log
timeout -k 10 200 python tools/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || { echo GEMMBENCH_FAIL; tail -20 gpurun_out/bench_gemm.log; exit 1; }
cat gpurun_out/bench_gemm.log
bash tools/gpu_round.sh
