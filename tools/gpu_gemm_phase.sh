set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_dense.py -x -q > gpurun_out/dense_tests.log 2>&1 || { echo DENSE_FAIL; tail -40 gpurun_out/dense_tests.log; exit 1; }
tail -1 gpurun_out/dense_tests.log
timeout -k 10 100 python tools/bench_gemm.py --only fwd || exit 1
timeout -k 10 100 python tools/bench_gemm.py --only dx || exit 1
V=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants/libmrec_gemmprof.so
MREC_LIB_PATH=$V timeout -k 10 100 python tools/bench_gemm.py --only fwd --prof || exit 1
MREC_LIB_PATH=$V timeout -k 10 100 python tools/bench_gemm.py --only dx --prof || exit 1
