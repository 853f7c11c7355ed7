# all GPU tests, one process, then smoke
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${MREC_TESTS:-} > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
