# C5-sized sharded test + the rest of the sharded GPU tests -> gpurun_out/r3c5
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1
echo C5TEST_OK
