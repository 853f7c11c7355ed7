set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3p
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py -m gpu -x -q --timeout 120 --timeout-method thread -k cluster > gpurun_out/r3p/tower.log 2>&1
MREC_TOWER_CL_SC1=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py -m gpu -x -q --timeout 120 --timeout-method thread -k cluster > gpurun_out/r3p/tower_sc1.log 2>&1
timeout -k 10 120 python tools/bench_tower.py > gpurun_out/r3p/cl.txt 2>&1
MREC_TOWER_CL_SC1=1 timeout -k 10 120 python tools/bench_tower.py > gpurun_out/r3p/cl_sc1.txt 2>&1
MREC_TOWER_CL_DIAG=2 timeout -k 10 120 python tools/bench_tower.py > gpurun_out/r3p/cl_d2.txt 2>&1
