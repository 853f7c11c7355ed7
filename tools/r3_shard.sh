set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3p
timeout -k 10 120 python tools/bench_tower.py > gpurun_out/r3p/cl.txt 2>&1
timeout -k 10 120 python tools/bench_tower.py --no-cluster > gpurun_out/r3p/old.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3p/shard.log 2>&1
