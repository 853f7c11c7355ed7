set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3t
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3t/tower.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_dense.py tests/test_gpu_din.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3t/more.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r3t/bench.json 2> gpurun_out/r3t/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3t/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-h2d --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/r3t/prof.log 2>&1
