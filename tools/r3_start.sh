set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3s
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3s/gputest.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/r3s/bench.json 2> gpurun_out/r3s/bench.err
