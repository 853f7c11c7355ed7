set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3s
timeout -k 10 900 python -u -m pytest ${PYFILES:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3s/gputest.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/r3s/bench.json 2> gpurun_out/r3s/bench.err
