export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01_end_gpu_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01_end_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r01_end_bench.json 2> gpurun_out/r01_end_bench.err
