export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_loader.py tests/test_abi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01_loader_gpu3.log 2>&1 && \
timeout -k 10 200 python tools/h2d_probe.py > gpurun_out/h2d_probe4.json 2> gpurun_out/h2d_probe4.err && \
timeout -k 10 300 python bench.py > gpurun_out/r01_bench_final3.json 2> gpurun_out/r01_bench_final3.err
