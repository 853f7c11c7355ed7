export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_loader.py tests/test_cli.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01_loader_gpu2.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r01_bench_final2.json 2> gpurun_out/r01_bench_final2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python bench.py --no-cpu-baseline --no-h2d > gpurun_out/prof_final.log 2>&1
