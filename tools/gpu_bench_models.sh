# C2 / C3 / C4 bench lines (1 GPU) + the GPU test suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for m in deepfm dcnv2 din; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err || { echo BENCH_FAIL $m; tail -30 gpurun_out/bench_$m.err; exit 1; }
  cut -c1-330 gpurun_out/bench_$m.json
done
