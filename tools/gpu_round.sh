# smoke, all GPU tests (one process), C2 bench, C3/C4 bench lines, rocprof kernel stats of the C2 bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/round
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/round/smoke.log; exit 1; }
tail -1 gpurun_out/round/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/round/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/round/gpu_tests.log; exit 1; }
tail -1 gpurun_out/round/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/round/bench.json 2> gpurun_out/round/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/round/bench.err; exit 1; }
cut -c1-240 gpurun_out/round/bench.json
for m in dcnv2 din; do
  timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/round/bench_$m.json 2> gpurun_out/round/bench_$m.err || { echo BENCH_FAIL $m; tail -30 gpurun_out/round/bench_$m.err; exit 1; }
  cut -c1-200 gpurun_out/round/bench_$m.json
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/round/prof -o run --output-format csv -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/round/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/round/prof.log; exit 1; }
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/round/prof_dcn -o run --output-format csv -- python3 -u $R/bench.py --model dcnv2 --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/round/prof_dcn.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/round/prof_dcn.log; exit 1; }
echo ok
