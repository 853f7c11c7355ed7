# GPU test suite, then the sharded + data-parallel path at world 1 with RCCL
# collectives forced: bench (graphs) and a kernel profile (eager: rocprofv3 +
# graph capture of the sharded step hangs on this image)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/dp
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dp/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/dp/tests.log; exit 1; }
tail -1 gpurun_out/dp/tests.log
timeout -k 10 200 python -u bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-roofline --shard --force-collectives > gpurun_out/dp/bench.json 2> gpurun_out/dp/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/dp/bench.err; exit 1; }
grep metric gpurun_out/dp/bench.json | cut -c1-200
timeout -k 10 200 python -u bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-roofline > gpurun_out/dp/bench_c2.json 2> gpurun_out/dp/bench_c2.err || { echo BENCH_FAIL; tail -30 gpurun_out/dp/bench_c2.err; exit 1; }
grep metric gpurun_out/dp/bench_c2.json | cut -c1-200
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dp/prof -o run --output-format csv -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --shard --force-collectives --no-graph > $R/gpurun_out/dp/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/dp/prof.log; exit 1; }
echo ok
