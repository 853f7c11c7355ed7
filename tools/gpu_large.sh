# embedding GPU tests (incl. the large-batch path) and the DIN bench + profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/lg
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lg/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/lg/tests.log; exit 1; }
tail -1 gpurun_out/lg/tests.log
timeout -k 10 200 python -u bench.py --model din --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lg/din.json 2> gpurun_out/lg/din.err || { echo BENCH_FAIL; tail -30 gpurun_out/lg/din.err; exit 1; }
cut -c1-200 gpurun_out/lg/din.json
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lg/prof_din -o run --output-format csv -- python3 -u $R/bench.py --model din --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/lg/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/lg/prof.log; exit 1; }
echo ok
