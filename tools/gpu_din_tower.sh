# score-tower (DIN attention unit) checks + DIN bench with the tower on / off
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/dt
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_din.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAIL; tail -50 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 python -u bench.py --model din --steps 30 --warmup 5 --no-cpu-baseline > $O/on.json 2> $O/on.err || { echo BENCH_FAIL; tail -30 $O/on.err; exit 1; }
cut -c1-220 $O/on.json
MREC_DIN_TOWER=0 timeout -k 10 200 python -u bench.py --model din --steps 30 --warmup 5 --no-cpu-baseline > $O/off.json 2> $O/off.err || { echo BENCH_FAIL off; tail -30 $O/off.err; exit 1; }
cut -c1-220 $O/off.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 -u $R/bench.py --model din --steps 10 --warmup 3 --no-cpu-baseline > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
cd $R && python tools/prof_summary.py $O/prof/run_kernel_stats.csv 22
