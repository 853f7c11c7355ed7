# C2 bench line + C3/C4 lines + rocprof kernel stats of the C2 bench (out: gpurun_out/bench/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/bench
mkdir -p $O
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -30 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
for m in dcnv2 din; do
  timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_$m.json 2> $O/bench_$m.err || { echo BENCH_FAIL $m; tail -30 $O/bench_$m.err; exit 1; }
  cut -c1-200 $O/bench_$m.json
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-h2d > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
cd $R && python tools/kstats.py $O/prof/run_kernel_stats.csv | head -16
