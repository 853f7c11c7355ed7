# DIN (C4) bench + rocprof kernel stats; out: gpurun_out/din/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/din
mkdir -p $O
cd $R
timeout -k 10 200 python -u bench.py --model din --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u $R/bench.py --model din --steps 20 --warmup 5 --no-cpu-baseline --no-h2d > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof.log; exit 1; }
cd $R && python tools/kstats.py $O/prof/run_kernel_stats.csv | head -30
