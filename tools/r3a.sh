# round-3 re-entry check: GPU suite, C2 + C4 bench lines, tower L2-warm experiment
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 200 python bench.py --model din --no-cpu-baseline > $O/bench_din.json 2> $O/din.err
MREC_TOWER_WARM=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d > $O/bench_c2_warm.json 2> $O/warm.err
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv"
$P -d $O/prof_c2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-h2d --no-roofline --steps 20 > $O/prof_c2.log 2>&1
MREC_TOWER_WARM=1 $P -d $O/prof_warm -o run -- python3 $R/bench.py --no-cpu-baseline --no-h2d --no-roofline --steps 20 > $O/prof_warm.log 2>&1
echo OK
