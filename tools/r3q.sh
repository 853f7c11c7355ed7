# owner apply from wire records (ABI 23): sharded parity + W=1 compact step + kernel stats
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_mp.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline > $O/bench_shard_w1_compact.json 2> $O/shc.err
timeout -k 10 400 python bench.py --shard --force-collectives --exchange compact --rows-per-table 100000000 --no-cpu-baseline --no-roofline --no-h2d > $O/bench_c5_w1_compact.json 2> $O/c5.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_compact -o run -- python3 $R/bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/prof_compact.log 2>&1
echo OK
