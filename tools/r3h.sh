# kernel sequence of the row-sharded step at world 1 (compact exchange, RCCL forced)
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_compact -o run -- python3 $R/bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline --no-h2d --steps 4 --warmup 2 --graph-steps 1 > $O/trace_compact.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-roofline --no-h2d --steps 4 --warmup 2 --graph-steps 1 > $O/trace_c2.log 2>&1
echo OK
