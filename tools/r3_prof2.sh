# Kernel stats of the sharded step (slot / compact exchange at W=1), Zipf C2, and the
# C5-sized sharded bank at W=1 -> gpurun_out/r3p2
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3p2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv"
$P -d $O/compact -o run -- python3 $R/bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/compact.log 2>&1
$P -d $O/slot -o run -- python3 $R/bench.py --shard --force-collectives --exchange slot --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/slot.log 2>&1
$P -d $O/zipf -o run -- python3 $R/bench.py --zipf 1.05 --no-cpu-baseline --no-h2d --steps 20 > $O/zipf.log 2>&1
timeout -k 10 400 python3 $R/bench.py --shard --force-collectives --exchange compact --rows-per-table 100000000 --no-cpu-baseline --no-roofline --no-h2d > $O/bench_c5_w1_compact.json 2> $O/c5.err
echo PROF2_OK
