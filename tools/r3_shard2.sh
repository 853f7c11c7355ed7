# sharded GPU tests + compact / slot W=1 kernel stats -> gpurun_out/r3s2
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3s2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/compact -o run -- python3 $R/bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/compact.log 2>&1
echo SHARD2_OK
