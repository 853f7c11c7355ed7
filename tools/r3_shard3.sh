# sharded + large-batch GPU tests, compact W=1 profile, DIN bench -> gpurun_out/r3s3
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3s3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_embedding.py tests/test_gpu_din.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
timeout -k 10 200 python bench.py --model din --no-cpu-baseline --no-h2d > $O/din.json 2> $O/din.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/compact -o run -- python3 $R/bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/compact.log 2>&1
echo SHARD3_OK
