# Zipf C2 (truncated Zipf ids) bench + kernel stats -> gpurun_out/r3z
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3z
mkdir -p $O
timeout -k 10 200 python bench.py --zipf 1.05 --no-cpu-baseline --no-h2d > $O/bench_zipf.json 2> $O/zipf.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/zipf -o run -- python3 $R/bench.py --zipf 1.05 --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/zipf.log 2>&1
echo ZIPF_OK
