# large-batch backward tests, DIN tests, DIN bench (fused and pair paths) + kernel stats -> gpurun_out/r3d
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_embedding.py tests/test_gpu_din.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
timeout -k 10 200 python bench.py --model din --no-cpu-baseline > $O/bench_din.json 2> $O/din.err
MREC_LARGE_FUSED=0 timeout -k 10 200 python bench.py --model din --no-cpu-baseline --no-roofline --no-h2d > $O/bench_din_pair.json 2> $O/din_pair.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/din -o run -- python3 $R/bench.py --model din --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/din.log 2>&1
echo DIN_OK
