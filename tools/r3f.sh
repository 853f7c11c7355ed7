# two-sample DIN forward: parity + C4 A/B
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
MREC_DIN_FWD_ONE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py -x -q --timeout 300 --timeout-method thread > $O/tests_one.log 2>&1
timeout -k 10 200 python bench.py --model din --no-cpu-baseline > $O/bench_din.json 2> $O/din.err
MREC_DIN_FWD_ONE=1 timeout -k 10 200 python bench.py --model din --no-cpu-baseline > $O/bench_din_one.json 2> $O/din_one.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_din -o run -- python3 $R/bench.py --model din --no-cpu-baseline --no-roofline --steps 20 > $O/prof_din.log 2>&1
echo OK
