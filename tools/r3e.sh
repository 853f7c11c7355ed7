# tower_dw on a side stream (MREC_DW_SIDE=1): parity + C2 A/B + kernel timeline
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3e
mkdir -p $O
MREC_DW_SIDE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_dense.py tests/test_gpu_pins.py tests/test_gpu_g9.py -x -q --timeout 300 --timeout-method thread > $O/tests_side.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d > $O/bench_c2.json 2> $O/c2.err
MREC_DW_SIDE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d > $O/bench_c2_side.json 2> $O/c2s.err
timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d > $O/bench_c2_b.json 2> $O/c2b.err
MREC_DW_SIDE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d > $O/bench_c2_side_b.json 2> $O/c2sb.err
cd /tmp && export TMPDIR=/tmp
MREC_DW_SIDE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_side -o run -- python3 $R/bench.py --no-cpu-baseline --no-h2d --no-roofline --steps 20 > $O/prof_side.log 2>&1
echo OK
