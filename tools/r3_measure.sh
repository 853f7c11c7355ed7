# Round-3 measurements: full GPU suite, bench lines, rocprof kernel stats -> gpurun_out/r3m
# (copied into profiles/r03/ by hand)
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3m3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_deepfm_c2.json 2> $O/bench_deepfm_c2.err
timeout -k 10 200 python bench.py --zipf 1.05 --no-cpu-baseline --no-h2d > $O/bench_deepfm_c2_zipf.json 2> $O/zipf.err
timeout -k 10 200 python bench.py --table-dtype fp32 --no-cpu-baseline --no-h2d > $O/bench_deepfm_c2_fp32.json 2> $O/fp32.err
timeout -k 10 200 python bench.py --model dcnv2 --no-cpu-baseline > $O/bench_dcnv2_c3.json 2> $O/dcn.err
timeout -k 10 200 python bench.py --model din --no-cpu-baseline > $O/bench_din_c4.json 2> $O/din.err
timeout -k 10 200 python bench.py --shard --force-collectives --exchange slot --no-cpu-baseline --no-roofline > $O/bench_shard_w1_slot.json 2> $O/shs.err
timeout -k 10 200 python bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline > $O/bench_shard_w1_compact.json 2> $O/shc.err
timeout -k 10 400 python bench.py --shard --force-collectives --exchange compact --rows-per-table 100000000 --no-cpu-baseline --no-roofline --no-h2d > $O/bench_c5_w1_compact.json 2> $O/c5.err
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv"
$P -d $O/prof_c2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-h2d --steps 20 > $O/prof_c2.log 2>&1
$P -d $O/prof_din -o run -- python3 $R/bench.py --model din --no-cpu-baseline --no-h2d --steps 20 > $O/prof_din.log 2>&1
$P -d $O/prof_zipf -o run -- python3 $R/bench.py --zipf 1.05 --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/prof_zipf.log 2>&1
$P -d $O/prof_compact -o run -- python3 $R/bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/prof_compact.log 2>&1
echo MEASURE_OK
