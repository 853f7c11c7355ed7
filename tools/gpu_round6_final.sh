# Round-6 end measurements on the GPU box -> gpurun_out/$OUT/, in two calls (each
# fits gpurun's limit):
#   PHASE=A: the whole -m gpu suite, smoke(), then the PMC traffic passes of every
#            bench workload (tools/gpu_pmc.sh; copy gpurun_out/pmc_traffic.json to
#            profiles/ before phase B so the bench lines carry the stamp);
#   PHASE=B: plain bench lines (C2 default with cpu_baseline, C3, C4, Zipf C2,
#            row-sharded W=1 compact, C5 1-GPU) and the same lines under
#            rocprofv3 --kernel-trace --stats.
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-final6}
mkdir -p $o
cd $GRAFT_REPO_ROOT
plain() { name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $o/$name.json 2> $o/$name.err || { tail -5 $o/$name.err; exit 1; }; python3 -c "import json; d=json.load(open('$o/$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], d['value'], r.get('frac'), r.get('traffic'))"; }
prof() { name=$1; shift; (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $o/$name.json 2> $o/$name.err) || { tail -5 $o/$name.err; exit 1; }; python3 -c "import json; d=json.load(open('$o/$name.json')); print('$name', d['ms_per_step'])"; }
if [ "${PHASE:-A}" = A ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
  tail -2 $o/pytest.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
  tail -1 $o/smoke.log
  bash tools/gpu_pmc.sh > $o/pmc.log 2>&1 || { tail -20 $o/pmc.log; exit 1; }
  tail -2 $o/pmc.log
else
  plain bench_deepfm_c2 && plain bench_dcnv2_c3 --model dcnv2 --no-cpu-baseline \
    && plain bench_din_c4 --model din --no-cpu-baseline \
    && plain bench_deepfm_c2_zipf --zipf 1.05 --no-cpu-baseline --no-h2d \
    && plain bench_shard_w1_compact --shard --force-collectives --exchange compact --no-cpu-baseline --no-h2d \
    && plain bench_c5_1gpu --rows-per-table 100000000 --no-cpu-baseline --no-h2d \
    && prof prof_deepfm_c2 --no-cpu-baseline --steps 50 \
    && prof prof_dcnv2_c3 --model dcnv2 --no-cpu-baseline --no-h2d --steps 50 \
    && prof prof_din_c4 --model din --no-cpu-baseline --no-h2d --steps 50 \
    && prof prof_deepfm_c2_zipf --zipf 1.05 --no-cpu-baseline --no-h2d --steps 50 \
    && prof prof_shard_w1_compact --shard --force-collectives --exchange compact --no-cpu-baseline --no-h2d --steps 50 \
    && prof prof_c5_1gpu --rows-per-table 100000000 --no-cpu-baseline --no-h2d --steps 50
fi
