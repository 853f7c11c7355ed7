# sharded W=1 compact bench lines with variant libraries (tools/build_variant.py): in-step times
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/svar; mkdir -p $o; cd $GRAFT_REPO_ROOT
for v in product ${VARIANTS}; do
  lib=""; [ $v != product ] && lib=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants/$v/libmrec.so
  MREC_BENCH_DIAG_NOCHECK=1 MREC_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-h2d --steps 50 > $o/$v.json 2> $o/$v.err || { echo FAIL $v; tail -3 $o/$v.err; continue; }
  python3 -c "import json; d=json.load(open('$o/$v.json')); print('$v', d['ms_per_step'], json.dumps({k: v['avg_us'] for k, v in d['roofline_kernels'].items() if 'bucketize' in k}))"
done
