export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/r6d; mkdir -p $o; cd $GRAFT_REPO_ROOT
for v in 0 1; do
  MREC_SHARD_UNPACK=$v timeout -k 10 300 python3 bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-h2d > $o/shard_unpack$v.json 2> $o/shard_unpack$v.err || exit 1
  python3 -c "import json; d=json.load(open('$o/shard_unpack$v.json')); print('unpack=$v', d['ms_per_step'], d['roofline']['collectives_us'], json.dumps({k: v['avg_us'] for k, v in d['roofline_kernels'].items()}))"
done
