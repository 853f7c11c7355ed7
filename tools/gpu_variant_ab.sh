# A/B bench lines of the product library against variant libraries built by
# tools/build_variant.py: VARIANTS="name ..." ARGS="bench args" -> in-step kernel times
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/vab; mkdir -p $o; cd $GRAFT_REPO_ROOT
for v in product ${VARIANTS}; do
  lib=""; [ $v != product ] && lib=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants/$v/libmrec.so
  MREC_LIB_PATH=$lib timeout -k 10 300 python3 bench.py ${ARGS} --no-cpu-baseline --no-h2d > $o/$v.json 2> $o/$v.err || { tail -5 $o/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/$v.json')); print('$v', d['ms_per_step'], json.dumps({k: v['avg_us'] for k, v in d['roofline_kernels'].items() if 'avg_us' in v}))"
done
