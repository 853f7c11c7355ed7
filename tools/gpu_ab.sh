# A/B of bench.py (step time) between the product library and variants, in ONE
# call (boxes differ by several %): VARIANTS="head exp8 ..." (pytorchrec_amd/lib/variants)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in prod ${VARIANTS:-head}; do
    if [ $v = prod ]; then L=; else L=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants/libmrec_$v.so; fi
    MREC_ABI_ANY=1 MREC_LIB_PATH=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-h2d ${BENCH_ARGS:-} > gpurun_out/ab/$v.$rep.json 2> gpurun_out/ab/$v.$rep.err || { echo FAIL $v; tail -5 gpurun_out/ab/$v.$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.$rep.json')); r=d.get('roofline_kernels',{}); print('$v', d['ms_per_step'], {k: v['avg_us'] for k, v in r.items()})"
  done
done
