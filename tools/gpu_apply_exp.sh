# apply microbenchmark: product library + MREC_APPLY_EXP variants (tools/build_variant.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 python tools/bench_apply.py || exit 1
for e in ${APPLY_EXPS:-7 8 9}; do
  MREC_LIB_PATH=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants/libmrec_exp$e.so timeout -k 10 60 python tools/bench_apply.py || exit 1
done
