set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/bench_gemm.py --only fwd && timeout -k 10 100 python tools/bench_gemm.py --only dx
for nb in 4 6 8; do
  echo "== NBUF $nb"
  MREC_LIB_PATH=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants/libmrec_nb$nb.so timeout -k 10 100 python tools/bench_gemm.py --only fwd || exit 1
  MREC_LIB_PATH=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants/libmrec_nb$nb.so timeout -k 10 100 python tools/bench_gemm.py --only dx || exit 1
done
