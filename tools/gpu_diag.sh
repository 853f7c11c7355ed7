# Embedding-path and tower diagnostics: apply variants (MREC_APPLY_EXP), plan phase
# stamps, tower phase stamps.  out: gpurun_out/diag/
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/diag
mkdir -p $O
V=$R/pytorchrec_amd/lib/variants
{
timeout -k 10 60 python tools/bench_apply.py || exit 1
for e in 1 2 3 4 5 6; do
  MREC_LIB_PATH=$V/libmrec_exp$e.so timeout -k 10 60 python tools/bench_apply.py || exit 1
done
timeout -k 10 60 python tools/bench_plan.py || exit 1
MREC_LIB_PATH=$V/libmrec_planprof.so timeout -k 10 60 python tools/bench_plan.py || exit 1
timeout -k 10 60 python tools/bench_tower.py || exit 1
} > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.log; exit 1; }
cat $O/diag.log
