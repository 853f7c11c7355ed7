# hash-plan cost: phase clocks and the lut stores' share (diagnostic variants)
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3k
V=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants
mkdir -p $O
for r in 1 2; do
timeout -k 10 120 python tools/bench_plan.py > $O/plan_$r.txt 2>&1
MREC_LIB_PATH=$V/libmrec_nolut.so timeout -k 10 120 python tools/bench_plan.py > $O/plan_nolut_$r.txt 2>&1
timeout -k 10 120 python tools/bench_interact.py > $O/interact_$r.txt 2>&1
MREC_LIB_PATH=$V/libmrec_nolut.so timeout -k 10 120 python tools/bench_interact.py > $O/interact_nolut_$r.txt 2>&1
done
MREC_LIB_PATH=$V/libmrec_pprof.so timeout -k 10 120 python tools/bench_plan.py > $O/plan_prof.txt 2>&1
echo OK
