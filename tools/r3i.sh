# tower phase stamps inside the C2 step and standalone (PF 4 / 6 / 8)
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3i
mkdir -p $O
timeout -k 10 120 python tools/step_tower_stamps.py > $O/step_stamps.txt 2>&1
timeout -k 10 120 python tools/bench_tower.py > $O/bench_tower.txt 2>&1
MREC_TOWER_PF=6 timeout -k 10 120 python tools/bench_tower.py > $O/bench_tower_pf6.txt 2>&1
MREC_TOWER_PF=8 timeout -k 10 120 python tools/bench_tower.py > $O/bench_tower_pf8.txt 2>&1
echo OK
