# DIN forward A/B (r3f) + PMC traffic restamp + C5-sized N=2 rehearsal (gloo, one GPU)
set -e
cd $GRAFT_REPO_ROOT
bash tools/r3f.sh
bash tools/gpu_pmc.sh > $GRAFT_REPO_ROOT/gpurun_out/pmc_summary.txt 2>&1
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3g
mkdir -p $O
timeout -k 10 600 python bench.py --gpus 2 --same-gpu --dist-backend gloo --steps 5 --warmup 2 --no-roofline > $O/bench_c5_rehearsal_n2.json 2> $O/c5_rehearsal.err
echo OK
