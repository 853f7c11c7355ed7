# N > 1 rehearsal on a one-GPU box: two processes over gloo on cuda:0
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_mp.py -x -v --timeout 300 --timeout-method thread > $O/mp_test.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --same-gpu --dist-backend gloo --rows-per-table 1000000 --steps 10 --warmup 3 --no-roofline > $O/bench_rehearsal_n2.json 2> $O/rehearsal.err
echo OK
