set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_embedding.py tests/test_gpu_sharded.py -x -q > gpurun_out/emb_tests.log 2>&1 || { echo EMB_FAIL; tail -40 gpurun_out/emb_tests.log; exit 1; }
tail -1 gpurun_out/emb_tests.log
for a in "4096 38462" "4096 3" "4096 50" "4096 1000000" "4096 38462 zipf" "4096 1000000 zipf" "8192 38462"; do
  timeout -k 10 60 python tools/bench_plan.py $a || exit 1
done

bash tools/gpu_round.sh
