# bench in its three single-GPU modes: plain, row-sharded (W=1), sharded with RCCL collectives forced
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/b_plain.json 2> gpurun_out/b_plain.err || { echo PLAIN_FAIL; tail -30 gpurun_out/b_plain.err; exit 1; }
cat gpurun_out/b_plain.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --shard > gpurun_out/b_shard.json 2> gpurun_out/b_shard.err || { echo SHARD_FAIL; tail -30 gpurun_out/b_shard.err; exit 1; }
cat gpurun_out/b_shard.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline --shard --force-collectives > gpurun_out/b_coll.json 2> gpurun_out/b_coll.err || { echo COLL_FAIL; tail -30 gpurun_out/b_coll.err; exit 1; }
cat gpurun_out/b_coll.json
tail -5 gpurun_out/b_coll.err
