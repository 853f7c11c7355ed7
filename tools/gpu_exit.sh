# does the sharded + RCCL bench exit cleanly, directly and under torch.distributed.run?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/dp
timeout -k 10 120 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-roofline --shard --force-collectives > gpurun_out/dp/bench.json 2> gpurun_out/dp/bench.err; echo "rc=$?"
grep metric gpurun_out/dp/bench.json | cut -c1-200
timeout -k 10 120 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29577 bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-roofline --force-collectives > gpurun_out/dp/bench_tr.json 2> gpurun_out/dp/bench_tr.err; echo "rc=$?"
grep metric gpurun_out/dp/bench_tr.json | cut -c1-200
