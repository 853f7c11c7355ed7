# exploratory: kernel profile of the sharded + DP step at world 1 (RCCL collectives forced)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/x
export TMPDIR=/tmp
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/x/prof_shard_rccl -o run --output-format csv -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --shard --force-collectives --no-graph > $R/gpurun_out/x/prof_shard_rccl.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/x/prof_shard_rccl.log; exit 1; }
tail -1 $R/gpurun_out/x/prof_shard_rccl.log | cut -c1-200
cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/x/prof_din -o run --output-format csv -- python3 -u $R/bench.py --model din --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/x/prof_din.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/x/prof_din.log; exit 1; }
tail -1 $R/gpurun_out/x/prof_din.log | cut -c1-200
echo ok
