# bench.py with every collective issued at world 1 (RCCL captured in HIP graphs)
# must exit through destroy_process_group: timed, under its own limit
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exit
t0=$(date +%s.%N)
timeout -k 10 180 python -u bench.py --force-collectives --steps 20 --warmup 5 --no-cpu-baseline --no-h2d > gpurun_out/exit/bench_force.json 2> gpurun_out/exit/bench_force.err
rc=$?
t1=$(date +%s.%N)
echo "force-collectives bench rc=$rc wall=$(python -c "print(round($t1-$t0,1))")s"
grep -v amdgpu.ids gpurun_out/exit/bench_force.err | tail -5
cut -c1-300 gpurun_out/exit/bench_force.json
exit $rc
