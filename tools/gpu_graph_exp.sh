set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --graph-steps 1 --no-roofline --no-cpu-baseline > gpurun_out/g1.json 2>gpurun_out/g1.err || { tail gpurun_out/g1.err; exit 1; }
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --graph-steps 4 --no-roofline --no-cpu-baseline > gpurun_out/g4.json 2>gpurun_out/g4.err || { tail gpurun_out/g4.err; exit 1; }
DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --graph-steps 4 --no-roofline --no-cpu-baseline > gpurun_out/g4q2.json 2>gpurun_out/g4q2.err || { tail gpurun_out/g4q2.err; exit 1; }
for f in g1 g4 g4q2; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f', d['value'], d['ms_per_step'])"; done
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profq2 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $R/gpurun_out/profq2.log 2>&1 || { tail -20 $R/gpurun_out/profq2.log; exit 1; }
