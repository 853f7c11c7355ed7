# Round-5 check on the GPU box: the round's new GPU tests, then C2 / C3 / C4 bench lines
# under rocprofv3 --kernel-trace --stats (kernel summaries) -> gpurun_out/$OUT/
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r5d}
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests/test_gpu_embedding.py tests/test_gpu_sharded.py tests/test_gpu_sharded_mp.py tests/test_loader.py tests/test_gpu_din.py tests/test_gpu_tower.py -k "${TESTK:-plan_body or checkpoint or two_process or large_batch_default or graph_epochs or pipelined or din or cross}" -v --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
run() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$name -o run -- python3 bench.py --no-cpu-baseline "$@" > $o/$name.json 2> $o/$name.err || { tail -5 $o/$name.err; exit 1; }; python3 -c "import json; d=json.load(open('$o/$name.json')); print('$name', d['ms_per_step'], d.get('pcie_inclusive', {}).get('ms_per_step'))"; }
run c2 && run c3 --model dcnv2 && run c4 --model din
