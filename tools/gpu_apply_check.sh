set -o pipefail
mkdir -p gpurun_out/tw
timeout -k 10 300 python -u -m pytest tests/test_gpu_embedding.py tests/test_gpu_optim.py tests/test_gpu_sharded.py tests/test_gpu_pins.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tw/tests.txt 2>&1 || { tail -30 gpurun_out/tw/tests.txt; exit 1; }
tail -1 gpurun_out/tw/tests.txt
true
true
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/tw/bench$i.json 2> gpurun_out/tw/bench$i.err || { tail -30 gpurun_out/tw/bench$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/tw/bench$i.json'));print(d['ms_per_step'], d['value'])"
done
