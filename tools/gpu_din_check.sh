set -o pipefail
mkdir -p gpurun_out/din
timeout -k 10 300 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_pins.py tests/test_gpu_embedding.py -x -q --timeout 120 --timeout-method thread > gpurun_out/din/tests.txt 2>&1 || { tail -30 gpurun_out/din/tests.txt; exit 1; }
tail -1 gpurun_out/din/tests.txt
timeout -k 10 200 python -u bench.py --model din --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/din/bench.json 2> gpurun_out/din/bench.err || { tail -30 gpurun_out/din/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/din/bench.json'));print('din', d['ms_per_step'], d['value'])"
