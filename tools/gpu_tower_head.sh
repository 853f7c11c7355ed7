set -o pipefail
mkdir -p gpurun_out/tw
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_dense.py tests/test_gpu_pins.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tw/tests.txt 2>&1 || { tail -30 gpurun_out/tw/tests.txt; exit 1; }
tail -1 gpurun_out/tw/tests.txt
timeout -k 10 150 python -u tools/step_tower_stamps.py > gpurun_out/tw/step.txt 2>&1 || { tail -20 gpurun_out/tw/step.txt; exit 1; }
grep -E "start|fwd3|head dot|dh_L|parts|head:" gpurun_out/tw/step.txt
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/tw/bench$i.json 2> gpurun_out/tw/bench$i.err || { tail -30 gpurun_out/tw/bench$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/tw/bench$i.json'));print(d['ms_per_step'], d['value'])"
done
