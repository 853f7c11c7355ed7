set -o pipefail
mkdir -p gpurun_out/plan
timeout -k 10 300 python -u -m pytest tests/test_gpu_embedding.py tests/test_gpu_sharded.py tests/test_gpu_optim.py -x -q --timeout 120 --timeout-method thread > gpurun_out/plan/tests.txt 2>&1 || { tail -30 gpurun_out/plan/tests.txt; exit 1; }
tail -1 gpurun_out/plan/tests.txt
bash tools/gpu_plan_prof.sh || exit 1
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/plan/bench$i.json 2> gpurun_out/plan/bench$i.err || { tail -30 gpurun_out/plan/bench$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/plan/bench$i.json'));print(d['ms_per_step'], d['value'], d['roofline']['avg_us'], d['roofline']['frac'])"
done
