set -o pipefail
mkdir -p gpurun_out/blk4
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_dense.py tests/test_gpu_pins.py tests/test_gpu_optim.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/blk4/tests.txt 2>&1 || { tail -30 gpurun_out/blk4/tests.txt; exit 1; }
tail -1 gpurun_out/blk4/tests.txt
for v in base noblk4 base noblk4; do
  if [ $v = base ]; then L=""; else L=pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_LIB_PATH=$L timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/blk4/bench_$v.json 2> gpurun_out/blk4/bench_$v.err || { tail -30 gpurun_out/blk4/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/blk4/bench_$v.json'));print(d['ms_per_step'], d['value'], d['roofline']['avg_us'])")"
done
