set -o pipefail
mkdir -p gpurun_out/b8
MREC_LIB_PATH=pytorchrec_amd/lib/variants/libmrec_b8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_embedding.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b8/tests.txt 2>&1 || { tail -30 gpurun_out/b8/tests.txt; exit 1; }
tail -1 gpurun_out/b8/tests.txt
for v in base b8; do
  if [ $v = base ]; then L=""; else L=pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_LIB_PATH=$L timeout -k 10 120 python -u tools/bench_plan.py > gpurun_out/b8/plan_$v.txt 2>&1 || { tail -20 gpurun_out/b8/plan_$v.txt; exit 1; }
  echo "$v $(grep plan gpurun_out/b8/plan_$v.txt)"
done
for v in base b8 base b8; do
  if [ $v = base ]; then L=""; else L=pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_LIB_PATH=$L timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/b8/bench_$v.json 2> gpurun_out/b8/bench_$v.err || { tail -30 gpurun_out/b8/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/b8/bench_$v.json'));print(d['ms_per_step'], d['value'], d['roofline']['avg_us'])")"
done
