set -o pipefail
mkdir -p gpurun_out/sp
bash tools/gpu_apply_check.sh || exit 1
timeout -k 10 120 python -u tools/bench_interact.py | grep interact
for s in 2 4 8 2 4 8; do
  MREC_TDW_SPLITS=$s timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/sp/b$s.json 2> gpurun_out/sp/b$s.err || { tail -30 gpurun_out/sp/b$s.err; exit 1; }
  echo "splits=$s $(python -c "import json;d=json.load(open('gpurun_out/sp/b$s.json'));print(d['ms_per_step'], d['value'])")"
done
