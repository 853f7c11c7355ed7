# full GPU suite, then the C2 bench with the tower weight gradients by mrec_tower_dw
# (default) vs the generic GEMM launch (MREC_TOWER_DW=0), interleaved
set -o pipefail
bash tools/gpu_tests.sh || exit 1
mkdir -p gpurun_out/ab
for v in 1 0 1 0 1 0; do
  MREC_TOWER_DW=$v timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > gpurun_out/ab/tdw$v.json 2> gpurun_out/ab/tdw$v.err || { tail -30 gpurun_out/ab/tdw$v.err; exit 1; }
  echo "tower_dw=$v $(python -c "import json;d=json.load(open('gpurun_out/ab/tdw$v.json'));print(d['ms_per_step'], d['value'])")"
done
