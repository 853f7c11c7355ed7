# GPU tests touched by the apply / reduce changes, then C2 uniform + Zipf under
# hot-segment variants, DIN -> gpurun_out/r3hv
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3hv
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_embedding.py tests/test_gpu_sharded.py tests/test_gpu_optim.py tests/test_gpu_tower.py tests/test_gpu_dense.py tests/test_gpu_din.py tests/test_gpu_pins.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1
for v in base hp2 hp8; do
  if [ $v = base ]; then L=pytorchrec_amd/lib/libmrec.so; else L=pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py --zipf 1.05 --no-cpu-baseline --no-h2d > $O/zipf_$v.json 2> $O/zipf_$v.err
  MREC_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d > $O/c2_$v.json 2> $O/c2_$v.err
done
timeout -k 10 200 python bench.py --model din --no-cpu-baseline --no-h2d > $O/din.json 2> $O/din.err
echo HOTVAR_OK
