# C2 uniform + Zipf + DCN-v2 under plan-bucket variants -> gpurun_out/r3pv
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3pv
mkdir -p $O
for v in base pb4 pb5; do
  if [ $v = base ]; then L=pytorchrec_amd/lib/libmrec.so; else L=pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d > $O/c2_$v.json 2> $O/c2_$v.err
  MREC_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py --zipf 1.05 --no-cpu-baseline --no-h2d > $O/zipf_$v.json 2> $O/zipf_$v.err
done
MREC_LIB_PATH=$PWD/pytorchrec_amd/lib/variants/libmrec_pb4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_embedding.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > $O/test_pb4.log 2>&1
echo PLANVAR_OK
