# DIN bench under libmrec variants (bucket size / chunk per thread) -> gpurun_out/r3dv
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3dv
mkdir -p $O
for v in base b2048 b512 p4 b2048p4; do
  if [ $v = base ]; then L=pytorchrec_amd/lib/libmrec.so; else L=pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py --model din --no-cpu-baseline --no-roofline --no-h2d > $O/din_$v.json 2> $O/din_$v.err
done
echo DINVAR_OK
