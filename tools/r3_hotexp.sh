# Zipf C2 apply-kernel time with the hot segments / all segment blocks skipped -> gpurun_out/r3he
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3he
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in base exp10 exp8; do
  if [ $v = base ]; then L=$R/pytorchrec_amd/lib/libmrec.so; else L=$R/pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_LIB_PATH=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/bench.py --zipf 1.05 --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/$v.log 2>&1
done
echo HOTEXP_OK
