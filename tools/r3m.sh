# wire kernels: elements per thread 2 / 4 / 8 (W=1 compact step, kernel stats)
set -e
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3m
V=$R/pytorchrec_amd/lib/variants
mkdir -p $O
MREC_LIB_PATH=$V/libmrec_wp8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread > $O/tests_wp8.log 2>&1
cd /tmp && export TMPDIR=/tmp
for v in wp2 wp4 wp8; do
  if [ $v = wp2 ]; then L=""; else L="MREC_LIB_PATH=$V/libmrec_$v.so"; fi
  env $L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 $R/bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-roofline --no-h2d --steps 20 > $O/prof_$v.log 2>&1
done
echo OK
