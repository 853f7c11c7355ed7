# tower preload A/B (variants named in the loops): parity + C2 step + standalone
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3n
V=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_pins.py tests/test_gpu_g9.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for v in hpre0 hpre2 hpre4; do
    if [ $v = hpre2 ]; then L=""; else L="MREC_LIB_PATH=$V/libmrec_$v.so"; fi
    env $L timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d --no-roofline > $O/bench_${v}_$r.json 2> $O/${v}_$r.err
  done
done
for v in hpre0 hpre2 hpre4; do
  if [ $v = hpre2 ]; then L=""; else L="MREC_LIB_PATH=$V/libmrec_$v.so"; fi
  env $L timeout -k 10 120 python tools/bench_tower.py > $O/tower_$v.txt 2>&1
done
timeout -k 10 120 python tools/step_tower_stamps.py > $O/step_stamps.txt 2>&1
echo OK
