# DIN top-tower weight-gradient K slices: 16 (default) / 8 / 4 (MREC_TDW_SPLITS)
set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3s
mkdir -p $O
for r in 1 2; do
for k in 16 8 4; do
  MREC_TDW_SPLITS=$k timeout -k 10 200 python bench.py --model din --no-cpu-baseline --no-roofline > $O/din_s${k}_$r.json 2> $O/din_s$k.err
done
done
echo OK
