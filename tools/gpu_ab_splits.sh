# A/B of mrec_tower_dw's K slices (MREC_TDW_SPLITS) on the C2 and C3 bench lines
export TMPDIR=/tmp
o=gpurun_out/${OUT:-r5e}
mkdir -p $o
for m in deepfm dcnv2; do
  for s in 0 2 3 4 5; do
    if [ $s = 0 ]; then unset MREC_TDW_SPLITS; else export MREC_TDW_SPLITS=$s; fi
    timeout -k 10 200 python3 bench.py --model $m --no-cpu-baseline --no-roofline --no-h2d > $o/$m.s$s.json 2> $o/$m.s$s.err || { tail -3 $o/$m.s$s.err; exit 1; }
    python3 -c "import json; d=json.load(open('$o/$m.s$s.json')); print('$m', 'splits=$s', d['ms_per_step'])"
  done
done
