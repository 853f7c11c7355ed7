# Same-box A/B of an environment knob on a bench line: AB="VAR=a VAR=b ..." (each a
# bench run; "-" = unset), ARGS = extra bench arguments, REP = alternations
export TMPDIR=/tmp
o=gpurun_out/${OUT:-ab}
mkdir -p $o
for r in $(seq 1 ${REP:-2}); do
  for kv in $AB; do
    (
      if [ "$kv" != "-" ]; then export "$kv"; fi
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --no-h2d $ARGS > $o/run.json 2> $o/run.err || { tail -3 $o/run.err; exit 1; }
      python3 -c "import json; d=json.load(open('$o/run.json')); print('$kv', d['ms_per_step'])"
    ) || exit 1
  done
done
