# Same-box A/B of an environment knob on the PCIe-inclusive (host-fed) leg: AB="VAR=a ..."
# (each a bench run; "-" = unset), ARGS = extra bench arguments, REP = alternations
export TMPDIR=/tmp
o=gpurun_out/${OUT:-abh}
mkdir -p $o
for r in $(seq 1 ${REP:-2}); do
  for kv in $AB; do
    (
      if [ "$kv" != "-" ]; then export "$kv"; fi
      timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-roofline $ARGS > $o/run.json 2> $o/run.err || { tail -3 $o/run.err; exit 1; }
      python3 -c "import json; d=json.load(open('$o/run.json')); print('$kv', d['ms_per_step'], d['pcie_inclusive']['ms_per_step'])"
    ) || exit 1
  done
done
