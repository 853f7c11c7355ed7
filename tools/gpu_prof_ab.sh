# rocprof kernel summaries of one bench line under env settings: AB="VAR=a VAR=b" ("-" =
# unset), ARGS = bench arguments -> gpurun_out/$OUT/<i>/ ; prints ms/step per setting
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-profab}
mkdir -p $o
cd /tmp
i=0
for kv in $AB; do
  i=$((i+1))
  (
    if [ "$kv" != "-" ]; then export "$kv"; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-roofline --no-h2d --steps 50 $ARGS > $o/$i.json 2> $o/$i.err || { tail -3 $o/$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$o/$i.json')); print('$i $kv', d['ms_per_step'])"
  ) || exit 1
done
