# Quick GPU check -> gpurun_out/$OUT/: the -m gpu suite (or $TESTS), then plain bench
# lines named in $LINES ("c2 c3 c4 zipf shard", default "c2 c3").
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-quick}
mkdir -p $o
cd $GRAFT_REPO_ROOT
if [ "${TESTS:-all}" != "none" ]; then
  sel=${TESTS:-tests}; [ "$sel" = all ] && sel=tests
  timeout -k 10 900 python3 -u -m pytest $sel -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
  tail -2 $o/pytest.log
fi
plain() { name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $o/$name.json 2> $o/$name.err || { tail -5 $o/$name.err; exit 1; }; python3 -c "import json; d=json.load(open('$o/$name.json')); print('$name', d['ms_per_step'], d['value'], d.get('pcie_inclusive',{}).get('ms_per_step') if isinstance(d.get('pcie_inclusive'),dict) else '')"; }
for l in ${LINES:-c2 c3}; do
  case $l in
    c2) plain c2 --no-cpu-baseline || exit 1 ;;
    c3) plain c3 --model dcnv2 --no-cpu-baseline --no-h2d || exit 1 ;;
    c4) plain c4 --model din --no-cpu-baseline --no-h2d || exit 1 ;;
    zipf) plain zipf --zipf 1.05 --no-cpu-baseline --no-h2d || exit 1 ;;
    shard) plain shard --shard --force-collectives --exchange compact --no-cpu-baseline --no-h2d || exit 1 ;;
  esac
done
