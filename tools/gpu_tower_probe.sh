# Tower bound probe: the L2 broadcast-read micro (tools/micro/l2bcast.hip) and the
# tower's per-phase stamps (tools/bench_tower.py); out: gpurun_out/tower/
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/tower
mkdir -p $O
timeout -k 10 120 ./tools/micro/l2bcast > $O/l2bcast.json 2> $O/l2bcast.err || { echo L2B_FAIL; cat $O/l2bcast.err; exit 1; }
python -c "
import json;d=json.load(open('$O/l2bcast.json'))
for r in d['runs']: print(r)"
timeout -k 10 180 python -u tools/bench_tower.py > $O/tower.txt 2>&1 || { echo TOWER_FAIL; tail -20 $O/tower.txt; exit 1; }
cat $O/tower.txt
echo PROBE_OK
