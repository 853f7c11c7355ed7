# HBM traffic of the bench lines' kernels from PMC counters, one bench workload per
# pair of passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass) ->
# gpurun_out/pmc_traffic.json (copy it to profiles/).  Each workload's stamp carries
# its bench args' workload key and the library digest (bench.py reports the traffic
# only for its own workload and library).  MREC_COMMIT names the commit (no .git on
# the box).  WORKLOADS selects: c2 zipf c3 c4 shard c5 (default all).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
args_of() {
  case $1 in
    c2) echo "--model deepfm" ;;
    zipf) echo "--model deepfm --zipf 1.05" ;;
    c3) echo "--model dcnv2" ;;
    c4) echo "--model din" ;;
    shard) echo "--model deepfm --shard --force-collectives --exchange compact" ;;
    c5) echo "--model deepfm --rows-per-table 100000000" ;;
  esac
}
pairs=""
for w in ${WORKLOADS:-c2 zipf c3 c4 shard c5}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c -d $O/${w}_$c -o run --output-format csv -- python3 $R/bench.py $(args_of $w) --steps 5 --warmup 3 --no-cpu-baseline --no-h2d > $O/${w}_$c.log 2>&1 || { echo PMC_FAIL $w $c; tail -20 $O/${w}_$c.log; exit 1; }
  done
  pairs="$pairs $O/${w}_FETCH_SIZE $O/${w}_WRITE_SIZE"
done
cd $R
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json 2>/dev/null
python3 tools/pmc_traffic.py gpurun_out/pmc_traffic.json $pairs && echo PMC_OK
