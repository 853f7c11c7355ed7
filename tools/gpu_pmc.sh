# HBM traffic of the embedding-path kernels from PMC counters, per model (separate
# passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass) -> gpurun_out/pmc_traffic.json
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for m in deepfm dcnv2 din; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c -d $O/${m}_$c -o run --output-format csv -- python3 $R/bench.py --model $m --steps 5 --warmup 3 --no-cpu-baseline --no-h2d > $O/${m}_$c.log 2>&1 || { echo PMC_FAIL $m $c; tail -20 $O/${m}_$c.log; exit 1; }
  done
done
cd $R
python tools/pmc_traffic.py gpurun_out/pmc_traffic.json deepfm 4096 38462 $O/deepfm_FETCH_SIZE $O/deepfm_WRITE_SIZE dcnv2 4096 38462 $O/dcnv2_FETCH_SIZE $O/dcnv2_WRITE_SIZE din 4096 38462 $O/din_FETCH_SIZE $O/din_WRITE_SIZE > /dev/null && echo PMC_OK
