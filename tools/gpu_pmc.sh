# HBM traffic of the embedding-path kernels from PMC counters (separate passes:
# FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), then profiles/pmc_traffic.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 --no-cpu-baseline > $R/gpurun_out/pmc_$c.log 2>&1 || { echo PMC_FAIL $c; tail -20 $R/gpurun_out/pmc_$c.log; exit 1; }
done
cd $R
python tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc_traffic.json && cat gpurun_out/pmc_traffic.json
