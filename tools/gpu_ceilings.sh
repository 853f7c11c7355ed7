# Step-0 memory ceilings + PMC calibration of FETCH_SIZE / WRITE_SIZE on kernels
# with known byte counts (tools/micro/ceilings.hip); out: gpurun_out/ceil/
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/ceil
mkdir -p $O
timeout -k 10 120 ./tools/micro/ceilings > $O/ceilings.json 2> $O/ceilings.err || { echo CEIL_FAIL; cat $O/ceilings.err; exit 1; }
cat $O/ceilings.json
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- $R/tools/micro/ceilings > $O/pmc_$c.log 2>&1 || { echo PMC_FAIL $c; tail -20 $O/pmc_$c.log; exit 1; }
done
lscpu > $O/lscpu.txt 2>&1 || true
echo CEIL_OK
