# rocprof kernel traces of bench.py for the product library and variants in ONE call
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/abprof && cd /tmp
export TMPDIR=/tmp
for v in prod ${VARIANTS:-head}; do
  if [ $v = prod ]; then L=; else L=$R/pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_ABI_ANY=1 MREC_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abprof/$v -o run --output-format csv -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-h2d --no-roofline ${BENCH_ARGS:-} > $R/gpurun_out/abprof/$v.log 2>&1 || { echo PROF_FAIL $v; tail -20 $R/gpurun_out/abprof/$v.log; exit 1; }
  echo "== $v"; python3 $R/tools/kstats.py $R/gpurun_out/abprof/$v/run_kernel_stats.csv | head -6
done
