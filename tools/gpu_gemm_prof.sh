set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python tools/bench_gemm.py > gpurun_out/bench_gemm.txt 2>&1 || { cat gpurun_out/bench_gemm.txt; exit 1; }
cat gpurun_out/bench_gemm.txt
export TMPDIR=/tmp
cd /tmp
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  tag=$(echo $pmc | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $pmc -d $R/gpurun_out/pmc_$tag -o run --output-format csv -- python3 $R/tools/bench_gemm.py --reps 20 --only fwd > $R/gpurun_out/pmc_$tag.log 2>&1 || { echo PMC_FAIL $tag; tail -5 $R/gpurun_out/pmc_$tag.log; exit 1; }
done
echo done
