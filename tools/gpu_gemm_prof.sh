# per-workgroup phase stamps of the GEMM (variant lib built with -DMREC_GEMM_PROF)
set -o pipefail
mkdir -p gpurun_out/dw
for c in dw/s4 dw/s8 fwd; do
  MREC_LIB_PATH=pytorchrec_amd/lib/variants/libmrec_prof.so timeout -k 10 120 python -u tools/bench_gemm.py --reps 100 --only $c --prof > gpurun_out/dw/prof_${c/\//_}.txt 2>&1 || { tail -20 gpurun_out/dw/prof_${c/\//_}.txt; exit 1; }
  cat gpurun_out/dw/prof_${c/\//_}.txt
done
