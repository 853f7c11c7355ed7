set -o pipefail
mkdir -p gpurun_out/dw
for v in base tdw1 tdw2 tdw3 tdw4; do
  if [ $v = base ]; then L=""; else L=pytorchrec_amd/lib/variants/libmrec_$v.so; fi
  MREC_LIB_PATH=$L timeout -k 10 200 python -u tools/bench_gemm.py --reps 200 --only tdw > gpurun_out/dw/tdw_$v.txt 2>&1 || { tail -20 gpurun_out/dw/tdw_$v.txt; exit 1; }
  echo "== $v"; grep tdw gpurun_out/dw/tdw_$v.txt
done
