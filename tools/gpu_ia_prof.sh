set -o pipefail
mkdir -p gpurun_out/ia
timeout -k 10 120 python -u tools/bench_interact.py > gpurun_out/ia/base.txt 2>&1 || { tail -20 gpurun_out/ia/base.txt; exit 1; }
grep interact gpurun_out/ia/base.txt
MREC_LIB_PATH=pytorchrec_amd/lib/variants/libmrec_iaprof.so timeout -k 10 120 python -u tools/bench_interact.py > gpurun_out/ia/prof.txt 2>&1 || { tail -20 gpurun_out/ia/prof.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ia/prof.txt
