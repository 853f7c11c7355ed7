set -o pipefail
mkdir -p gpurun_out/plan
timeout -k 10 120 python -u tools/bench_plan.py > gpurun_out/plan/base.txt 2>&1 || { tail -20 gpurun_out/plan/base.txt; exit 1; }
grep plan gpurun_out/plan/base.txt
MREC_LIB_PATH=pytorchrec_amd/lib/variants/libmrec_planprof.so timeout -k 10 120 python -u tools/bench_plan.py > gpurun_out/plan/prof.txt 2>&1 || { tail -20 gpurun_out/plan/prof.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/plan/prof.txt
