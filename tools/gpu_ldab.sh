# A/B of the working tree's library against the committed one (libmrec_head.so, built
# from HEAD): the embedding / pins / DIN / sharded GPU tests, then bench lines (ARGS_LIST)
export TMPDIR=/tmp
mkdir -p gpurun_out/ldab
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_embedding.py tests/test_gpu_pins.py tests/test_gpu_din.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ldab/t.log 2>&1; tail -2 gpurun_out/ldab/t.log
H=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/libmrec_head.so
IFS='|' read -ra LIST <<< "${ARGS_LIST:---model deepfm|--model deepfm --zipf 1.05}"
for m in "${LIST[@]}"; do
  AB="MREC_LIB_PATH=$H - MREC_LIB_PATH=$H -" ARGS="$m" REP=1 OUT=ldab/x bash tools/gpu_ab_env.sh || exit 1
done
