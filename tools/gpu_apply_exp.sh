# In-step apply time (kernel clock) for apply-experiment builds (tools/build_variant.py
# NAME emb_bwd.hip -D...), Zipf C2 ids and uniform C2 ids.
#   bash tools/gpu_apply_exp.sh OUTDIR variant [variant ...]   (base = the product build)
export TMPDIR=/tmp
o=gpurun_out/$1
shift
mkdir -p $o
for v in "$@"; do
  lib=pytorchrec_amd/lib/libmrec.so
  [ $v != base ] && lib=pytorchrec_amd/lib/variants/libmrec_$v.so
  MREC_LIB_PATH=$lib timeout -k 10 200 python bench.py --zipf 1.05 --no-cpu-baseline --no-h2d --steps 20 > $o/$v.zipf.json 2> $o/$v.zipf.err || exit 1
  [ -n "$ZIPF_ONLY" ] || MREC_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2d --steps 20 > $o/$v.uni.json 2> $o/$v.uni.err || exit 1
done
