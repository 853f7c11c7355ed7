# the apply's block kinds clocked apart (variant built with -DMREC_KC_CAT): uniform and Zipf C2
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/kccat; mkdir -p $o; cd $GRAFT_REPO_ROOT
for z in 0 1.05; do
  MREC_LIB_PATH=$GRAFT_REPO_ROOT/pytorchrec_amd/lib/variants/kccat/libmrec.so MREC_BENCH_KC_CAT=1 timeout -k 10 300 python3 bench.py --zipf $z --no-cpu-baseline --no-h2d > $o/z$z.json 2> $o/z$z.err || { tail -5 $o/z$z.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/z$z.json')); print('zipf $z', d['ms_per_step'], json.dumps(d['roofline_kernels']['mrec_emb_bwd_apply_ex'].get('block_kinds_us')))"
done
