# sharded W=1 compact bench under env settings (ENVS="A=1 B=2|A=0" ...): in-step times
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/senv; mkdir -p $o; cd $GRAFT_REPO_ROOT
IFS='|' read -ra LIST <<< "${ENVS}"
i=0
for e in "${LIST[@]}"; do
  i=$((i+1))
  env $e timeout -k 10 300 python3 bench.py --shard --force-collectives --exchange compact --no-cpu-baseline --no-h2d --steps 100 > $o/e$i.json 2> $o/e$i.err || { echo FAIL "$e"; tail -3 $o/e$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/e$i.json')); print('$e', d['ms_per_step'], json.dumps({k: v['avg_us'] for k, v in d['roofline_kernels'].items()}))"
done
