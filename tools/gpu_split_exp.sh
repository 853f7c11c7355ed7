set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in 1 0; do
for s in 0 5; do
  MREC_ASYNC_PLAN=$a MREC_DW_SPLIT=$s timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-roofline --no-cpu-baseline > gpurun_out/s$s.json 2>gpurun_out/s$s.err || { tail gpurun_out/s$s.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s$s.json'));print('async $a split $s', d['value'], d['ms_per_step'])"
done
done
