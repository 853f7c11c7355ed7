# One SQ PMC pass per model (wave cycles split into active / parked / issue-stalled,
# VALU and LDS instruction counts) -> gpurun_out/$OUT/<model>/
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-pmc_sq}
mkdir -p $o
cd /tmp
for m in ${MODELS:-deepfm din}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $o/$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model $m --no-cpu-baseline --no-roofline --no-h2d --steps 5 --warmup 2 > $o/$m.json 2> $o/$m.err || { tail -5 $o/$m.err; exit 1; }
done
