# Same-box A/B of the 16-bit ids in the host records (MREC_FEED_NARROW=1: the copy
# widens them; 0: int32 records) on the C2 bench's PCIe-inclusive leg, after the
# loader GPU tests (bit-exact batches, training == resident).
export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-fnarrow}; mkdir -p $o
timeout -k 10 300 python3 -u -m pytest tests/test_loader.py tests/test_gpu_tower.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1; tail -2 $o/t.log
for r in 1 2; do for v in 1 0; do
  MREC_FEED_NARROW=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline > $o/c2_$v.json 2> $o/c2_$v.err || { tail -5 $o/c2_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/c2_$v.json')); p=d['pcie_inclusive']; print('narrow=$v', d['ms_per_step'], p['ms_per_step'], p['h2d_bytes_per_step'])"
done; done
