# Round-end checks on the GPU box: the GPU suite, smoke(), the default bench line and
# its rocprof kernel summary (gpurun_out/r4z*).
export TMPDIR=/tmp
o=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/r4z_pytest.log 2>&1 || { tail -30 $o/r4z_pytest.log; exit 1; }
tail -3 $o/r4z_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $o/r4z_smoke.log 2>&1 || { tail -20 $o/r4z_smoke.log; exit 1; }
tail -1 $o/r4z_smoke.log
timeout -k 10 300 python bench.py > $o/r4z_bench.json 2> $o/r4z_bench.err || { tail -20 $o/r4z_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/r4z_prof -o run -- python3 bench.py > $o/r4z_benchp.json 2> $o/r4z_benchp.err || exit 1
echo FINAL_OK
