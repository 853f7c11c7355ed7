# destroy_process_group after graph-captured RCCL: one variant per process, each
# under its own time limit (a hang is the finding, not a failure of the script)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/destroy
for v in ${VARIANTS:-eager graph_keep graph_del graph_reset}; do
  echo "== $v"
  timeout -k 5 45 python -u tools/destroy_probe.py $v > gpurun_out/destroy/$v.log 2>&1
  echo "rc=$?"
  grep -v amdgpu.ids gpurun_out/destroy/$v.log | tail -8
done
exit 0
