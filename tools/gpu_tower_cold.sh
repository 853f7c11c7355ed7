set -o pipefail
mkdir -p gpurun_out/tw
for o in "" "--reemit" "--cold"; do
  timeout -k 10 120 python -u tools/bench_tower.py $o > gpurun_out/tw/cold.txt 2>&1 || { tail -20 gpurun_out/tw/cold.txt; exit 1; }
  echo "[$o] $(grep widths gpurun_out/tw/cold.txt)"; grep -E "x0 loaded|fwd1|bwd done" gpurun_out/tw/cold.txt
done
