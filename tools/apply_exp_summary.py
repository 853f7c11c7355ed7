"""Print ms/step and the in-step apply time of tools/gpu_apply_exp.sh outputs."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads([ln for ln in open(f).read().splitlines() if ln.startswith("{")][-1])
    rk = d["roofline_kernels"]
    ap = [v for k, v in rk.items() if "apply" in k][0]
    print(f"{os.path.basename(f):24s} {d['ms_per_step']:.4f} ms  apply {ap['avg_us']:6.2f} us "
          f"(span {ap.get('wave_span_us')})")
