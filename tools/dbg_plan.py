import sys, torch
sys.path.insert(0, '.')
import bench
from pytorchrec_amd import dense, embedding
orig_run = dense._run
def run(jobs):
    print("run", len(jobs), "pending plan:", [(type(p).__name__, p.launched) for p in dense._PLAN])
    return orig_run(jobs)
dense._run = run
orig_get = embedding._FusedPlan.get
def get(self):
    print("get launched=", self.launched)
    return orig_get(self)
embedding._FusedPlan.get = get
orig_init = embedding._FusedPlan.__init__
def init(self, *a):
    print("FusedPlan created")
    orig_init(self, *a)
embedding._FusedPlan.__init__ = init
sys.argv = ["bench.py", "--steps", "1", "--warmup", "0", "--no-graph", "--no-roofline", "--no-cpu-baseline"]
bench.main()
