"""bench.py --gpus N as its own launcher: without
torch.distributed.run, a parent that never touches the GPU starts one child per
rank and relays rank 0's single JSON line.  Exercised on the CPU with the gloo
stub step (--stub-step): the launcher, the env each rank sees, the max-over-ranks
timing and the failure path; the GPU step itself is the driver's N-GPU run."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None, timeout=120):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                          env=e, capture_output=True, text=True, timeout=timeout)


def test_launcher_two_ranks_one_line():
    p = _bench("--gpus", "2", "--stub-step", "--steps", "4", "--warmup", "1")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 2 * 4096
    assert d["config"]["rows_per_table"] == 100_000_000  # N > 1 defaults to C5


def test_launcher_single_gpu_unchanged():
    p = _bench("--gpus", "1", "--stub-step", "--steps", "2", "--warmup", "0")
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip())
    assert d["n_gpus"] == 1 and d["config"]["rows_per_table"] == 38462  # C2


def test_launcher_refuses_mismatched_world():
    p = _bench("--gpus", "1", "--stub-step", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr


def test_launcher_failing_rank_fails_the_job():
    p = _bench("--gpus", "2", "--stub-step", "--steps", "2", env={"BENCH_STUB_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert "rank 1 exited with 3" in p.stderr
    assert p.stdout.strip() == ""
