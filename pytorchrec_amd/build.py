"""Build libmrec.so in-tree with hipcc for gfx950.

``python -m pytorchrec_amd.build`` or ``__graft_entry__.build()``.  The shared
library lands in ``pytorchrec_amd/lib/`` (git-ignored, but it travels to the GPU
box with the gpurun snapshot).  A content hash of the sources is stored next to
it so unchanged sources are not recompiled.
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libmrec.so")
ARCH = os.environ.get("MREC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall",
          "-Wno-unused-function", "-Wno-unused-variable"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _digest(srcs):
    h = hashlib.sha256()
    for p in srcs + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(INCLUDE, "mrec.h")]:
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    h.update(" ".join(CFLAGS).encode())
    return h.hexdigest()


def build_lib(force: bool = False, verbose: bool = True) -> str:
    srcs = _sources()
    os.makedirs(LIB_DIR, exist_ok=True)
    stamp = LIB + ".sha256"
    digest = _digest(srcs)
    if not force and os.path.exists(LIB) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return LIB
    objs = []
    obj_dir = os.path.join(LIB_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    procs = []
    for s in srcs:
        o = os.path.join(obj_dir, os.path.basename(s) + ".o")
        objs.append(o)
        cmd = [HIPCC, *CFLAGS, f"-I{INCLUDE}", f"-I{CSRC}", "-c", s, "-o", o]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed ({' '.join(cmd)}):\n{out.decode()}")
        if verbose and out.strip():
            sys.stderr.write(out.decode())
    tmp = LIB + ".tmp"
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-ldl", "-o", tmp]
    r = subprocess.run(link, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {r.stdout.decode()}")
    os.replace(tmp, LIB)
    with open(stamp, "w") as f:
        f.write(digest)
    if verbose:
        print(f"built {LIB} from {len(srcs)} sources for {ARCH}")
    return LIB


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv)
