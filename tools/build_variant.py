"""Build a diagnostic variant of libmrec with extra preprocessor flags:
    python tools/build_variant.py NAME -DMREC_APPLY_EXP=15 [...]
-> pytorchrec_amd/lib/variants/NAME/libmrec.so (run with MREC_LIB_PATH=...).  The
product library (pytorchrec_amd/build.py) is not touched."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pytorchrec_amd import build as B  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    out_dir = os.path.join(B.LIB_DIR, "variants", name)
    obj_dir = os.path.join(B.LIB_DIR, "variants", "obj_" + name)
    os.makedirs(out_dir, exist_ok=True)
    os.makedirs(obj_dir, exist_ok=True)
    procs, objs = [], []
    for s in B._sources():
        o = os.path.join(obj_dir, os.path.basename(s) + ".o")
        objs.append(o)
        cmd = [B.HIPCC, *B.CFLAGS, *defs, f"-I{B.INCLUDE}", f"-I{B.CSRC}", "-c", s, "-o", o]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out, _ = p.communicate()
        if p.returncode:
            raise SystemExit(out.decode())
    lib = os.path.join(out_dir, "libmrec.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-ldl", "-o", lib],
                   check=True)
    print(lib)


if __name__ == "__main__":
    main()
