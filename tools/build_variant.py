"""Build a variant of libmrec.so with one source recompiled under extra -D flags,
for A/B timing on the GPU box (MREC_LIB_PATH=<variant> selects it at run time).

  python tools/build_variant.py NAME SOURCE.hip[,SOURCE2.hip...] -DFOO=1 [-DBAR=2 ...]

Needs the objects of a normal build (pytorchrec_amd/build.py) and writes
pytorchrec_amd/lib/variants/libmrec_NAME.so."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchrec_amd import build as B  # noqa: E402


def main():
    name, src, defines = sys.argv[1], sys.argv[2], sys.argv[3:]
    B.build_lib(verbose=False)
    obj_dir = os.path.join(B.LIB_DIR, "obj")
    out_dir = os.path.join(B.LIB_DIR, "variants")
    os.makedirs(out_dir, exist_ok=True)
    srcs = B._sources()
    targets = {}
    for one in src.split(","):
        target = os.path.join(B.CSRC, os.path.basename(one))
        assert target in srcs, target
        vobj = os.path.join(out_dir, f"{name}_{os.path.basename(one)}.o")
        subprocess.run([B.HIPCC, *B.CFLAGS, *defines, f"-I{B.INCLUDE}", f"-I{B.CSRC}", "-c",
                        target, "-o", vobj], check=True)
        targets[target] = vobj
    objs = [targets.get(s, os.path.join(obj_dir, os.path.basename(s) + ".o")) for s in srcs]
    lib = os.path.join(out_dir, f"libmrec_{name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-ldl", "-o",
                    lib], check=True)
    print(lib)


if __name__ == "__main__":
    main()
