"""Build a diagnostic variant of libmrec.so with extra preprocessor defines:

    python tools/build_variant.py NAME -DMREC_APPLY_EXP=2 [...]

-> pytorchrec_amd/lib/variants/libmrec_NAME.so (select it with MREC_LIB_PATH).
Only the sources whose text mentions one of the defined macros are recompiled;
the others reuse the product objects in pytorchrec_amd/lib/obj/."""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchrec_amd import build as B  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    B.build_lib(verbose=False)
    macros = [re.match(r"-D(\w+)", d).group(1) for d in defs]
    out_dir = os.path.join(B.LIB_DIR, "variants")
    obj_dir = os.path.join(out_dir, "obj_" + name)
    os.makedirs(obj_dir, exist_ok=True)
    objs, procs = [], []
    for s in B._sources():
        text = open(s).read()
        base = os.path.basename(s) + ".o"
        hdrs = [h for h in re.findall(r'#include "(\w+\.h)"', text)]
        mention = any(m in text for m in macros) or any(
            m in open(os.path.join(B.CSRC, h)).read() for h in hdrs
            if os.path.exists(os.path.join(B.CSRC, h)) for m in macros)
        if not mention:
            objs.append(os.path.join(B.LIB_DIR, "obj", base))
            continue
        o = os.path.join(obj_dir, base)
        objs.append(o)
        cmd = [B.HIPCC, *B.CFLAGS, *defs, f"-I{B.INCLUDE}", f"-I{B.CSRC}", "-c", s, "-o", o]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit("compile failed")
    lib = os.path.join(out_dir, f"libmrec_{name}.so")
    subprocess.check_call([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-ldl", "-o", lib])
    print(lib)


if __name__ == "__main__":
    main()
