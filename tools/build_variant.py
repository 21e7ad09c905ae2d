#!/usr/bin/env python3
"""Build a variant of libfvo.so with extra -D defines for one source (launch-shape
experiments; tooling only):  python tools/build_variant.py NAME SOURCE -DFOO=1 ...
-> exp/libfvo_NAME.so, loaded by setting FVO_LIB=exp/libfvo_NAME.so.  SOURCE may be
PATH:NAME.hip to compile an edited copy at PATH in place of csrc/NAME.hip, and a comma-separated
list of such entries."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import forest_slam_amd.build as b  # noqa: E402


def main():
    name, srcs, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
    b.build()
    os.makedirs(os.path.join(ROOT, "exp"), exist_ok=True)
    repl = {}
    for ent in srcs.split(","):
        path, src = ent.split(":") if ":" in ent else (None, ent)
        obj = os.path.join(ROOT, "exp", f"{os.path.splitext(src)[0]}_{name}.o")
        subprocess.run([b.HIPCC] + b.FLAGS + defs + ["-I", b.INCLUDE, "-I", b.CSRC, "-c", "-x", "hip",
                                                     path or os.path.join(b.CSRC, src), "-o", obj], check=True)
        repl[src] = obj
    objs = [repl.get(s, b._obj(s)) for s in b.SOURCES]
    out = os.path.join(ROOT, "exp", f"libfvo_{name}.so")
    subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, check=True)
    print(out)


if __name__ == "__main__":
    main()
