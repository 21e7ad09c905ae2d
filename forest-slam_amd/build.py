"""Build libfvo.so (all HIP kernels + the C ABI) for gfx950 with hipcc, in-tree.

    python -m forest_slam_amd.build        (or __graft_entry__.build())

Every source is compiled to its own object in parallel (build/obj/), then linked; a
source is recompiled when it, a header of csrc/ or include/fvo.h is newer than its object.
-ffp-contract=off is mandatory: the ORB/BF/back-projection kernels reproduce OpenCV's /
NumPy's float roundings operation by operation."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libfvo.so")
OBJ = os.path.join(HERE, "build", "obj")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
SOURCES = ["capi.cpp", "orb.hip", "bf.hip", "sgbm.hip", "pose.hip", "ba.hip", "essential.hip", "ingest.hip", "map.hip", "util.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-Wno-unused-result", "-Wno-unused-function", "-Wno-unused-variable"]


def _headers() -> list[str]:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".inc"))]
    return hs + [os.path.join(INCLUDE, "fvo.h")]


def _obj(src: str) -> str:
    return os.path.join(OBJ, os.path.splitext(src)[0] + ".o")


def _stale(src: str) -> bool:
    o = _obj(src)
    if not os.path.exists(o):
        return True
    t = os.path.getmtime(o)
    return any(os.path.getmtime(d) > t for d in [os.path.join(CSRC, src)] + _headers())


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(INCLUDE, "fvo.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    if not force and not needs_build():
        return OUT
    os.makedirs(OBJ, exist_ok=True)
    todo = [s for s in SOURCES if force or _stale(s)]

    def compile_one(s: str):
        # hipcc compiles .cpp as host C++; route every file through the HIP front end
        cmd = [HIPCC] + FLAGS + ["-I", INCLUDE, "-c", "-x", "hip", os.path.join(CSRC, s), "-o", _obj(s) + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(_obj(s) + ".tmp", _obj(s))

    n = jobs or min(len(todo) or 1, max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(max_workers=n) as ex:
        list(ex.map(compile_one, todo))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp"] + [_obj(s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
