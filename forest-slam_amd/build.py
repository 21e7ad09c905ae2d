"""Build libfvo.so (all HIP kernels + the C ABI) for gfx950 with hipcc, in-tree.

    python -m forest_slam_amd.build        (or __graft_entry__.build())

-ffp-contract=off is mandatory: the ORB/BF/back-projection kernels reproduce OpenCV's /
NumPy's float roundings operation by operation."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libfvo.so")
SOURCES = ["capi.cpp", "orb.hip", "bf.hip", "sgbm.hip", "pose.hip", "ba.hip", "essential.hip", "ingest.hip", "map.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-fast-math", "-Wno-unused-result", "-Wno-unused-function", "-Wno-unused-variable"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "fvo.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    srcs = []
    for s in SOURCES:
        p = os.path.join(CSRC, s)
        # hipcc compiles .cpp as host C++; route every file through the HIP front end
        srcs += (["-x", "hip", p] if s.endswith(".hip") else ["-x", "hip", p])
    cmd = [HIPCC] + FLAGS + ["-I", os.path.join(os.path.dirname(HERE), "include"), "-o", OUT + ".tmp"] + srcs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
