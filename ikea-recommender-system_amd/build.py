"""Build the gfx950 C-ABI library in-tree:
    ikea-recommender-system_amd/recommenders/hip/libikea_rec_hip.so

    python ikea-recommender-system_amd/build.py [--jobs N]

Plain hipcc (no hipify, no torch extension machinery): each csrc/*.hip is
compiled for --offload-arch=gfx950 in parallel, then linked as one shared
object exporting the extern "C" entry points of include/ikea_rec_hip.h.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "recommenders", "hip")
LIB = os.path.join(OUT_DIR, "libikea_rec_hip.so")
OBJ = os.path.join(HERE, "build", "obj")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result"]
LINK = ["-L/opt/rocm/lib", "-lrccl"]


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MI355X path cannot be built")


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o"))
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps = [src, *headers, os.path.abspath(__file__)]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(p) for p in deps):
        return obj
    cmd = [hipcc(), *FLAGS, "-I", CSRC, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(jobs: int = 8, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(OUT_DIR, exist_ok=True)
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        # librccl: csrc/comm.hip (the item-sharded step's collectives on the compute stream)
        cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", LIB, *LINK]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    build(a.jobs)
    sys.exit(0)
