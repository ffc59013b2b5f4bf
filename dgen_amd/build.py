"""Build libdgen_hip.so in-tree (gfx950).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container; the resulting .so is git-ignored but travels to the GPU box with
the repository snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "dgen_hip.hip")
HDR = os.path.join(REPO, "include", "dgen_hip.h")
OUT_DIR = os.path.join(HERE, "lib")
OUT = os.path.join(OUT_DIR, "libdgen_hip.so")
ARCH = os.environ.get("DGEN_OFFLOAD_ARCH", "gfx950")

FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    # keep a*b+c as two roundings: the bracket / Brent path stays bit-identical
    # to scipy and numpy, and the kernels agree with the oracle
    "-ffp-contract=off",
    "-Wall", "-Wno-unused-function",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in (SRC, HDR, __file__))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = OUT + ".tmp"
    cmd = [hipcc(), *FLAGS, "-o", tmp, SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stderr[-4000:]}")
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
