"""Build libdladmm_hip.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo).

    python d-ladmm_amd/build.py [--force]
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", "dladmm_fused.hip")]
DEPS = SRC + [os.path.join(ROOT, "include", "dladmm.h")]
OUT = os.path.join(HERE, "lib", "libdladmm_hip.so")
ARCH = os.environ.get("DLADMM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include")]


def hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    cmd = [hipcc()] + FLAGS + ["-o", tmp] + SRC
    if verbose:
        print("[dladmm build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
