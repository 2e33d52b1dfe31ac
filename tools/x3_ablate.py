"""Timing-experiment builds of the split-f16 kernel (X3_ABL bits, csrc/dladmm_fused_x3.hip): each
variant is the in-tree library with only dladmm_fused_x3.hip recompiled, linked to
d-ladmm_amd/lib/abl/libdladmm_hip_x3abl<N>.so.  Run a variant with DLADMM_LIB=<that path>.
Every nonzero variant computes WRONG results: timing only.

    python tools/x3_ablate.py 1 2 4 8 16     # build (CPU)
    python tools/x3_ablate.py X3_ABL=0,X3_STORE_AUX=16   # arbitrary -D sets
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "d-ladmm_amd"))
import build as B  # noqa: E402


def one(spec: str) -> str:
    os.makedirs(os.path.join(B.HERE, "lib", "abl"), exist_ok=True)
    defs = [d if "=" in d else f"X3_ABL={d}" for d in spec.split(",")]
    tag = spec.replace(",", "_").replace("=", "").replace("DLADMM_", "")
    obj = os.path.join(B.OBJ, f"dladmm_fused_x3_abl{tag}.o")
    subprocess.run([B.hipcc()] + B.FLAGS + B.UNIT_FLAGS["dladmm_fused_x3.hip"] +
                   [f"-D{d}" for d in defs] +
                   ["-c", os.path.join(B.CSRC, "dladmm_fused_x3.hip"), "-o", obj], check=True)
    objs = [os.path.join(B.OBJ, u.replace(".hip", ".o")) for u in B.UNITS
            if u != "dladmm_fused_x3.hip"] + [obj]
    out = os.path.join(B.HERE, "lib", "abl", f"libdladmm_hip_x3abl{tag}.so")
    subprocess.run([B.hipcc(), "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", out] + objs,
                   check=True)
    return out


if __name__ == "__main__":
    B.build()
    with ThreadPoolExecutor(4) as ex:
        for p in ex.map(one, sys.argv[1:]):
            print(p)
