"""Timing-experiment builds with extra compile flags on chosen units (A/B of knobs that span
several kernels).  Each variant lands in d-ladmm_amd/lib/abl/<name>/libdladmm_hip.so:

    python tools/ablate_units.py dma0=-DDLADMM_DMA4=0@dladmm_layered.hip+dladmm_backward.hip

Units not listed are linked from the regular in-tree objects.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "d-ladmm_amd"))
import build as B  # noqa: E402


def one(spec):
    name, _, rest = spec.partition("=")
    flags, _, units = rest.partition("@")
    flags = [f for f in flags.split(",") if f]
    units = units.split("+") if units else list(B.UNITS)
    out = os.path.join(B.HERE, "lib", "abl", name)
    os.makedirs(out, exist_ok=True)
    objs = []
    for u in B.UNITS:
        if u in units:
            o = os.path.join(out, u.replace(".hip", ".o"))
            subprocess.run([B.hipcc()] + B.FLAGS + B.UNIT_FLAGS.get(u, []) + flags +
                           ["-c", os.path.join(B.CSRC, u), "-o", o], check=True)
        else:
            o = os.path.join(B.OBJ, u.replace(".hip", ".o"))
        objs.append(o)
    subprocess.run([B.hipcc(), "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o",
                    os.path.join(out, "libdladmm_hip.so")] + objs, check=True)
    return name


if __name__ == "__main__":
    B.build()
    with ThreadPoolExecutor(max_workers=4) as ex:
        for n in ex.map(one, sys.argv[1:]):
            print("built", n)
