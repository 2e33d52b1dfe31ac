"""Build libdladmm_hip.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo).

    python d-ladmm_amd/build.py [--force]

Each translation unit compiles to an object in parallel (the fused kernel's unrolled bodies
dominate: ~1.5 min), then one shared library is linked.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
UNITS = ("dladmm_capi.hip", "dladmm_fused.hip", "dladmm_fused_savep.hip", "dladmm_fused_x3.hip", "dladmm_layered.hip",
         "dladmm_backward.hip", "dladmm_lskm.hip", "dladmm_eval.hip", "dladmm_tile_bf16.hip",
         "dladmm_reverse.hip")
HEADERS = (os.path.join(ROOT, "include", "dladmm.h"), os.path.join(CSRC, "dladmm_common.h"),
           os.path.join(CSRC, "dladmm_fused_kernel.h"),
           os.path.join(CSRC, "dladmm_internal.h"), os.path.join(CSRC, "dladmm_slice.h"),
           os.path.join(CSRC, "dladmm_layer_epi.h"))
OUT = os.path.join(HERE, "lib", "libdladmm_hip.so")
OBJ = os.path.join(HERE, "lib", "obj")
ARCH = os.environ.get("DLADMM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", f"--offload-arch={ARCH}",
         "-I", os.path.join(ROOT, "include")]
# per-unit extras: the split-f16 kernel keeps scalar f32 VALU beside its MFMAs (packed v_pk_*
# f32 ops issue slower there; MI355X_MICROARCH.md, price of one filler beside MFMAs)
UNIT_FLAGS = {"dladmm_fused_x3.hip": ["-fno-slp-vectorize"],
              "dladmm_reverse.hip": ["-fno-slp-vectorize"]}


def hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _units():
    return [u for u in UNITS if os.path.exists(os.path.join(CSRC, u))]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def up_to_date() -> bool:
    deps = [os.path.join(CSRC, u) for u in _units()] + list(HEADERS)
    return not _stale(OUT, deps)


def build(force: bool = False, verbose: bool = True, extra_flags=()) -> str:
    if not force and not extra_flags and up_to_date():
        return OUT
    os.makedirs(OBJ, exist_ok=True)
    cc = hipcc()
    jobs = []
    objs = []
    for u in _units():
        src = os.path.join(CSRC, u)
        obj = os.path.join(OBJ, u.replace(".hip", ".o"))
        objs.append(obj)
        if force or extra_flags or _stale(obj, [src] + list(HEADERS)):
            jobs.append([cc] + FLAGS + UNIT_FLAGS.get(u, []) + list(extra_flags) +
                        ["-c", src, "-o", obj])

    def run(cmd):
        if verbose:
            print("[dladmm build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(max_workers=max(1, min(len(jobs), 6))) as ex:
        list(ex.map(run, jobs))
    tmp = OUT + ".tmp"
    run([cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
