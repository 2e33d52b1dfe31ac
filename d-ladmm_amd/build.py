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
UNITS = ("dladmm_capi.hip", "dladmm_fused.hip", "dladmm_fused_savep.hip", "dladmm_fused_x3.hip",
         "dladmm_fused_x3_savep.hip", "dladmm_fused_rs.hip", "dladmm_fused_xs.hip",
         "dladmm_layered.hip", "dladmm_backward.hip", "dladmm_lskm.hip", "dladmm_eval.hip",
         "dladmm_tile_bf16.hip", "dladmm_wgrad_x3.hip",
         "dladmm_reverse.hip", "dladmm_reverse_rs.hip",
         "dladmm_lena.hip",
         # reverse-sweep instantiations: one unit per E-step form and shape group (minutes each)
         "dladmm_reverse_vvar.hip", "dladmm_reverse_v1.hip", "dladmm_reverse_lasso.hip",
         "dladmm_reverse_vvar_small.hip", "dladmm_reverse_v1_small.hip",
         "dladmm_reverse_lasso_small.hip", "dladmm_reverse_v2.hip", "dladmm_reverse_v3.hip",
         "dladmm_reverse_v2_small.hip", "dladmm_reverse_v3_small.hip")
INCLUDE = os.path.join(ROOT, "include")
OUT = os.path.join(HERE, "lib", "libdladmm_hip.so")
OBJ = os.path.join(HERE, "lib", "obj")
ARCH = os.environ.get("DLADMM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", f"--offload-arch={ARCH}",
         "-I", os.path.join(ROOT, "include")]
# per-unit extras: the split-f16 kernel and the reverse sweep keep scalar f32 VALU beside their
# MFMAs (packed v_pk_* f32 ops issue slower there; MI355X_MICROARCH.md, price of one filler
# beside MFMAs)
UNIT_FLAGS = {u: ["-fno-slp-vectorize"] for u in UNITS
              if u.startswith("dladmm_fused_x3") or u.startswith("dladmm_reverse")}
# the split-f16 weight gradient unscales every MFMA result with VALU: MFMA results in VGPRs
# (no v_accvgpr_read per element)
UNIT_FLAGS["dladmm_wgrad_x3.hip"] = ["-mllvm", "-amdgpu-mfma-vgpr-form"]


def deps(path, seen=None):
    """The file and every local header it includes (recursively): a unit is rebuilt only when
    one of ITS sources changed."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    for line in open(path):
        line = line.strip()
        if line.startswith("#include \""):
            name = line.split('"')[1]
            for d in (os.path.dirname(path), CSRC, INCLUDE):
                cand = os.path.join(d, name)
                if os.path.exists(cand):
                    deps(cand, seen)
                    break
    return seen


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
    srcs = set()
    for u in _units():
        srcs |= deps(os.path.join(CSRC, u))
    return not _stale(OUT, sorted(srcs))


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
        if force or extra_flags or _stale(obj, sorted(deps(src))):
            jobs.append([cc] + FLAGS + UNIT_FLAGS.get(u, []) + list(extra_flags) +
                        ["-c", src, "-o", obj])

    def run(cmd):
        if verbose:
            print("[dladmm build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    # the long reverse-sweep units first, so they do not end up last in the pool
    jobs.sort(key=lambda c: 0 if os.path.basename(c[-3]).startswith("dladmm_reverse_") else 1)
    with ThreadPoolExecutor(max_workers=max(1, min(len(jobs), os.cpu_count() or 6, 8))) as ex:
        list(ex.map(run, jobs))
    tmp = OUT + ".tmp"
    run([cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
