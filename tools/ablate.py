"""Build timing-experiment variants of the fused kernel (never shipped; results are WRONG by design).

    python tools/ablate.py [--unit dladmm_tile_bf16.hip] name=-DFLAG=1[,-DOTHER=2] ...

Each variant recompiles one translation unit (default dladmm_fused.hip) with the extra flags and links it with the regular
capi/layered objects into d-ladmm_amd/lib/abl/<name>/libdladmm_hip.so.  Time one with
    DLADMM_LIB=d-ladmm_amd/lib/abl/<name>/libdladmm_hip.so python bench.py --no-cpu-baseline
Knobs: DLADMM_ABLATE (1 = no weight stream, 2 = no epilogue, 8 = no V1 beta loads, 16 = one
dwordx4 store per block with the same bytes; DLADMM_ABL_AUX its cache policy),
DLADMM_ABLATE_NOSTORE, DLADMM_SYNC_MODE, DLADMM_CHUNK.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "d-ladmm_amd"))
import build as B  # noqa: E402


UNIT = "dladmm_fused.hip"


def one(spec):
    name, _, flags = spec.partition("=")
    flags = [f for f in flags.split(",") if f]
    out = os.path.join(B.HERE, "lib", "abl", name)
    os.makedirs(out, exist_ok=True)
    obj = os.path.join(out, UNIT.replace(".hip", ".o"))
    cc = B.hipcc()
    subprocess.run([cc] + B.FLAGS + B.UNIT_FLAGS.get(UNIT, []) + flags +
                   ["-c", os.path.join(B.CSRC, UNIT), "-o", obj],
                   check=True)
    others = [os.path.join(B.OBJ, u.replace(".hip", ".o")) for u in B.UNITS if u != UNIT]
    subprocess.run([cc, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o",
                    os.path.join(out, "libdladmm_hip.so"), obj] + others, check=True)
    return name


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--unit":
        UNIT = args[1]
        args = args[2:]
    B.build()
    with ThreadPoolExecutor(max_workers=4) as ex:
        for n in ex.map(one, args):
            print("built", n)
