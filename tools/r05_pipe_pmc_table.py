"""Per-dispatch mean counters of config 5's tile kernels from tools/r05_pipe_pmc.sh's output
(gpurun_out/pipepmc/) -> JSON on stdout.  Kernels by role: G1 = the one-phase PH 0 instance or the
pipelined G1 kernel, G2 = PH 1, prologue = PH 2."""
import collections
import csv
import glob
import json
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pipepmc"
out = {}
for mode in ("onephase", "pipe", "pnost"):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{root}/{mode}_p*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "pipe_g1" in k:
                role = "G1"
            else:
                m = re.search(r"tile_bf16_kernel<\d+, \d+, (\d), \d>", k)
                if not m:
                    continue
                role = {"0": "G1", "1": "G2", "2": "prologue"}[m.group(1)]
            vals[role][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    res = {}
    for role, d in vals.items():
        per = collections.defaultdict(list)
        for (c, _), v in d.items():
            per[c].append(sum(v))  # one dispatch: sum over the counter's instances
        res[role] = {c: sum(v) / len(v) for c, v in sorted(per.items())}
        wc = res[role].get("SQ_WAVE_CYCLES")
        if wc:
            for c in list(res[role]):
                if c.startswith(("SQ_WAIT", "SQ_ACTIVE")):
                    res[role][c + "/wave_cycles"] = res[role][c] / wc
    out[mode] = res
json.dump(out, sys.stdout, indent=1)
print()
