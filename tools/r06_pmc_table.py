"""Round-6 counter table (tools/r06_pmc.sh) -> profiles/r06_cfg5_pmc.json.

Per workload and kernel: the counters' mean per dispatch (warmup dispatches included: every
dispatch of a pass is counted), the duration of the same dispatches, and the derived MFMA-side
figures, each of which must be PHYSICAL to be quoted:
  * busy_from_counter  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
    (the counter is per SIMD, summed over the 32 SE instances; GRBM_GUI_ACTIVE is summed over
    the 8 XCDs) -- valid only when <= 1;
  * busy_from_insts    = SQ_INSTS_MFMA * cycles per MFMA / (GRBM_GUI_ACTIVE / 8 * 1024):
    16 cycles per v_mfma_f32_16x16x32_bf16, 32 per v_mfma_f32_16x16x4_f32 (MI355X_MICROARCH.md
    issue table);
  * flop_from_mops     = (MOPS_BF16 + MOPS_F32) * 512, against the algorithmic FLOP per launch;
  * clock_ghz          = GRBM_GUI_ACTIVE / 8 / duration;
  * cu_busy_frac       = SQ_BUSY_CU_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs)   (quad-cycles x 4
    if the counter counts quad-cycles: both readings are given).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CYC = {"bf16": 16.0, "f32": 32.0}


def load(dirpath):
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(dirpath, "*counter_collection.csv")):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (r["Dispatch_Id"], k)
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return vals, dur


def short(k):
    return k.split("(")[0].replace("void ", "")[:60]


def main(src="gpurun_out/r06pmc", dst="profiles/r06_cfg5_pmc.json"):
    out = {"what": __doc__.strip().split("\n\n")[1], "source": "tools/r06_pmc.sh", "workloads": {}}
    for wl, kinds in (("head", ["fused_kernel"]), ("cfg2", ["fused_kernel"]),
                      ("cfg5", ["tile_bf16_kernel"])):
        res = {}
        for tag in ("pa", "pb", "pc"):
            d = os.path.join(src, f"{wl}_{tag}")
            if not os.path.isdir(d):
                continue
            vals, dur = load(d)
            for k, cs in vals.items():
                if not any(s in k for s in kinds):
                    continue
                ent = res.setdefault(short(k), {"dispatches": len(dur[k]), "passes": {}})
                ent["passes"][tag] = {c: sum(v) / len(v) for c, v in cs.items()}
                ent["passes"][tag]["duration_us"] = 1e6 * sum(dur[k]) / len(dur[k])
        for name, ent in res.items():
            pa = ent["passes"].get("pa", {})
            dt = pa.get("duration_us", 0) * 1e-6
            g = pa.get("GRBM_GUI_ACTIVE", 0) / 8.0
            dt_ = "bf16" if "bf16" in name else "f32"
            der = {}
            if g and dt:
                der["clock_ghz"] = g / dt / 1e9
                der["busy_from_counter"] = pa["SQ_VALU_MFMA_BUSY_CYCLES"] / (g * 1024)
                der["busy_from_insts"] = pa["SQ_INSTS_MFMA"] * CYC[dt_] / (g * 1024)
                der["flop_from_mops"] = 512 * (pa.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) +
                                               pa.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0))
                der["cu_busy_frac"] = pa["SQ_BUSY_CU_CYCLES"] / (g * 256)
                der["cu_busy_frac_if_quad"] = 4 * pa["SQ_BUSY_CU_CYCLES"] / (g * 256)
            pc = ent["passes"].get("pc", {})
            if pc.get("GRBM_GUI_ACTIVE"):
                der["busy_from_counter_alone"] = pc["SQ_VALU_MFMA_BUSY_CYCLES"] / (
                    pc["GRBM_GUI_ACTIVE"] / 8.0 * 1024)
            if "MfmaUtil" in ent["passes"].get("pb", {}):
                der["MfmaUtil_pct"] = ent["passes"]["pb"]["MfmaUtil"]
            ent["derived"] = der
        out["workloads"][wl] = res
    json.dump(out, open(dst, "w"), indent=1)
    for wl, res in out["workloads"].items():
        for name, ent in res.items():
            print(wl, name, {k: round(v, 4) if isinstance(v, float) else v
                             for k, v in ent["derived"].items()})


if __name__ == "__main__":
    main(*sys.argv[1:])
