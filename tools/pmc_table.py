"""Per-launch means of the rocprofv3 PMC passes of tools/x3_pmc.sh for one kernel.

    python tools/pmc_table.py gpurun_out/prof fused_x3_kernel [out.json]

Prints counter, mean per launch, and the derived shares: SQ_* wave-cycle counters are
quad-cycles summed over waves (SQ_WAVE_CYCLES = their total); the clock estimate is
GRBM_GUI_ACTIVE / 8 XCDs / kernel duration.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    src, kern = sys.argv[1], sys.argv[2]
    agg, dur = defaultdict(list), []
    for f in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"),
                              recursive=True)):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(src, "p1", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    c = {k: sum(v) / len(v) for k, v in agg.items()}
    res = {"kernel": kern, "counters_mean_per_launch": c}
    if dur:
        res["duration_ms_profiled"] = 1e3 * sum(dur) / len(dur)
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        res["share_of_wave_cycles"] = {k: v / wc for k, v in c.items()
                                       if k.startswith(("SQ_WAIT", "SQ_ACTIVE_INST"))}
    if dur and "GRBM_GUI_ACTIVE" in c:
        res["clock_ghz_est"] = c["GRBM_GUI_ACTIVE"] / 8 / (sum(dur) / len(dur)) / 1e9
    if "FETCH_SIZE" in c:
        res["hbm_read_bytes_x2"] = 2 * 1024 * c["FETCH_SIZE"]
    if "WRITE_SIZE" in c:
        res["hbm_write_bytes"] = 1024 * c["WRITE_SIZE"]
    if "TCC_HIT_sum" in c:
        res["l2_hit_rate"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1)
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
