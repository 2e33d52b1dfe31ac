"""Summarise the rocprofv3 passes of tools/profile.sh for the fused kernel.

    python tools/prof_summary.py gpurun_out/prof profiles/<round>  [--workload "..."]

Writes <out>_kernel_stats.csv (copy of the kernel-trace --stats summary), <out>_pmc.json
(per-launch counter means for the fused kernel) and updates profiles/traffic.json, which bench.py
reads for roofline.traffic.  bench.py also launches the fused kernel for its config-2 and config-3
lines, so only launches with the headline's grid (--grid, default 262,144 work-items = B 65,536 /
16 columns per wave x 64 lanes) are averaged; <out>_headline_stats.csv restates rocprofv3's
--stats row for those launches alone (its own summary averages every grid of one kernel name).  HBM bytes follow MI355X_MICROARCH.md section HBM: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half of the bytes of WIDE (16 B/lane) coalesced
reads, so the 16-B LDS-DMA weight stream is doubled while the kernel's 4-B-per-lane loads are not
(their correction is uncalibrated -- both bounds are recorded).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

KERNEL = "fused_kernel"
GRID = 262144


def grid_of(r):
    return int(r["Grid_Size"] if "Grid_Size" in r else r["Grid_Size_X"])


def counters(d):
    agg = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"] and grid_of(r) == GRID:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def durations(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"] and grid_of(r) == GRID:
                out.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return out


def main():
    global GRID
    src, out = sys.argv[1], sys.argv[2]
    if "--grid" in sys.argv:
        GRID = int(sys.argv[sys.argv.index("--grid") + 1])
    wl = "v4 m=256 n=512 K=15 B=65536 keep_all=1"
    if "--workload" in sys.argv:
        wl = sys.argv[sys.argv.index("--workload") + 1]
    os.makedirs(os.path.dirname(out), exist_ok=True)
    ks = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    if ks:
        shutil.copy(ks[0], out + "_kernel_stats.csv")
    res = {"workload": wl, "grid_work_items": GRID}
    for name in ("pmc_fetch", "pmc_write", "pmc_sq"):
        c, n = counters(os.path.join(src, name))
        dur = durations(os.path.join(src, name))
        res[name] = {"counters_mean_per_launch": c, "launches": n,
                     "duration_s_mean": sum(dur) / max(len(dur), 1)}
    fetch_kib = res["pmc_fetch"]["counters_mean_per_launch"].get("FETCH_SIZE")
    write_kib = res["pmc_write"]["counters_mean_per_launch"].get("WRITE_SIZE")
    sq = res["pmc_sq"]["counters_mean_per_launch"]
    if fetch_kib is not None and write_kib is not None:
        rd_raw = fetch_kib * 1024
        res["hbm_read_bytes_raw"] = rd_raw
        res["hbm_read_bytes_x2"] = 2 * rd_raw
        res["hbm_write_bytes"] = write_kib * 1024
        # bench's roofline.traffic: raw FETCH (4-B loads dominate the kernel's reads) + WRITE
        res["hbm_bytes_per_launch"] = rd_raw + write_kib * 1024
        res["hbm_bytes_per_launch_upper"] = 2 * rd_raw + write_kib * 1024
    if "GRBM_GUI_ACTIVE" in sq:
        dur = res["pmc_sq"]["duration_s_mean"]
        res["clock_ghz_est"] = sq["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9
        if "SQ_VALU_MFMA_BUSY_CYCLES" in sq:
            # SIMD-cycles of MFMA / (1024 SIMDs x per-XCD active cycles)
            res["mfma_busy_frac"] = sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * sq["GRBM_GUI_ACTIVE"] / 8)
    # kernel-trace durations (the first launch is a cold warmup: bench.py's timed region excludes
    # it) beside the bench line of the same profiled run, whose kernel_ms is measured with HIP
    # events on the launch stream
    import statistics
    kt = durations(os.path.join(src, "kt"))
    if kt:
        res["trace"] = {"launches": len(kt), "mean_ms_all": 1e3 * statistics.mean(kt),
                        "mean_ms_excl_first": 1e3 * statistics.mean(kt[1:] or kt),
                        "median_ms": 1e3 * statistics.median(kt)}
        ns = [int(round(t * 1e9)) for t in kt]
        with open(out + "_headline_stats.csv", "w") as f:
            f.write('"Name","Grid_Size","Calls","TotalDurationNs","AverageNs","MinNs","MaxNs",'
                    '"AverageNs_excl_first"\n')
            f.write(f'"{KERNEL} (headline launches)",{GRID},{len(ns)},{sum(ns)},'
                    f'{sum(ns) / len(ns):.1f},{min(ns)},{max(ns)},'
                    f'{sum(ns[1:]) / max(len(ns) - 1, 1):.1f}\n')
    for line in open(os.path.join(src, "kt.log"), errors="replace") if os.path.exists(
            os.path.join(src, "kt.log")) else []:
        if line.startswith('{"metric"'):
            b = json.loads(line)
            res["bench_line_same_run"] = {"value": b["value"], "kernel_ms_hip_events":
                                          b["roofline"]["kernel_ms"], "frac": b["roofline"]["frac"]}
    json.dump(res, open(out + "_pmc.json", "w"), indent=1)
    tr = {k: res[k] for k in ("workload", "hbm_bytes_per_launch", "hbm_bytes_per_launch_upper",
                              "hbm_read_bytes_raw", "hbm_write_bytes") if k in res}
    tr["source"] = os.path.basename(out) + "_pmc.json"
    json.dump(tr, open(os.path.join(os.path.dirname(out), "traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
