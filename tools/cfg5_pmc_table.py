"""Per-kernel HBM traffic of the config-5 bf16 forward from tools/cfg5_pmc.sh's passes.

    python tools/cfg5_pmc_table.py [gpurun_out/cfg5pmc] [profiles/r03_cfg5_pmc.json]

For every kernel of the run: launches, mean duration (p1 kernel trace), FETCH_SIZE and WRITE_SIZE
per launch (KiB units of rocprofv3), read bytes = 2 x FETCH_SIZE (MI355X_MICROARCH.md: on gfx950
FETCH_SIZE tallies wide streaming reads at half their bytes) and raw, write bytes = WRITE_SIZE.
Then per forward: the traffic of the 2K+1 tile launches against the algorithmic bytes of the
API (inputs X, Z0, E0, L0 + every layer's Z, E, L, T + the weights once).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

M, N, K, B = 1024, 4096, 15, 16384


def rows(pat):
    for f in sorted(glob.glob(pat, recursive=True)):
        yield from csv.DictReader(open(f))


def main(src="gpurun_out/cfg5pmc", dst="profiles/r03_cfg5_pmc.json"):
    dur = defaultdict(list)
    for r in rows(os.path.join(src, "p1", "**", "*kernel_trace.csv")):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    ctr = defaultdict(lambda: defaultdict(list))
    for p in ("p2", "p3"):
        for r in rows(os.path.join(src, p, "**", "*counter_collection.csv")):
            ctr[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kern = {}
    for name in sorted(set(dur) | set(ctr)):
        d = dur.get(name, [])
        c = {k: sum(v) / len(v) for k, v in ctr[name].items()}
        e = dict(launches_traced=len(d), mean_ms=1e3 * sum(d) / len(d) if d else None)
        if "FETCH_SIZE" in c:
            e["read_bytes_raw"] = 1024 * c["FETCH_SIZE"]
            e["read_bytes_x2"] = 2 * 1024 * c["FETCH_SIZE"]
        if "WRITE_SIZE" in c:
            e["write_bytes"] = 1024 * c["WRITE_SIZE"]
        kern[name] = e
    tiles = {k: v for k, v in kern.items() if "tile_bf16" in k}
    # per forward: the prologue product once, then G1 and G2 per layer
    per_fwd = {"read_bytes_x2": 0.0, "read_bytes_raw": 0.0, "write_bytes": 0.0, "ms": 0.0}
    for k, v in tiles.items():
        mt = (re.search(r"tile_bf16_kernel<(\d+), (\d+), (\d+), (\d+)>", k) or
              re.search(r"tile_bf16_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", k))
        ph = int(mt.group(3)) if mt else -1
        v["phase"] = {0: "G1 (Z_k)", 1: "G2 (E_k, L_k, T_k+1)", 2: "prologue (T0, Var0)"}.get(ph, "")
        n_per_fwd = 1 if ph == 2 else K
        for f in ("read_bytes_x2", "read_bytes_raw", "write_bytes"):
            per_fwd[f] += n_per_fwd * v.get(f, 0.0)
        per_fwd["ms"] += n_per_fwd * (v["mean_ms"] or 0.0)
    alg = 4 * B * ((M + N + 2 * M) + K * (N + 2 * M) + (K + 1) * M) + 2 * 2 * (K + 1) * M * N
    # the per-layer kernels' own bytes (fp32 state 4 B, packed bf16 operands 2 B per element):
    #   G1 reads Z_{k-1} + packed Var_k, writes Z_k + packed Z_k
    #   G2 reads X, E_{k-1}, L_{k-1} + packed Z_k, writes E_k, L_k, T_{k+1} + packed Var_{k+1}
    # FETCH_SIZE counts the epilogue's 4-B-per-lane loads at their bytes and the operands'
    # 16-B-per-lane LDS-DMA at half (MI355X_MICROARCH.md): reads = raw + half the DMA bytes
    model = {0: dict(dma=2 * M * B, epi_read=4 * N * B, write=4 * N * B + 2 * N * B),
             1: dict(dma=2 * N * B, epi_read=12 * M * B, write=12 * M * B + 2 * M * B)}
    for k, v in tiles.items():
        mt = re.search(r"tile_bf16_kernel<(\d+), (\d+), (\d+), (\d+)>", k)
        ph = int(mt.group(3)) if mt else -1
        if ph in model and "read_bytes_raw" in v:
            mo = model[ph]
            v["model_read_bytes"] = mo["dma"] + mo["epi_read"]
            v["model_write_bytes"] = mo["write"]
            v["read_bytes_corrected"] = v["read_bytes_raw"] + mo["dma"] / 2
            v["achieved_TBps"] = (v["read_bytes_corrected"] + v.get("write_bytes", 0)) / \
                (v["mean_ms"] * 1e-3) / 1e12
    per_fwd["read_bytes_corrected"] = sum(
        (1 if v.get("phase", "").startswith("prologue") else K) *
        v.get("read_bytes_corrected", v.get("read_bytes_raw", 0.0)) for v in tiles.values())
    out = dict(workload=f"v4 bf16 m={M} n={N} K={K} B={B} keep_all=1", kernels=kern,
               per_forward_tile_kernels=per_fwd,
               algorithmic_bytes_per_forward=alg,
               traffic_over_algorithmic=(per_fwd["read_bytes_corrected"] +
                                         per_fwd["write_bytes"]) / alg,
               note="algorithmic = X, Z0, E0, L0 read + every layer's Z, E, L (K) and T (K+1) "
                    "written, fp32, plus the bf16 weights once; the per-layer kernels also re-read "
                    "Z_{k-1}, E_{k-1}, L_{k-1}, X and move the packed bf16 operands")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
