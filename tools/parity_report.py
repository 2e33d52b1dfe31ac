"""Summarise the parity log of a GPU test run into profiles/r03_parity.json.

    DLADMM_PARITY_JSON=gpurun_out/parity_log.json python -m pytest tests -m gpu ...
    python tools/parity_report.py gpurun_out/parity_log.json [profiles/r03_parity.json]

Every error the parity tests checked (tests/parity.py: golden fixtures, oracle cases, the
BASELINE config workloads, the bf16 fixtures) is grouped by (case, path) with the worst error, the
worst error as a fraction of its bar (err / tol), and -- where the bar is the gap bound -- the
worst err / gap (how far from the reference's own fp32 rounding the GPU result is).
"""
import json
import sys
from collections import defaultdict


def main(src, dst="profiles/r03_parity.json"):
    log = json.load(open(src))
    groups = defaultdict(list)
    for r in log:
        groups[(r["case"], r["path"])].append(r)
    rows = []
    for (case, path), rs in sorted(groups.items()):
        worst = max(rs, key=lambda r: r["err"] / r["tol"])
        f32 = [r for r in rs if "err32" in r]
        row = dict(case=case, path=path, checks=len(rs),
                   max_err_over_tol=worst["err"] / worst["tol"], worst=worst["what"],
                   passed=all(r["err"] <= r["tol"] for r in rs))
        if f32:   # the fp32 bar: err32 vs the reference's fp32, err64 vs the exact result
            row.update(max_err_vs_ref32=max(r["err32"] for r in f32),
                       max_err_vs_ref64=max(r["err64"] for r in f32),
                       max_ref_gap=max(r["gap"] for r in f32),
                       max_err64_over_gap=max((r["err64"] / r["gap"] for r in f32
                                               if r["gap"] > 0), default=None),
                       checks_passed_by_gap_clause=sum(r["by"] != "1e-5" for r in f32))
        else:
            row.update(max_err=max(r["err"] for r in rs), worst_tol=worst["tol"])
        rows.append(row)
    by_path = defaultdict(lambda: dict(cases=0, checks=0, max_err_over_tol=0.0, failed=0))
    for r in rows:
        b = by_path[r["path"]]
        b["cases"] += 1
        b["checks"] += r["checks"]
        b["max_err_over_tol"] = max(b["max_err_over_tol"], r["max_err_over_tol"])
        b["failed"] += 0 if r["passed"] else 1
    out = dict(
        bar="fp32 paths (f32 fused, split-f16, per-layer), per layer, norm-relative: <= 1e-5 "
            "vs the reference's fp32 output or the exact (fp64) result, or <= 2 x the reference "
            "algorithm's own fp32-vs-fp64 gap vs the exact result (tests/parity.py); bf16: <= max(1e-5, 0.25 s_k, 2 d_k) vs "
            "the reference with bf16-operand GEMMs and 1e-5 + max(1.25 s_k, s_k + that) vs fp32 "
            "(tests/test_gpu_bf16.py); max_err_over_tol <= 1 = passed",
        source=src, summary_by_path=dict(by_path), cases=rows)
    json.dump(out, open(dst, "w"), indent=1)
    for p, b in sorted(by_path.items()):
        print(f"{p:8s} cases {b['cases']:4d} checks {b['checks']:6d} "
              f"worst err/tol {b['max_err_over_tol']:.3f} failed {b['failed']}")


if __name__ == "__main__":
    main(*sys.argv[1:])
