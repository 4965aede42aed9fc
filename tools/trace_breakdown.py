#!/usr/bin/env python3
"""Where a launch's GPU time goes, from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv).

    python3 tools/trace_breakdown.py <kernel_trace.csv> [--tail-frac 0.4] [--per-launch-kernel k_env_steps_sync]

Kernels are grouped by category (step kernel, admission, fused actor, torch GEMM, torch elementwise /
other).  Over the last `tail-frac` of the trace's time span (the timed replays, after the warm-up) it
reports per category: dispatches, total and mean kernel time, time per step-kernel launch; the span's
wall time, the time covered by at least one kernel (union of intervals) and the idle gaps, and how
much of the span two or more kernels overlap (concurrent stream groups)."""
import argparse
import csv
import json
import re

CATS = [("step kernel", r"k_env_steps"), ("admission", r"k_policy_admit"), ("fused actor", r"k_policy_actor"),
        ("policy head + scatter", r"k_policy_apply"), ("torch GEMM", r"Cijk|gemm|Gemm|GEMM|hipblaslt|rocblas"),
        ("torch elementwise", r"elementwise|vectorized|at::native|triton|reduce"), ("other", r".")]


def category(name):
    for c, rx in CATS:
        if re.search(rx, name):
            return c
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail-frac", type=float, default=0.4)
    ap.add_argument("--per-launch-kernel", default="k_env_steps")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    cut = t1 - (t1 - t0) * a.tail_frac
    sel = [r for r in rows if r[0] >= cut]
    span = max(r[1] for r in sel) - sel[0][0]
    per = {}
    for s, e, n in sel:
        c = category(n)
        d = per.setdefault(c, {"dispatches": 0, "total_us": 0.0, "names": {}})
        d["dispatches"] += 1
        d["total_us"] += (e - s) / 1e3
        d["names"][n[:90]] = d["names"].get(n[:90], 0) + 1
    launches = sum(1 for r in sel if a.per_launch_kernel in r[2])
    # union of busy intervals, and the time covered by >= 2 kernels
    ev = sorted([(s, 1) for s, _, _ in sel] + [(e, -1) for _, e, _ in sel])
    busy = over = 0
    depth, last = 0, ev[0][0]
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            over += t - last
        depth += d
        last = t
    for d in per.values():
        d["mean_us"] = d["total_us"] / d["dispatches"]
        d["us_per_step_kernel_launch"] = d["total_us"] / launches if launches else None
        d["names"] = dict(sorted(d["names"].items(), key=lambda kv: -kv[1])[:6])
    out = {"trace": a.trace, "window": f"last {a.tail_frac:.0%} of the trace's span", "dispatches": len(sel),
           "step_kernel_launches": launches, "span_us": span / 1e3, "busy_us": busy / 1e3,
           "idle_us": (span - busy) / 1e3, "overlapped_us": over / 1e3,
           "span_us_per_step_kernel_launch": span / 1e3 / launches if launches else None,
           "categories": dict(sorted(per.items(), key=lambda kv: -kv[1]["total_us"]))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
