#!/usr/bin/env python3
"""Every bench line's roofline against the profiles it can be recomputed from.

    python3 tools/roofline_sources.py <bench json line file> <out json> line=<rocprof stats csv>[,<kernel trace csv>] ...

For each bench line (c3 = the headline, c5, c3_f64, c5_torch_actor) given as line=<run_kernel_stats.csv>
of a rocprofv3 --kernel-trace --stats run of THAT line's launch shape: the step kernel's rocprof
average and minimum per launch, the bench's HIP-event median (the statistic its roofline.achieved
uses), each per step, the algorithmic bytes per launch, the achieved GB/s and HBM fraction from each
statistic, and the PMC summary (profiles/*pmc*.json of the same launch configuration, as bench.py's
latest_pmc finds it) whose HBM bytes the line reports as `traffic`."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

KEYS = {"c3": None, "c5": "c5", "c3_f64": "c3_f64", "c5_torch_actor": "c5_torch_actor"}


def kernel_stats(path, name):
    for r in csv.DictReader(open(path)):
        if name in r["Name"]:
            return {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6, "min_ms": float(r["MinNs"]) / 1e6,
                    "max_ms": float(r["MaxNs"]) / 1e6}
    return None


def timed_launches(trace, name, n):
    """Average and min (ms) of the last n dispatches of the kernel in a rocprofv3 kernel-trace CSV: the
    bench's timed launches (they come last)."""
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace))
                  if name in r["Kernel_Name"])
    d = [(e - s) / 1e6 for s, e in rows[-n:]]
    return {"launches": len(d), "avg_ms": sum(d) / len(d), "min_ms": min(d), "max_ms": max(d)} if d else None


def main():
    line = open(sys.argv[1]).read().strip().splitlines()[-1]
    b = json.loads(line)
    out = {"what": __doc__.split("\n\n")[0], "bench": os.path.relpath(sys.argv[1], ROOT), "lines": {}}
    for arg in sys.argv[3:]:
        key, paths = arg.split("=", 1)
        path, trace = (paths.split(",", 1) + [None])[:2]
        d = b if KEYS[key] is None else b[KEYS[key]]
        rl, cfg = d["roofline"], d["config"]
        chunk = cfg["fused_steps_per_launch"]
        ks = kernel_stats(path, "k_env_steps_sync")
        alg = rl["algorithmic_bytes_per_launch"]
        prec = 64 if key == "c3_f64" else 32
        serve = "queue" if key == "c5_torch_actor" else "kernel"
        n_env = cfg["envs_per_gpu"] // cfg.get("stream_groups", 1)
        pmc = bench.latest_pmc(prec, cfg["mode"], n_env, chunk, serve)
        ent = {"kernel": rl["kernel"], "steps_per_launch": chunk, "algorithmic_bytes_per_launch": alg,
               "bench": {"statistic": rl.get("kernel_ms_statistic"), "kernel_ms_per_launch": rl["kernel_ms_per_launch"],
                         "us_per_step": rl["kernel_ms_per_launch"] * 1e3 / chunk, "achieved_gbs": rl["achieved"],
                         "frac": rl["frac"], "line_ms_per_step_us": d["ms_per_step"] * 1e3},
               "rocprof": None, "pmc": None}
        if ks:
            ent["rocprof"] = {"file": os.path.relpath(path, ROOT), "calls_all_launches_incl_warmup": ks["calls"],
                              "avg_ms": ks["avg_ms"], "min_ms": ks["min_ms"],
                              "avg_us_per_step": ks["avg_ms"] * 1e3 / chunk, "min_us_per_step": ks["min_ms"] * 1e3 / chunk,
                              "achieved_gbs_from_avg": alg / (ks["avg_ms"] * 1e-3) / 1e9,
                              "frac_from_avg": alg / (ks["avg_ms"] * 1e-3) / 1e9 / bench.HBM_PEAK_GBS,
                              "avg_vs_bench_kernel_ms": ks["avg_ms"] / rl["kernel_ms_per_launch"] - 1.0}
        if pmc:
            ent["pmc"] = {"source": pmc.get("source"), "round": pmc.get("round"), "hbm_bytes_per_launch": pmc["hbm_bytes_per_launch"],
                          "traffic_over_algorithmic": pmc["hbm_bytes_per_launch"] / alg,
                          "kernel_ms_per_launch_under_pmc": pmc.get("kernel_ns_per_launch", 0) / 1e6,
                          "per_wave_step": pmc.get("per_wave_step")}
        if trace and os.path.exists(trace):
            n_timed = d["steps"] // chunk
            tl = timed_launches(trace, "k_env_steps_sync", n_timed)
            if tl:
                ent["rocprof_timed_launches"] = dict(tl, avg_us_per_step=tl["avg_ms"] * 1e3 / chunk,
                                                     min_us_per_step=tl["min_ms"] * 1e3 / chunk,
                                                     frac_from_avg=alg / (tl["avg_ms"] * 1e-3) / 1e9 / bench.HBM_PEAK_GBS,
                                                     how="the last steps/chunk dispatches of the kernel trace (the timed launches)")
        out["lines"][key] = ent
    with open(sys.argv[2], "w") as f:
        json.dump(out, f, indent=1)
    for k, e in out["lines"].items():
        r = e["rocprof"] or {}
        print(f"{k}: bench {e['bench']['us_per_step']:.3f} us/step (frac {e['bench']['frac']:.4f}); rocprof avg "
              f"{r.get('avg_us_per_step', float('nan')):.3f} min {r.get('min_us_per_step', float('nan')):.3f}; "
              f"traffic/alg {((e['pmc'] or {}).get('traffic_over_algorithmic') or float('nan')):.4f}")


if __name__ == "__main__":
    main()
