#!/usr/bin/env python3
"""Cut a rocprofv3 kernel trace of one bench.py run into that run's legs.

bench.py's default run issues integrate launches of two shapes: the
headline's (queued blocks, e.g. 4 x 1 GiB per launch for configs[1]) and the
one-block-per-launch leg beside it.  rocprofv3 --stats averages them
together under one kernel name, so its figure matches neither.  The bench
line lists its integrate launches in issue order per phase
(roofline.launch_phases); this slices the trace's integrate dispatches
(ordered by dispatch id) by those counts and reports each leg's launch
durations, and for the headline the HBM fraction they imply.  The secondary
layouts (`secondary` in the line) follow, each as its warm-up region and its
timed launches, with their own HBM fractions.

  tools/trace_legs.py --trace gpurun_out/prof/run_kernel_trace.csv \\
      --bench-log gpurun_out/prof.log [--out profiles/r04_c2_kernel_legs.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics

KERNEL = "b2p_integrate_kernel"


def legs(trace_path: str, line: dict) -> dict:
    rows = [r for r in csv.DictReader(open(trace_path)) if KERNEL in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]  # us
    names = [r["Kernel_Name"] for r in rows]
    rf = line["roofline"]
    phases = rf.get("launch_phases") or []
    # the secondary legs (bench.py secondary_leg) run after those phases, in
    # the line's order: one untimed warm-up region, then the timed regions
    sec = []
    for name, v in (line.get("secondary") or {}).items():
        r = v.get("roofline") or {}
        timed = (r.get("hbm") or {}).get("launches_timed") if r.get("bound") == "pcie" else r.get("launches_timed")
        if timed and v.get("timed_regions"):
            sec.append((f"secondary.{name}", timed // v["timed_regions"], timed, r))
    want = sum(c for _, c in phases) + sum(w + t for _, w, t, _ in sec)
    out = {"trace": trace_path, "integrate_dispatches": len(dur), "launches_in_bench_line": want,
           "counts_agree": len(dur) == want, "legs": {}}
    phases = list(phases)
    for name, w, t, _ in sec:
        phases += [(name + "_warmup", w), (name, t)]
    i = 0
    for name, c in phases:
        d = dur[i:i + c]
        kn = sorted(set(names[i:i + c]))
        i += c
        if not d:
            continue
        out["legs"][name] = {"launches": len(d), "kernels": kn, "avg_us": round(statistics.fmean(d), 2),
                             "median_us": round(statistics.median(d), 2),
                             "min_us": round(min(d), 2), "max_us": round(max(d), 2)}
    h = out["legs"].get("headline")
    if h:
        b = rf["algorithmic_bytes_per_launch"]
        h["algorithmic_bytes_per_launch"] = b
        h["frac_of_8TBps"] = round(b / (h["avg_us"] * 1e-6) / 1e9 / rf["peak"], 4)
        h["bench_line_avg_launch_us"] = rf["avg_launch_us"]
        h["bench_line_kernel_only_us"] = rf.get("kernel_only_us")
    for name, _, _, r in sec:
        leg = out["legs"].get(name)
        if leg and r.get("bound") == "hbm":
            b = r["algorithmic_bytes_per_launch"]
            leg["frac_of_8TBps"] = round(b / (leg["avg_us"] * 1e-6) / 1e9 / r["peak"], 4)
            leg["bench_line_avg_launch_us"] = r.get("avg_launch_us")
    one = out["legs"].get("one_per_launch")
    if one:
        b1 = line["config"]["bytes_per_integration"]
        one["frac_of_8TBps"] = round(b1 / (one["avg_us"] * 1e-6) / 1e9 / rf["peak"], 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--bench-log", required=True, help="stdout of the profiled bench.py (its JSON line)")
    ap.add_argument("--out")
    a = ap.parse_args()
    line = next(json.loads(ln) for ln in open(a.bench_log) if ln.startswith("{"))
    res = legs(a.trace, line)
    txt = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
