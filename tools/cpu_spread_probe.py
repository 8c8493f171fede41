#!/usr/bin/env python3
"""Why the CPU baseline moved between boxes: the same 16 threads of the tuned
port (oracle/cpu_baseline.py, one full configs[1] block in host RAM) bound
three ways on one host, one child process each:

  packed  -- 16 cores filling the fewest L3 domains (CCDs) of one node
  spread  -- 16 cores dealt over every L3 domain of one node
  idlest  -- the 16 idlest cores of the node in core order (round 3's rule)
  spread2 -- 16 cores dealt over every L3 domain of every node, node-major
             (bench.py's rule; spread2:K = its first K CPUs, K threads)
             (threads 0..7 on node 0: the time tiles they first-touch stay local)

A streaming pass is bound by each CCD's link to the IO die, so `packed` is
expected to fall to (CCDs used) x the per-CCD rate.  Prints one JSON line per
binding.  CPU only; no GPU is touched.

  python3 tools/cpu_spread_probe.py [SECONDS [binding,...]]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cpu_baseline as cb  # noqa: E402

GEOM = {"nbit": 8, "nchan_chunk": 256, "nsamp_df": 1}


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    n = cb.effective_cpus()
    picked = cb.pick_cpus(n)
    nd = picked["nodes"][0] if picked["nodes"] else None
    nodes = cb.numa_nodes()
    allowed = set(cb.allowed_cpus())
    cores = {}
    for c in sorted(allowed & nodes.get(nd, allowed)):
        t = "/sys/devices/system/cpu/cpu%d/topology/" % c
        key = ((cb._read(t + "physical_package_id") or "0").strip(), (cb._read(t + "core_id") or str(c)).strip())
        cores.setdefault(key, c)
    reps = sorted(cores.values())
    busy0 = cb.busy_fraction(reps, 0.25)
    doms = {}
    for c in reps:
        doms.setdefault(cb.l3_domain(c), []).append(c)
    spread_l3_node = sorted(cb.spread_l3(sorted(reps, key=lambda c: (busy0.get(c, 0.0), c)), n))
    packed = [c for cs in sorted(doms.values(), key=lambda cs: cs[0]) for c in cs][:n]
    busy = cb.busy_fraction(reps, 0.25)
    idlest = sorted(sorted(reps, key=lambda c: (busy.get(c, 0.0), c))[:n])
    every = {}
    for c in cb.allowed_cpus():
        t = "/sys/devices/system/cpu/cpu%d/topology/" % c
        key = ((cb._read(t + "physical_package_id") or "0").strip(), (cb._read(t + "core_id") or str(c)).strip())
        every.setdefault(key, c)
    spread2 = sorted(cb.spread_l3(sorted(every.values()), n))
    bindings = {"packed": packed, "spread": spread_l3_node, "idlest": idlest, "spread2": spread2}
    if len(sys.argv) > 2:
        want = sys.argv[2].split(",")
        bindings.update({k: None for k in want if k not in bindings})
        bindings = {k: bindings[k] for k in want}
    waits = {}
    for name in list(bindings):   # "spread2:15": the first 15 CPUs of a binding, 15 threads
        if ":" in name:           # "spread2:15:active": and that OpenMP wait policy ("default": unset)
            base, k, *w = name.split(":")
            full = bindings[base] if base != "spread2" else sorted(cb.spread_l3(sorted(every.values()), int(k)))
            bindings[name] = full[:int(k)]
            if w:
                waits[name] = w[0]
    for name, cpus in bindings.items():
        env = cb.child_env(len(cpus), cpus=cpus, wait=waits.get(name, "passive"))
        if waits.get(name) == "default":
            env.pop("OMP_WAIT_POLICY", None)
        r = subprocess.run([sys.executable, os.path.join(REPO, "oracle", "cpu_baseline.py"),
                            json.dumps(GEOM), str(secs), "20181105", "only"], env=env,
                           capture_output=True, text=True, timeout=max(120, secs * 20))
        res = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"error": r.stderr[-300:]}
        print(json.dumps({"binding": name, "cpus": cpus, "node": nd,
                          "nodes": sorted({k for k, cs in nodes.items() for c in cpus if c in cs}),
                          "l3_domains": len({cb.l3_domain(c) for c in cpus}),
                          "l3_domains_on_node": len(doms), "threads": len(cpus),
                          "wait": waits.get(name, "passive"),
                          "value": res.get("value"), "iqr": res.get("iqr"), "passes": res.get("passes"),
                          "iqr_rel": ([round(q / res["value"] - 1, 4) for q in res["iqr"]]
                                      if res.get("value") and res.get("iqr") else None),
                          "throttled_frac": res.get("throttled_frac"),
                          "passes_range": res.get("passes_range"),
                          "cgroup_cpu_stat_delta": res.get("cgroup_cpu_stat_delta"),
                          "error": res.get("error")}), flush=True)


if __name__ == "__main__":
    main()
