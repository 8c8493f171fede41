#!/usr/bin/env python3
"""Summarise rocprofv3 output for the integrate kernel into profiles/.

  tools/pmc_summary.py --config c2 --fetch gpurun_out/pmc_fetch/run_counter_collection.csv \
      --write gpurun_out/pmc_write/run_counter_collection.csv \
      --stats gpurun_out/prof/run_kernel_stats.csv --round r01

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes (they do not fit one TCC pass),
are in KiB, and FETCH_SIZE reports exactly half the bytes of a wide
coalesced streaming read on gfx950, so it is doubled.

Provenance: the summary records the sha256 of the integrate kernel's sources
(bench.KERNEL_SOURCES) the passes ran -- read from the profiled bench.py's own
JSON line (--bench-log; the GPU box has no git) or else hashed here -- and of
the library's gfx950 code objects (bench.device_code_sha), plus the git
commit and the last commit that touched those sources.  bench.py
marks the traffic it quotes STALE when today's sources hash differently.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "b2p_integrate_kernel"
# bytes one integrate launch must read (bench.py configs, one integration)
ALGORITHMIC = {"c2": 1 << 30, "c5": 1 << 32, "bmf": 2818572288,
               # b2p_assemble of a full BMF block: 393216 x (7232 read + 7168 written)
               "assemble": 393216 * (7232 + 7168)}


def counter(path, name, kernel=KERNEL):
    vals = []
    for row in csv.DictReader(open(path)):
        if kernel in row["Kernel_Name"] and row["Counter_Name"] == name:
            vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--stats")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--algorithmic-bytes", type=int, default=0)
    ap.add_argument("--blocks-per-launch", type=int, default=1,
                    help="integrations per integrate launch in the profiled run (bench.py's)")
    ap.add_argument("--kernel", default=KERNEL)
    ap.add_argument("--name", help="file stem instead of the config (e.g. c2_bpl1 for the one-block "
                                    "launch shape; bench.py reads pmc_<config>.json only)")
    ap.add_argument("--bench-log", help="stdout of a profiled bench.py run (its JSON line names the "
                                        "kernel sources' sha256 it ran)")
    a = ap.parse_args()
    sys.path.insert(0, REPO)
    import bench
    sha, sha_from = bench.kernel_sources_sha(), "hashed by tools/pmc_summary.py at summary time"
    dev_sha = bench.device_code_sha()  # the code objects of the library in this tree
    for path in filter(None, [a.bench_log]):
        for ln in open(path):
            if ln.startswith("{"):
                prov = json.loads(ln).get("provenance") or {}
                if prov.get("kernel_sources_sha256"):
                    sha, sha_from = prov["kernel_sources_sha256"], \
                        f"from the profiled run's JSON line ({os.path.relpath(path, REPO)})"
                dev_sha = prov.get("device_code_sha256") or dev_sha

    def git(*args):
        r = subprocess.run(["git", "-C", REPO, *args], capture_output=True, text=True)
        return r.stdout.strip() if r.returncode == 0 else None
    f = counter(a.fetch, "FETCH_SIZE", a.kernel)
    w = counter(a.write, "WRITE_SIZE", a.kernel)
    fetch_kib, write_kib = statistics.median(f), statistics.median(w)
    hbm = int(fetch_kib * 1024 * 2 + write_kib * 1024)
    alg = a.algorithmic_bytes or ALGORITHMIC.get(a.config, 0) * a.blocks_per_launch
    name = a.name or a.config
    fetch_dst = f"profiles/{a.round}_{name}_pmc_fetch.csv"
    write_dst = f"profiles/{a.round}_{name}_pmc_write.csv"
    out = {
        "kernel": a.kernel,
        "config": a.config,
        "launches_measured": len(f),
        "fetch_size_kib_median": fetch_kib,
        "write_size_kib_median": write_kib,
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream under-count, MI355X_MICROARCH.md HBM)",
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": alg or None,
        "blocks_per_launch": a.blocks_per_launch,
        "traffic_over_algorithmic": round(hbm / alg, 4) if alg else None,
        "source": [fetch_dst, write_dst],
        "kernel_sources_sha256": sha,
        "kernel_sources_sha256_from": sha_from,
        "kernel_sources_match_tree": sha == bench.kernel_sources_sha(),
        "device_code_sha256": dev_sha,
        "commit": git("rev-parse", "HEAD"),
        "kernel_sources_commit": git("log", "-1", "--format=%H", "--", *bench.KERNEL_SOURCES),
    }
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    json.dump(out, open(os.path.join(REPO, "profiles", f"pmc_{name}.json"), "w"), indent=1)
    shutil.copy(a.fetch, os.path.join(REPO, fetch_dst))
    shutil.copy(a.write, os.path.join(REPO, write_dst))
    if a.stats:
        shutil.copy(a.stats, os.path.join(REPO, "profiles", f"{a.round}_{name}_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
