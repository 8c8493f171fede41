"""Measure the GPU-resident ring path:

  paf_dfdb -R (replay producer) -> device ring (dada_db -g) ->
  paf_baseband2power (integrates the block in place) -> host ring -> paf_dbdisk

on full-size BMF blocks (8192 frames x 48 chunks, 2.625 GiB), or on
configs[1]-shaped blocks (--layout int8:256, 1 GiB), where the replaying
producer keeps blocks queued and the stage integrates them several per launch
(b2p_integrate_n, b2p_blocks_per_launch).  The producer
re-hands the ring's blocks without rewriting them, so the figure is what the
consumer sustains through the ring: integrate launch + fences + semaphores +
output block per integration.  "steady_*" leaves out the first 8 outputs
(first-launch and producer start-up costs).  Prints one JSON line.

  python tools/bench_ring.py [--blocks 200] [--ndf 8192] [--layout int8:256 --nbufs 8]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import statistics
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "paf-baseband2power_amd"))
from paf_b2p import dada  # noqa: E402

BIN = dada.BIN_DIR
HDR = os.path.join(os.path.dirname(BIN), "conf", "header_baseband2power.txt")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=200)
    ap.add_argument("--ndf", type=int, default=8192)
    ap.add_argument("--nbufs", type=int, default=4)
    ap.add_argument("--layout", default="bmf", choices=["bmf", "int8:256"])
    ap.add_argument("--nsub", type=int, default=1,
                    help="sub-bands served by one stage (-n N: rings key + 0x10*r, spectra gathered)")
    ap.add_argument("--sync", action="store_true",
                    help="paf_baseband2power -S: one block per launch, waited for (the unpipelined baseline)")
    ap.add_argument("--trace", action="store_true", help="paf_baseband2power -V: log every launch / round")
    ap.add_argument("--host", action="store_true",
                    help="host ring instead (the consumer copies every block H2D)")
    a = ap.parse_args()
    if a.layout == "bmf":
        bufsz, nout = a.ndf * 48 * 7168, 336
        samples = a.ndf * 128 * nout * 2  # channels x pols x time, as bench.py counts
    else:  # 256 ch x 2 pol int8, 2^20 samples: configs[1]
        bufsz, nout = 256 * 2 * 2 * (1 << 20), 256
        samples = bufsz // 2
    kin, kout = 0x7e00, 0x7f00
    kins = [kin + 0x10 * r for r in range(a.nsub)]
    for k in kins + [kout]:
        dada.destroy_ring(k)
    d = tempfile.mkdtemp(prefix="bench_ring_")
    for k in kins:
        dada.create_ring(k, a.nbufs, bufsz, device=-1 if a.host else 0)
    dada.create_ring(kout, 8, a.nsub * nout * 4)
    procs = []
    try:
        t0 = time.perf_counter()
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o",
                                   os.path.join(d, "power.dada")], stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b",
                                   f"{kout:x}", "-c", d, "-d", "0", "-f", a.layout]
                                  + (["-n", str(a.nsub)] if a.nsub > 1 else [])
                                  + (["-S"] if a.sync else []) + (["-V"] if a.trace else []),
                                  stderr=subprocess.PIPE)]
        procs += [subprocess.Popen([os.path.join(BIN, "paf_dfdb"), "-a", f"{k:x}", "-b", HDR,
                                    "-R", str(a.blocks), "-f", a.layout]
                                   + (["-r", "20181105"] if a.layout != "bmf" else []), stderr=subprocess.PIPE)
                  for k in kins]
        for p in procs:
            p.wait(timeout=600)
        wall = time.perf_counter() - t0
        errs = [p.stderr.read().decode(errors="replace") for p in procs]
        if any(p.returncode for p in procs):
            print("\n".join(e[-800:] for e in errs), file=sys.stderr)
            return 1
        log = open(os.path.join(d, "paf_baseband2power.log")).read()
        if os.environ.get("BENCH_RING_KEEP_LOG"):
            with open(os.environ["BENCH_RING_KEEP_LOG"], "w") as f:
                f.write(log)
        per = [float(m) for m in re.findall(r"integration \d+: ([0-9.]+) ms", log)]
        m = re.search(r"FINISH PAF_PROCESS: (\d+) integrations.* ([0-9.]+) s from the first", log)
        steady = per[a.nbufs + 1:] or per
        med = statistics.median(steady) if steady else None  # the pipelined path logs no per-block time
        launches = [int(x) for x in re.findall(r"(?:launch|round) \d+: (\d+) integration", log)]
        n_int, el = (int(m.group(1)), float(m.group(2))) if m else (0, 0.0)
        ms = re.search(r"([0-9.]+) s for the last (\d+)", log)
        el_s, n_s = (float(ms.group(1)), int(ms.group(2))) if ms else (0.0, 0)
        print(json.dumps({
            "path": ("host ring -> paf_baseband2power (pinned H2D, overlapped)" if a.host else
                     "device ring (dada_db -g) -> paf_baseband2power in place"),
            "layout": a.layout, "nbufs": a.nbufs, "nsub": a.nsub,
            "block_bytes": bufsz, "blocks": a.blocks, "integrations_logged": len(per),
            "launches_logged": len(launches),
            "max_blocks_per_launch_logged": max(launches) if launches else None,
            "consumer_ms_per_block_median": round(med, 3) if med else None,
            # host ring: the stage logs every block (asked -> output, ~5 us
            # between blocks); the median leaves out the last blocks, which
            # overlap the replaying producer's exit and copy 15-20 % slower
            "consumer_GBps_median": round(a.nsub * bufsz / (med * 1e-3) / 1e9, 1) if med else None,
            "ms_per_block": round(el / n_int * 1e3, 4) if n_int else None,
            "consumer_elapsed_s": el,
            "ring_Msamples_s": round(a.nsub * n_int * samples / el / 1e6, 1) if el else None,
            "ring_GBps": round(a.nsub * n_int * bufsz / el / 1e9, 1) if el else None,
            "steady_blocks": n_s,
            "steady_ms_per_block": round(el_s / n_s * 1e3, 4) if n_s else None,
            "steady_Msamples_s": round(a.nsub * n_s * samples / el_s / 1e6, 1) if n_s else None,
            "steady_GBps": round(a.nsub * n_s * bufsz / el_s / 1e9, 1) if n_s else None,
            "wall_s_incl_startup": round(wall, 2),
        }), flush=True)
        return 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in kins + [kout]:
            dada.destroy_ring(k)


if __name__ == "__main__":
    sys.exit(main())
