#!/usr/bin/env python3
"""Where a bench region's host time goes beyond its launches (GPU, one call).

bench.py's region is [host clock; K integrations, 4 blocks per launch; wait;
host clock].  Its HIP-event span (set_timing 2) covers the launches and the
closing finalize; the host span adds the first dispatch from an idle GPU and
the wake-up of the final wait.  This times N regions of the driver's
configs[1] shape with three ways to wait, interleaved:
  sync   b2p_sync (flush + hipStreamSynchronize), what bench.py does
  poll   b2p_flush + b2p_fence, then b2p_fence_done polled in a tight loop
  poll2  the same, 20 us sleeps between polls
and prints host-minus-event per region (median, p10, p90) for each.
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "paf-baseband2power_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--regions", type=int, default=400)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process, paf_b2p/_lib.py)
    import paf_b2p
    from paf_b2p import _lib as L
    from paf_b2p.geometry import CONFIGS
    lib = L.lib()
    it = paf_b2p.Integrator(CONFIGS["c2"]["geom"](), device=0)
    blocks = []
    for b in range(4):
        d = it.alloc(it.block_bytes)
        it.fill_synthetic(d, 20181105, 0, b)
        blocks.append(d)
    out = it.alloc(a.steps * it.nout * 4)
    it.sync()

    def wait(mode):
        if mode == "sync":
            it.sync()
            return
        L.check(lib.b2p_flush(it._ctx), it._ctx)
        t = it.fence()
        while True:
            d = lib.b2p_fence_done(it._ctx, C.c_uint64(t))
            if d < 0:
                L.check(d, it._ctx)
            if d:
                return
            if mode == "poll2":
                time.sleep(20e-6)

    def region(mode):
        it.sync()
        t0 = time.perf_counter()
        it.set_timing(2)
        for j in range(0, a.steps, 4):
            it.integrate_n(blocks, out.ptr + j * it.nout * 4, True)
        it.set_timing(0)
        wait(mode)
        return time.perf_counter() - t0

    modes = ["sync", "poll", "poll2"]
    for m in modes:  # warm
        region(m)
    res = {m: [] for m in modes}
    for i in range(a.regions):
        for m in modes:
            it.reset_stats()
            host = region(m)
            ev = it.stats()["kernel_ms"] / 1e3
            res[m].append((host - ev) * 1e6)
    summary = {}
    for m in modes:
        v = sorted(res[m])
        summary[m] = {"host_minus_events_us_median": round(statistics.median(v), 2),
                      "p10": round(v[len(v) // 10], 2), "p90": round(v[9 * len(v) // 10], 2)}
    print(json.dumps({"tool": "sync_probe", "regions": a.regions, "steps": a.steps, "modes": summary}))
    for d in blocks + [out]:
        d.free()
    it.close()


if __name__ == "__main__":
    main()
