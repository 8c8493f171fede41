#!/usr/bin/env python3
"""Launch-shape sweep for the integrate kernel, interleaved in ONE process
(cdna_hip_programming.md §5.4 rule 24): every variant is opened as its own
context (an explicit b2p_tuning_t through b2p_open_tuned) and timed with dispatch-packet
events over the same rotating HBM blocks, round after round.

    python3 tools/tune.py --config c2 --rounds 3 > gpurun_out/tune_c2.json
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "paf-baseband2power_amd"))

import paf_b2p  # noqa: E402
from paf_b2p.geometry import CONFIGS  # noqa: E402

def frame_variants(threads):
    """multi-column frames (BMF): exact workgroup sizes"""
    for t, u, il in itertools.product(threads, [4, 8, 16], [0, 1]):
        yield {"max_threads": 1024, "threads": t, "unroll": u, "nontemporal": 1,
               "wg_per_cu": 0, "interleave": il, "fuse": 0}


def variants(quick: bool):
    threads = [256, 512, 1024]
    unroll = [4, 8, 16]
    per_cu = [0, 1, 2, 4]  # 0: the planner's default
    for t, u, p, il, fu in itertools.product(threads, unroll, per_cu, [0, 1], [0, 1]):
        if quick and (p not in (0, 1) or u == 16):
            continue
        yield {"max_threads": t, "unroll": u, "nontemporal": 1, "wg_per_cu": p,
               "interleave": il, "fuse": fu}


def open_variant(geom, v):
    """one context per variant, its b2p_tuning_t passed explicitly"""
    return paf_b2p.Integrator(geom, tuning=v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--case", default="", help="a tools/perf_matrix.py layout by name (e.g. 'int8 336ch') instead of --config")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--launches", type=int, default=12)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--threads", default="", help="comma list of exact workgroup sizes (b2p_tuning_t.threads, BMF)")
    a = ap.parse_args()
    if a.case:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from perf_matrix import CASES
        geom = dict(CASES)[a.case]()
    else:
        geom = CONFIGS[a.config]["geom"]()
    base = paf_b2p.Integrator(geom)
    bb = base.block_bytes
    blocks = []
    for b in range(4):
        d = base.alloc(bb)
        base.fill_synthetic(d, 20181105, 0, b)
        blocks.append(d)
    base.sync()
    ref = None
    vs = (list(frame_variants([int(x) for x in a.threads.split(",")])) if a.threads
          else list(variants(a.quick)))
    res = {i: [] for i in range(len(vs))}
    info = {}
    for _ in range(a.rounds):
        for i, v in enumerate(vs):
            it = open_variant(geom, v)
            info[i] = {"threads": it.info.threads, "grid": it.info.columns * it.info.row_groups}
            dout = it.alloc(it.nout * 4)

            def one(k):
                if v["fuse"]:
                    it.integrate(blocks[k % 4], dout.ptr, True)
                else:
                    it.push(blocks[k % 4])
                    it.finish_async(dout.ptr, True)
            for k in range(2):
                one(k)
            it.sync()
            it.set_timing(2)  # region timing: end-to-end time per integration
            for k in range(a.launches):
                one(k)
            it.set_timing(0)
            it.sync()
            out = it.download(dout).view("float32")
            dout.free()
            st = it.stats()
            if ref is None:
                ref = out
            assert (out.view("uint32") == ref.view("uint32")).all(), f"variant {v} differs"
            res[i].append(st["kernel_ms"] / st["launches"])
            it.close()
    rows = []
    for i, v in enumerate(vs):
        ms = statistics.median(res[i])
        rows.append({**v, **info[i], "median_us": round(ms * 1e3, 2),
                     "min_us": round(min(res[i]) * 1e3, 2), "GBps": round(bb / (ms * 1e-3) / 1e9, 1)})
    rows.sort(key=lambda r: r["median_us"])
    print(json.dumps({"config": a.case or a.config, "block_bytes": bb, "rounds": a.rounds, "variants": rows},
                     indent=1))
    for d in blocks:
        d.free()
    base.close()


if __name__ == "__main__":
    main()
