"""Integrate-kernel throughput over the layouts the path supports, at full
integration size (1024 x 1024 samples), HBM-resident, region-timed:
int8 / int16 LE / int16 BE (BMF), 1 or 2 output pols, narrow and wide
channel counts.  One JSON line per case; a slow corner shows up as a low
GB/s against the ~7 TB/s of the headline layouts.

  python tools/perf_matrix.py [--steps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "paf-baseband2power_amd"))
import torch  # noqa: E402,F401  (one HIP runtime per process)

import paf_b2p  # noqa: E402
from paf_b2p.geometry import generic_geom, bmf_geom, make_geom  # noqa: E402

CASES = [
    ("int8 256ch (configs[1])", lambda **k: generic_geom(256, **k)),
    ("int8 1024ch (configs[2..4])", lambda **k: generic_geom(1024, **k)),
    ("int8 64ch", lambda **k: generic_geom(64, **k)),
    ("int8 336ch", lambda **k: generic_geom(336, **k)),
    ("int16 LE 256ch", lambda **k: generic_geom(256, nbit=16, **k)),
    ("int16 LE 48ch", lambda **k: generic_geom(48, nbit=16, **k)),
    ("int16 BE BMF 48x7", lambda **k: bmf_geom(**k)),
    ("int8 TFTFP 32x8", lambda **k: make_geom(nbit=8, nchunk=32, nsamp_df=128, nchan_chunk=8, **k)),
    ("int16 BE TFTFP 8x8", lambda **k: make_geom(nbit=16, big_endian=1, nchunk=8, nsamp_df=128,
                                                 nchan_chunk=8, **k)),
]


KEEP = []  # --keep: buffers are never freed (diagnostic: no hipFree between runs)


def run(name, geom, steps, keep=False, tuning=None, multi=1):
    """steps integrations region-timed; multi > 1: in launches of `multi`
    integrations each (b2p_integrate_n), steps rounded up to a multiple"""
    it = paf_b2p.Integrator(geom, tuning=tuning)
    bb = it.block_bytes
    blocks = []
    for b in range(2):
        d = it.alloc(bb)
        it.fill_synthetic(d, 20181105, 0, b)
        blocks.append(d)
    steps = -(-steps // multi) * multi
    out = it.alloc(it.nout * 4 * steps)

    def launch(k):  # integrations k .. k + multi - 1
        dst = out.ptr + k * it.nout * 4
        if multi == 1:
            it.integrate(blocks[k % 2], dst, True)
        else:
            it.integrate_n([blocks[(k + j) % 2] for j in range(multi)], dst, True)
    for k in range(0, 3 * multi, multi):
        launch(0)
    it.sync()
    it.reset_stats()
    it.set_timing(2)
    for k in range(0, steps, multi):
        launch(k)
    it.set_timing(0)
    it.sync()
    st = it.stats()
    us = st["kernel_ms"] / steps * 1e3
    res = {"case": name, "npol_out": geom.npol_out, "bytes": bb, "us_per_integration": round(us, 1),
           "GBps": round(bb / us / 1e3, 1), "threads": it.info.threads, "unroll": it.info.unroll,
           "row_groups": it.info.row_groups, "columns": it.info.columns, "blocks_per_launch": multi}
    if keep:
        KEEP.append((it, blocks, out))
        return res
    for d in blocks + [out]:
        d.free()
    it.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="", help="substring of the case names to run")
    ap.add_argument("--npol-out", type=int, default=0, help="1 or 2 (default both)")
    ap.add_argument("--repeat", type=int, default=1, help="run each case this many times")
    ap.add_argument("--sleep", type=float, default=2.0,
                    help="idle seconds before each run: the previous run freed GiBs, and launches "
                         "in the next seconds run 2-8 %% slower (profiles/archive/r01_free_effect.txt)")
    ap.add_argument("--keep", action="store_true", help="never free a run's buffers")
    ap.add_argument("--multi", type=int, default=1,
                    help="integrations per launch (b2p_integrate_n), e.g. 8")
    ap.add_argument("--tuning", default="", help='b2p_tuning_t fields as JSON, e.g. \'{"unroll": 8}\'')
    a = ap.parse_args()
    knobs = json.loads(a.tuning) if a.tuning else None
    for name, mk in CASES:
        if a.only and a.only not in name:
            continue
        for npo in ((a.npol_out,) if a.npol_out else (1, 2)):
            for rep in range(a.repeat):
                if a.sleep > 0:
                    time.sleep(a.sleep)
                r = run(name, mk(npol_out=npo), a.steps, a.keep, knobs, a.multi)
                if knobs:
                    r["tuning"] = knobs
                if a.repeat > 1:
                    r["rep"] = rep
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
