"""Measure b2p_assemble: a raw BMF data-frame stream
(7232-B frames with 64-B headers, capture.c:527-547) scattered into a
payload-only TFTFP block in HBM, then the same block integrated.

Prints one JSON line per arrival order:
  assemble GB/s  = ndf * (7232 read + 7168 written) / kernel time
  stream Msamples/s = samples of the block / (assemble + integrate) time

Timing: one HIP event pair on the integrator's stream around K launches
(b2p_set_timing mode 2).  Usage:
  python tools/bench_assemble.py [--ndf 8192] [--steps 10] [--warmup 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "paf-baseband2power_amd"))
import paf_b2p  # noqa: E402
from paf_b2p import dada  # noqa: E402

HBM_PEAK_GBS = 8000.0
DF, HDR, PAY = 7232, 64, 7168


def build_stream(block: np.ndarray, nchunk: int, ref_idf: int, ref_sec: int, order: np.ndarray):
    """host DF stream for a payload-only block (the frames paf_dfgen writes)"""
    nf = block.size // (nchunk * PAY)
    n = nf * nchunk
    dfs = np.empty((n, DF), dtype=np.uint8)
    pay = block.reshape(n, PAY)
    hdr = np.empty((n, HDR), dtype=np.uint8)
    ref = dada.DfHdr(1, ref_idf, ref_sec, 0, 0, 0.0)
    for t in range(nf):
        r = dada.df_ref_advance(ref, t)
        for c in range(nchunk):
            hdr[t * nchunk + c] = np.frombuffer(
                dada.df_encode(r.idf, r.sec, 1, 0, 0, 1300.0 + c), dtype=np.uint8)
    dfs[:, :HDR] = hdr[order]
    dfs[:, HDR:] = pay[order]
    chunk = (order % nchunk).astype(np.uint8)
    return dfs, chunk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndf", type=int, default=8192, help="frames per block (capture.h:20-28)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--order", choices=("both", "tm", "shuffled"), default="both")
    ap.add_argument("--grid", type=int, default=0, help="workgroup cap (b2p_tuning_t.assemble_grid)")
    a = ap.parse_args()
    nchunk = 48
    geom = paf_b2p.bmf_geom(nsamp_int=a.ndf * 128)
    it = paf_b2p.Integrator(geom, tuning={"assemble_grid": a.grid} if a.grid else None)
    bb = it.block_bytes
    n = a.ndf * nchunk
    d_blk = it.alloc(bb)
    it.fill_synthetic(d_blk, 20181105, 0, 0)
    block = it.download(d_blk)
    d_out = it.alloc(bb)
    d_spec = it.alloc(it.nout * 4 * max(a.steps, 1))
    d_cnt = it.upload(np.zeros(nchunk + 3, np.uint64))
    rng = np.random.default_rng(5)
    orders = {
        # frames of one time step arrive together, chunks in any order
        "time-major, chunks shuffled": (np.arange(n).reshape(a.ndf, nchunk)
                                        [:, rng.permutation(nchunk)].reshape(-1)),
        "fully shuffled": rng.permutation(n),
    }
    if a.order != "both":
        orders = {k: v for k, v in orders.items() if k.startswith("time") == (a.order == "tm")}
    for name, order in orders.items():
        t0 = time.perf_counter()
        dfs, chunk = build_stream(block, nchunk, 1000, 54, order)
        prep = time.perf_counter() - t0
        d_dfs, d_chk = it.upload(dfs.reshape(-1)), it.upload(chunk)
        del dfs

        def asm():
            it.assemble(d_dfs, n, d_chk, 1000, 54, d_out, a.ndf, nchunk, d_cnt)

        for _ in range(a.warmup):
            asm()
        it.sync()
        it.reset_stats()
        it.set_timing(2)
        for _ in range(a.steps):
            asm()
        it.set_timing(0)
        it.sync()
        asm_s = it.stats()["kernel_ms"] / a.steps / 1e3
        ok = bool(np.array_equal(it.download(d_out), block))

        # assemble + integrate, one block per step
        for _ in range(a.warmup):
            asm()
            it.integrate(d_out, d_spec.ptr, True)
        it.sync()
        it.reset_stats()
        it.set_timing(2)
        for k in range(a.steps):
            asm()
            it.integrate(d_out, d_spec.ptr + k * it.nout * 4, True)
        it.set_timing(0)
        it.sync()
        both_s = it.stats()["kernel_ms"] / a.steps / 1e3
        moved = n * (DF + PAY)
        print(json.dumps({
            "path": "b2p_assemble (DF stream -> TFTFP block)", "order": name,
            "frames": n, "block_bytes": bb, "payload_equal": ok,
            "assemble_us": round(asm_s * 1e6, 1),
            "roofline": {"bound": "hbm", "achieved": round(moved / asm_s / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(moved / asm_s / 1e9 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": moved},
            "stream_to_spectrum_us": round(both_s * 1e6, 1),
            # channels x pols x time, as bench.py counts samples
            "stream_to_spectrum_Msamples_s": round(a.ndf * 128 * it.nout * 2 / both_s / 1e6, 1),
            "host_stream_build_s": round(prep, 1),
            "grid": a.grid or "default",
        }), flush=True)
        d_dfs.free()
        d_chk.free()
    for b in (d_blk, d_out, d_spec, d_cnt):
        b.free()
    it.close()


if __name__ == "__main__":
    main()
