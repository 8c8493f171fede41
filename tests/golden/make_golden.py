"""Generate the committed golden fixtures under tests/golden/.

    python tests/golden/make_golden.py            # synthetic-layout fixtures
    python tests/golden/make_golden.py --hdr-pin  # + reference hdr.c pin (needs
                                                  #   `make -C oracle ref`, i.e.
                                                  #   /root/reference present)

The reference ships no golden vectors for its (empty) hot path, so the
expected outputs here come from the two oracle restatements, which must agree
bit for bit before anything is written.  hdr_pin.npz is different: its
expected values are outputs of the reference's own hdr.c (hdr.c:10-28),
compiled from /root/reference by oracle/Makefile, run on random 64-B BMF
data-frame headers.  It pins the BSWAP_64 word/lane convention that the
oracle's BMF payload decode uses (cudautil.cuh:118-125).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import b2p_oracle as npo  # noqa: E402
import oracle_c as co  # noqa: E402

SEED = 20181105

CASES = {
    # BMF-native TFTFP int16 BE, 2 chunks x 7 chans x 128 samp x 16 DF (224 KiB)
    "bmf_small": dict(geom=npo.Geom(nbit=16, big_endian=1, nchunk=2, nsamp_df=128,
                                    nchan_chunk=7, nsamp_int=2048), subband=0, block=0),
    # generic int8 [t][256][2][2] x 512 samples (512 KiB) -- configs 1/2 layout
    "int8_256": dict(geom=npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256,
                                   nsamp_int=512), subband=1, block=3),
    # generic int16 little-endian, 48 chans, TFTFP with 4 chunks x 12 chans
    "int16le_48": dict(geom=npo.Geom(nbit=16, big_endian=0, nchunk=4, nsamp_df=8,
                                     nchan_chunk=12, nsamp_int=256), subband=2, block=1),
}


def make_case(name: str, spec: dict) -> dict:
    g = spec["geom"]
    buf = npo.fill_synthetic(g, g.block_bytes, SEED, spec["subband"], spec["block"])
    buf_c = co.fill_synthetic(g, g.block_bytes, SEED, spec["subband"], spec["block"])
    assert np.array_equal(buf, buf_c), f"{name}: generators disagree"
    out = {"input": buf, "seed": np.uint64(SEED), "subband": np.uint32(spec["subband"]),
           "block": np.uint64(spec["block"])}
    for k, v in g.asdict().items():
        out[f"geom_{k}"] = np.uint64(v)
    for npol_out in (1, 2):
        for mean in (0, 1):
            gg = npo.Geom(**{**g.asdict(), "npol_out": npol_out, "mean": mean})
            acc = npo.integrate(gg, buf)
            acc_c = co.integrate(gg, buf)
            assert np.array_equal(acc, acc_c), f"{name}: integrate disagrees"
            p, p_c = npo.finalize(gg, acc), co.finalize(gg, acc_c)
            assert np.array_equal(p.view(np.uint32), p_c.view(np.uint32)), f"{name}: finalize"
            out[f"acc_p{npol_out}"] = acc
            out[f"power_p{npol_out}_m{mean}"] = p
    return out


def make_hdr_pin(n: int = 256) -> dict:
    L = co.ref_hdr_lib()
    if L is None:
        raise SystemExit("oracle/_ref/libhdr_ref.so missing: run `make -C oracle ref`")
    rng = np.random.default_rng(SEED)
    dfs = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
    fields = np.zeros((n, 6), dtype=np.float64)
    raw = np.zeros((n, 5), dtype=np.uint64)
    for i in range(n):
        h = co.HdrT()
        buf = np.ascontiguousarray(dfs[i])
        L.hdr_keys(buf.ctypes.data, h)
        raw[i] = (h.valid, h.idf, h.sec, h.epoch, h.beam)
        fields[i] = (h.valid, h.idf, h.sec, h.epoch, h.beam, h.freq)
    return {"df_headers": dfs, "valid_idf_sec_epoch_beam": raw, "freq": fields[:, 5]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hdr-pin", action="store_true")
    a = ap.parse_args()
    for name, spec in CASES.items():
        d = make_case(name, spec)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **d)
        print("wrote", name, d["input"].size, "B")
    if a.hdr_pin:
        np.savez_compressed(os.path.join(HERE, "hdr_pin.npz"), **make_hdr_pin())
        print("wrote hdr_pin")


if __name__ == "__main__":
    main()
