"""Layout descriptors of the reference's data and of the BASELINE configs.

BMF-native block: [DF 8192][chunk 48][samp 128][chan 7]
[pol 2][re,im] int16 big-endian, i.e. TFTFP (capture.c:540), 7168-B payloads
(capture.h:28), NCHK_NIC 48 (capture.h:20), NDF 8192
(paf-baseband2power.conf:9).  The BASELINE configs use 256 / 1024 channels
x 2 pols of int8 in [time][chan][pol][re,im] order (nchunk 1, nsamp_df 1).
"""
from __future__ import annotations

from . import _lib as L

NSAMP_INT = 1 << 20           # README.md:2: 1024 x 1024 samples
TSAMP_US = 27.0 / 32.0        # README.md:2: 0.84375 us


def make_geom(nbit: int = 8, big_endian: int = 0, nchunk: int = 1, nsamp_df: int = 1,
              nchan_chunk: int = 256, npol: int = 2, ndim: int = 2, npol_out: int = 1,
              nsamp_int: int = NSAMP_INT, mean: int = 0) -> L.Geom:
    return L.Geom(nbit, big_endian, nchunk, nsamp_df, nchan_chunk, npol, ndim, npol_out,
                  nsamp_int, mean, 0)


def bmf_geom(**kw) -> L.Geom:
    """BMF-native: 48 chunks x 7 channels = 336 (header_baseband2power.txt:42)."""
    d = dict(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7)
    d.update(kw)
    return make_geom(**d)


def generic_geom(nchan: int, nbit: int = 8, **kw) -> L.Geom:
    """[time][nchan][pol][re,im]; nsamp_df is chosen so a chunk is 16-B whole."""
    word = 2 * 2 * nbit // 8
    nsamp_df = 1
    while (nsamp_df * nchan * word) % 16:
        nsamp_df *= 2
    return make_geom(nbit=nbit, nchunk=1, nsamp_df=nsamp_df, nchan_chunk=nchan, **kw)


# BASELINE.json configs[0..4] (+ the reference-native layout)
CONFIGS = {
    "c1": dict(geom=lambda: generic_geom(256), subbands=1, gpus=0,
               what="1 sub-band, 256 ch x 2 pol int8, diskdb file, CPU plumbing"),
    "c2": dict(geom=lambda: generic_geom(256), subbands=1, gpus=1,
               what="1 sub-band, 256 ch x 2 pol int8, HBM-resident, 1 MI355X"),
    "c3": dict(geom=lambda: generic_geom(1024), subbands=1, gpus=1,
               what="1 sub-band, 1024 ch x 2 pol int8, pinned host buffer, H2D overlapped"),
    "c4": dict(geom=lambda: generic_geom(256), subbands=4, gpus=4,
               what="4 sub-bands x 256 ch over 4 MI355X, RCCL gather to rank 0"),
    "c5": dict(geom=lambda: generic_geom(1024), subbands=8, gpus=8,
               what="8 sub-bands x 1024 ch int8 in HBM over 8 MI355X"),
    "bmf": dict(geom=lambda: bmf_geom(), subbands=1, gpus=1,
                what="BMF-native 336 ch int16 BE TFTFP (2.625 GiB per integration)"),
}


def word_bytes(g: L.Geom) -> int:
    return g.npol * g.ndim * g.nbit // 8


def frame_bytes(g: L.Geom) -> int:
    return g.nchunk * g.nsamp_df * g.nchan_chunk * word_bytes(g)


def block_bytes(g: L.Geom) -> int:
    return g.nsamp_int // g.nsamp_df * frame_bytes(g)


BATCH_BYTES = 4 << 30  # include/b2p.h B2P_BATCH_BYTES
MAX_BLOCKS = 8         # B2P_MAX_BLOCKS


def blocks_per_launch(block_bytes: int) -> int:
    """queued blocks per b2p_integrate_n launch (b2p_blocks_per_launch in
    include/b2p.h): a launch reads >= 4 GiB, 1..8 blocks"""
    return max(1, min(MAX_BLOCKS, BATCH_BYTES // block_bytes if block_bytes else 1))


def nchan(g: L.Geom) -> int:
    return g.nchunk * g.nchan_chunk


def samples_per_block(g: L.Geom) -> int:
    """complex samples (channels x pols x time) in one integration"""
    return nchan(g) * g.npol * g.nsamp_int
