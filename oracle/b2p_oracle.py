"""oracle/b2p_oracle.py -- TEST INFRASTRUCTURE ONLY.

Second, independent restatement (NumPy) of the baseband->power integrate path
of xinpingdeng/paf-baseband2power.  Only tests/, ``__graft_entry__.smoke()``
and ``bench.py``'s cpu_baseline leg may import this module; the product
package never does.

Parity status: partially pinned -- see oracle/b2p_oracle.h.  The reference's
hot path is empty (kernel.cu:1-7, baseband2power.cu:1-16,
paf_baseband2power.cu:32-93) and it ships no fixtures, so the integrate
semantics restate the reference's specification:

* TFTFP block layout, payload only -- capture.c:222, 527, 540; capture.h:20,28;
  paf-baseband2power.conf:2-5,9.
* BMF words are big-endian 64-bit, unpacked with BSWAP_64 -- cudautil.cuh:118-125
  (pinned against the reference's own hdr.c, tests/golden/hdr_pin.npz).
* detect |X|^2+|Y|^2 and integrate 1024x1024 samples -- README.md:2,
  paf_baseband2power.cu:20.
* output NBIT 32 / NPOL 1 / NCHAN -- header_baseband2power.txt:39-42,
  paf-baseband2power.py:77-79.

It is written with array reshapes rather than loops (the C restatement uses
loops), so the two restatements share no code path.
"""
from __future__ import annotations

from dataclasses import dataclass, asdict

import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


@dataclass(frozen=True)
class Geom:
    """Layout descriptor; same fields/meaning as ``b2p_geom_t`` (include/b2p.h).

    Block = [frame][chunk][nsamp_df][nchan_chunk][npol][ndim] (TFTFP,
    capture.c:540).  BMF-native: nbit=16, big_endian=1, nchunk=48,
    nsamp_df=128, nchan_chunk=7 (capture.h:20,28; conf:2-5).
    """

    nbit: int = 8
    big_endian: int = 0
    nchunk: int = 1
    nsamp_df: int = 1
    nchan_chunk: int = 256
    npol: int = 2
    ndim: int = 2
    npol_out: int = 1
    nsamp_int: int = 1 << 20
    mean: int = 0

    @property
    def word_bytes(self) -> int:
        return self.npol * self.ndim * self.nbit // 8

    @property
    def frame_bytes(self) -> int:
        return self.nchunk * self.nsamp_df * self.nchan_chunk * self.word_bytes

    @property
    def nchan(self) -> int:
        return self.nchunk * self.nchan_chunk

    @property
    def nout(self) -> int:
        return self.nchan * self.npol_out

    @property
    def block_bytes(self) -> int:
        """bytes of one integration (nsamp_int samples of every channel)"""
        return self.nsamp_int // self.nsamp_df * self.frame_bytes

    def asdict(self) -> dict:
        return asdict(self)


BMF = Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7)


def components(g: Geom, buf: np.ndarray) -> np.ndarray:
    """Decode ``buf`` (uint8, whole frames) to int64 [frame, chunk, samp, chan, 4]
    with the last axis X.re, X.im, Y.re, Y.im."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    if g.npol != 2 or g.ndim != 2:
        raise ValueError("npol=2, ndim=2 only")
    if buf.size % g.frame_bytes:
        raise ValueError("ragged input: not a whole number of frames")
    nf = buf.size // g.frame_bytes
    if g.nbit == 8:
        c = buf.view(np.int8).astype(np.int64)
    elif g.big_endian:
        # BSWAP_64 of each 8-B word, lanes = little-endian int16 of the result:
        # lane k sits at stored bytes [6-2k, 7-2k] big-endian (cudautil.cuh:118)
        w = buf.view(">i2").reshape(-1, 4)  # stored order: lane3, lane2, lane1, lane0
        c = w[:, ::-1].astype(np.int64)
    else:
        c = buf.view("<i2").astype(np.int64)
    return c.reshape(nf, g.nchunk, g.nsamp_df, g.nchan_chunk, 4)


def integrate(g: Geom, buf: np.ndarray, acc: np.ndarray | None = None) -> np.ndarray:
    """Exact integer accumulate; returns uint64 [nout] (added into ``acc``)."""
    c = components(g, buf)
    sq = c * c
    px = (sq[..., 0] + sq[..., 1]).sum(axis=(0, 2), dtype=np.int64)  # [chunk, chan]
    py = (sq[..., 2] + sq[..., 3]).sum(axis=(0, 2), dtype=np.int64)
    if g.npol_out == 1:
        r = (px + py).reshape(-1)
    else:
        r = np.stack([px.reshape(-1), py.reshape(-1)], axis=1).reshape(-1)
    r = r.astype(np.uint64)
    if acc is None:
        return r
    acc += r
    return acc


def finalize(g: Geom, acc: np.ndarray) -> np.ndarray:
    """One round-to-nearest-even conversion to fp32 (sum, or sum/nsamp_int)."""
    acc = np.asarray(acc, dtype=np.uint64)
    if g.mean:
        return (acc.astype(np.float64) / float(g.nsamp_int)).astype(np.float32)
    # sums stay < 2**53, so the float64 step is exact and the cast is the one RNE
    return acc.astype(np.float64).astype(np.float32)


def power(g: Geom, buf: np.ndarray) -> np.ndarray:
    return finalize(g, integrate(g, buf))


# ---------------------------------------------------------------- synthetic


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def fill_synthetic(g: Geom, nbytes: int, seed: int, subband: int, block: int,
                   elem0: int = 0) -> np.ndarray:
    """Counter-based baseband: element e is a function of
    (seed, subband, block, e) only, so every host/GPU regenerates it."""
    with np.errstate(over="ignore"):
        k_sub = splitmix64(np.uint64(seed) ^ (np.uint64(0xD1B54A32D192ED03) * np.uint64(subband + 1)))
        key = splitmix64(k_sub ^ (np.uint64(0x8CB92BA72F3D8DD7) * np.uint64(block + 1)))
        eb = g.nbit // 8
        e = np.arange(elem0, elem0 + nbytes // eb, dtype=np.uint64)
        r = splitmix64(key + e)
    m = np.uint64(0xFFFF)
    gs = ((r & m).astype(np.int64) + ((r >> np.uint64(16)) & m).astype(np.int64)
          + ((r >> np.uint64(32)) & m).astype(np.int64) + (r >> np.uint64(48)).astype(np.int64)
          - 131070)
    comp = g.npol * g.ndim
    wpc = g.nsamp_df * g.nchan_chunk
    wf = (e // np.uint64(comp)) % np.uint64(wpc * g.nchunk)
    ch = (wf // np.uint64(wpc)) * np.uint64(g.nchan_chunk) + wf % np.uint64(g.nchan_chunk)
    amp = 35 if g.nbit == 8 else 3464
    tone = (ch == 0) | (ch == 7) | (ch == np.uint64(g.nchan - 1))
    a = np.where(tone, 2 * amp, amp).astype(np.int64)
    v = (gs * a) >> 16
    if g.nbit == 8:
        return np.clip(v, -128, 127).astype(np.int8).view(np.uint8)
    v = np.clip(v, -32768, 32767).astype(np.int16)
    return v.astype(">i2" if g.big_endian else "<i2").view(np.uint8)


# ---------------------------------------------------------------- data frames
# header words (hdr.c:10-28): w0 = idf | sec<<32 | valid<<63, w1 = epoch<<26,
# w2 = beam | freq<<16, each stored big-endian (bswap_64 on read)

DF_BYTES, DF_HDR, DF_PAYLOAD = 7232, 64, 7168


def df_encode(idf, sec, valid=1, epoch=0, beam=0, freq=0) -> np.ndarray:
    """[n, 64] uint8 headers for arrays of fields (the inverse of hdr_keys)."""
    idf, sec = np.atleast_1d(np.asarray(idf, np.uint64)), np.atleast_1d(np.asarray(sec, np.uint64))
    n = max(idf.size, sec.size)
    b = lambda x: np.broadcast_to(np.asarray(x, np.uint64), (n,))  # noqa: E731
    w0 = (b(idf) & np.uint64(0xFFFFFFFF)) | ((b(sec) & np.uint64(0x3FFFFFFF)) << np.uint64(32)) \
        | ((b(valid) & np.uint64(1)) << np.uint64(63))
    w1 = (b(epoch) & np.uint64(0x3F)) << np.uint64(26)
    w2 = (b(beam) & np.uint64(0xFFFF)) | ((b(freq) & np.uint64(0xFFFF)) << np.uint64(16))
    out = np.zeros((n, DF_HDR), dtype=np.uint8)
    out[:, 0:24] = np.stack([w0, w1, w2], axis=1).astype(">u8").view(np.uint8).reshape(n, 24)
    return out


def df_decode(hdrs: np.ndarray) -> dict:
    w = np.ascontiguousarray(hdrs[..., :24]).view(">u8").astype(np.uint64).reshape(-1, 3)
    return {"idf": w[:, 0] & np.uint64(0xFFFFFFFF),
            "sec": (w[:, 0] >> np.uint64(32)) & np.uint64(0x3FFFFFFF),
            "valid": w[:, 0] >> np.uint64(63),
            "epoch": (w[:, 1] >> np.uint64(26)) & np.uint64(0x3F),
            "freq": (w[:, 2] >> np.uint64(16)) & np.uint64(0xFFFF),
            "beam": w[:, 2] & np.uint64(0xFFFF)}


def df_stream(block: np.ndarray, nchunk: int, ref_idf: int, ref_sec: int, order=None,
              beam: int = 0, epoch: int = 0, freq0: int = 1300, ndf_period: int = 250000,
              period_sec: int = 27):
    """Disassemble a payload-only TFTFP block into (dfs [n, 7232], chunk_of_df [n]),
    frames numbered from the reference (wrapping into the next 27-s period as
    sync.c:119-125 does); `order` permutes / drops frames (arrival order)."""
    nf = block.size // (nchunk * DF_PAYLOAD)
    pay = block.reshape(nf * nchunk, DF_PAYLOAD)
    k = np.arange(nf * nchunk)
    t, c = k // nchunk, k % nchunk
    gidf = ref_idf + t
    idf, sec = gidf % ndf_period, ref_sec + (gidf // ndf_period) * period_sec
    hdr = df_encode(idf, sec, 1, epoch, beam, freq0 + c)
    dfs = np.concatenate([hdr, pay], axis=1)
    chunk = c.astype(np.uint8)
    if order is not None:
        dfs, chunk = dfs[order], chunk[order]
    return np.ascontiguousarray(dfs), np.ascontiguousarray(chunk)
