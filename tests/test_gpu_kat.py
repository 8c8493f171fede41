"""Known-answer tests of SURVEY.md 8c on the GPU (the oracle versions live
in tests/test_oracle.py): channel-mapping guard at BMF geometry, byte/lane
guard of the BSWAP_64 unpack (cudautil.cuh:118-125), int8 lane order."""
import numpy as np
import pytest

import b2p_oracle as npo
from test_gpu_parity import gpu_power, same_bits

pytestmark = pytest.mark.gpu


def _bmf_words(vals):
    """BE 8-B words whose BSWAP_64 lanes are (X.re, X.im, Y.re, Y.im) = vals[..., 0:4]"""
    v = np.asarray(vals, np.int64).astype(np.uint16).astype(np.uint64)
    w = v[..., 0] | (v[..., 1] << np.uint64(16)) | (v[..., 2] << np.uint64(32)) | (v[..., 3] << np.uint64(48))
    return np.ascontiguousarray(w, dtype=">u8").view(np.uint8).reshape(-1)


@pytest.mark.parametrize("npol_out", [1, 2])
def test_channel_mapping_guard_bmf(gpu, npol_out):
    # channel c = chunk*7 + chan carries X = (c, -c), Y = (2c, 1) in every word
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=128 * 16, npol_out=npol_out)
    c = (np.arange(48)[:, None] * 7 + np.arange(7)[None, :])          # [chunk, chan]
    lanes = np.stack([c, -c, 2 * c, np.ones_like(c)], axis=-1)          # [chunk, chan, 4]
    frame = np.broadcast_to(lanes[:, None, :, :], (48, 128, 7, 4))      # [chunk, samp, chan, 4]
    block = np.tile(_bmf_words(frame), g.nsamp_int // g.nsamp_df)
    cc = np.arange(g.nchan, dtype=np.float64)
    px, py = 2 * cc * cc * g.nsamp_int, (4 * cc * cc + 1) * g.nsamp_int
    want = (px + py) if npol_out == 1 else np.stack([px, py], axis=1).reshape(-1)
    out = gpu_power(g, block)
    assert same_bits(out, want.astype(np.float32))
    assert same_bits(out, npo.power(g, block))


@pytest.mark.parametrize("offset", range(8))
def test_byte_lane_guard(gpu, offset):
    # one 0x01 byte per 8-B word at `offset`; 336 channels so the kernel's
    # lane->channel mapping is exercised as in production
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=128 * 4, npol_out=2)
    buf = np.zeros(g.block_bytes, np.uint8)
    buf[offset::8] = 1
    val = 256 if offset % 2 == 0 else 1
    x, y = (val * val, 0) if offset >= 4 else (0, val * val)
    want = np.tile(np.array([x, y], np.float64) * g.nsamp_int, g.nchan).astype(np.float32)
    assert same_bits(gpu_power(g, buf), want)


def test_int8_lane_order_and_extremes(gpu):
    # int8 words are X.re, X.im, Y.re, Y.im in byte order; -128 is the extreme
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=4096, npol_out=2)
    w = np.zeros((g.nsamp_int, 256, 4), np.int8)
    w[:, :, 0], w[:, :, 1] = 3, -4                       # |X|^2 = 25
    w[:, :, 2], w[:, :, 3] = -128, -128                  # |Y|^2 = 32768
    buf = w.view(np.uint8).reshape(-1)
    want = np.tile(np.array([25.0, 32768.0]) * g.nsamp_int, 256).astype(np.float32)
    assert same_bits(gpu_power(g, buf), want)


@pytest.mark.parametrize("nbit,be", [(8, 0), (16, 1)])
def test_largest_output_count(gpu, nbit, be):
    # nout = 8192 (the ABI's limit, 64 KiB of LDS sums): 64 chunks x 64
    # channels x 2 output pols, against the oracle
    g = npo.Geom(nbit=nbit, big_endian=be, nchunk=64, nsamp_df=4, nchan_chunk=64, npol_out=2,
                 nsamp_int=4 * 24)
    assert g.nout == 8192
    import oracle_c as co
    buf = co.fill_synthetic(g, g.block_bytes, 99, 1, 2)
    assert same_bits(gpu_power(g, buf), co.power(g, buf, nthreads=8))
