"""The oracle, pinned before it is trusted (CPU only).

* both restatements (NumPy and C) reproduce the committed golden fixtures
  bit for bit, inputs included (the fixtures pin the synthetic generator too);
* hand-computed known answers (SURVEY.md 8c fixture 3): sign extremes, the
  channel-mapping guard, the byte-order / lane guard;
* the BSWAP_64 word decode agrees with the reference's own hdr.c
  (tests/golden/hdr_pin.npz, produced by the reference code compiled from
  /root/reference -- hdr.c:10-28).
"""
import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
from conftest import golden_geom, load_golden

CASES = ["bmf_small", "int8_256", "int16le_48"]


@pytest.mark.parametrize("name", CASES)
def test_fixture_inputs_regenerate(name):
    d = load_golden(name)
    g = golden_geom(d)
    args = (int(d["seed"]), int(d["subband"]), int(d["block"]))
    assert np.array_equal(npo.fill_synthetic(g, d["input"].size, *args), d["input"])
    assert np.array_equal(co.fill_synthetic(g, d["input"].size, *args), d["input"])


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("npol_out", [1, 2])
@pytest.mark.parametrize("mean", [0, 1])
@pytest.mark.parametrize("impl", ["numpy", "c", "c_mt"])
def test_fixture_outputs(name, npol_out, mean, impl):
    d = load_golden(name)
    g = golden_geom(d, npol_out=npol_out, mean=mean)
    if impl == "numpy":
        acc = npo.integrate(g, d["input"])
        p = npo.finalize(g, acc)
    else:
        acc = co.integrate(g, d["input"], nthreads=4 if impl == "c_mt" else 1)
        p = co.finalize(g, acc)
    assert np.array_equal(acc, d[f"acc_p{npol_out}"])
    assert np.array_equal(p.view(np.uint32), d[f"power_p{npol_out}_m{mean}"].view(np.uint32))


def _bmf_word(xre, xim, yre, yim):
    """store one BMF word so that BSWAP_64 yields lanes (xre, xim, yre, yim)"""
    lanes = np.array([xre, xim, yre, yim], dtype=np.int16).view(np.uint16).astype(np.uint64)
    v = lanes[0] | (lanes[1] << np.uint64(16)) | (lanes[2] << np.uint64(32)) | (lanes[3] << np.uint64(48))
    return np.array([v], dtype=">u8").view(np.uint8)  # BSWAP_64 inverse = big-endian store


def test_kat_bmf_extreme_overflow_guard():
    # every component -32768: |X|^2+|Y|^2 = 4 * 2^30 = 2^32 per sample
    g = npo.Geom(nbit=16, big_endian=1, nchunk=2, nsamp_df=128, nchan_chunk=7, nsamp_int=512)
    buf = np.tile(np.array([0x80, 0x00], dtype=np.uint8), g.block_bytes // 2)
    acc = npo.integrate(g, buf)
    assert np.all(acc == np.uint64(512 * 2 ** 32))
    assert np.array_equal(co.integrate(g, buf), acc)
    assert np.all(co.power(g, buf) == np.float32(512 * 2.0 ** 32))


def test_kat_int8_extreme():
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1000, npol_out=2)
    buf = np.full(g.block_bytes, 0x80, dtype=np.uint8)  # -128 everywhere
    acc = co.integrate(g, buf)
    assert np.all(acc == np.uint64(1000 * 2 * 128 * 128))
    assert np.array_equal(npo.integrate(g, buf), acc)


def test_kat_channel_mapping_guard():
    # every component of channel c equals c (TFTFP, 3 chunks x 5 chans):
    # P[c] = nsamp * 4 * c^2 ; checks chunk*nchan_chunk + chan ordering
    g = npo.Geom(nbit=16, big_endian=1, nchunk=3, nsamp_df=4, nchan_chunk=5, nsamp_int=8)
    frames = []
    for _ in range(g.nsamp_int // g.nsamp_df):
        for ck in range(g.nchunk):
            for _s in range(g.nsamp_df):
                for k in range(g.nchan_chunk):
                    c = ck * g.nchan_chunk + k
                    frames.append(_bmf_word(c, c, c, c))
    buf = np.concatenate(frames)
    expect = np.array([g.nsamp_int * 4 * c * c for c in range(g.nchan)], dtype=np.uint64)
    assert np.array_equal(npo.integrate(g, buf), expect)
    assert np.array_equal(co.integrate(g, buf), expect)


@pytest.mark.parametrize("offset", range(8))
def test_kat_byte_lane_guard(offset):
    # a single 0x01 byte at each offset of a BMF word: even offsets are the
    # high byte of a BE int16 (value 256 -> 65536), odd ones the low byte (1);
    # bytes 0-3 decode to Y (lanes 3,2), bytes 4-7 to X (lanes 1,0)
    g = npo.Geom(nbit=16, big_endian=1, nchunk=1, nsamp_df=2, nchan_chunk=1, nsamp_int=2,
                 npol_out=2)
    buf = np.zeros(g.block_bytes, dtype=np.uint8)
    buf[offset] = 1
    val = 256 if offset % 2 == 0 else 1
    x, y = (val * val, 0) if offset >= 4 else (0, val * val)
    assert list(npo.integrate(g, buf)) == [x, y]
    assert list(co.integrate(g, buf)) == [x, y]
    lanes = co.bmf_lanes(bytes(buf[:8]))
    k = 3 - offset // 2  # lane holding that byte
    assert lanes[k] == val and np.count_nonzero(lanes) == 1


def test_kat_int8_lane_order():
    # int8 words are stored X.re, X.im, Y.re, Y.im (byte order)
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=4, nchan_chunk=1, nsamp_int=4, npol_out=2)
    buf = np.zeros(16, dtype=np.uint8)
    buf[0:4] = np.array([3, -4, 0, 0], dtype=np.int8).view(np.uint8)
    buf[4:8] = np.array([0, 0, 6, 8], dtype=np.int8).view(np.uint8)
    assert list(co.integrate(g, buf)) == [25, 100]
    assert list(npo.integrate(g, buf)) == [25, 100]


def test_rne_rounding_and_mean():
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=4, nchan_chunk=4, nsamp_int=3, npol_out=1)
    acc = np.array([2 ** 24 + 1, 2 ** 24 + 3, 2 ** 25 + 2, 7], dtype=np.uint64)
    out = co.finalize(g, acc)
    # ties to even: 2^24+1 -> 2^24, 2^24+3 -> 2^24+4, 2^25+2 -> 2^25 (tie, even)
    assert list(out) == [2.0 ** 24, 2.0 ** 24 + 4, 2.0 ** 25, 7.0]
    assert np.array_equal(npo.finalize(g, acc), out)
    gm = npo.Geom(**{**g.asdict(), "mean": 1})
    assert np.array_equal(co.finalize(gm, acc), (acc.astype(np.float64) / 3).astype(np.float32))
    assert np.array_equal(npo.finalize(gm, acc), co.finalize(gm, acc))


def test_ragged_rejected():
    g = npo.BMF
    with pytest.raises(ValueError):
        npo.integrate(g, np.zeros(g.frame_bytes + 8, dtype=np.uint8))
    with pytest.raises(ValueError):
        co.integrate(g, np.zeros(g.frame_bytes - 16, dtype=np.uint8))


def test_empty_input():
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=16)
    z = np.zeros(0, dtype=np.uint8)
    assert np.all(co.integrate(g, z) == 0)
    assert np.all(npo.integrate(g, z) == 0)


def test_bmf_geometry_matches_reference_constants():
    g = npo.BMF
    assert g.frame_bytes == 48 * 7168           # NCHK_NIC x DT_SIZE (capture.h:20,28)
    assert g.block_bytes == 2818572288          # NDF 8192 (conf:9), py:67
    assert g.nchan == 336                       # header_baseband2power.txt:42
    assert g.nout * 4 == 1344                   # paf-baseband2power.py:77-79


def test_hdr_pin_against_reference_hdr_c():
    """The oracle's BSWAP_64 lane decode reproduces the fields that the
    reference's own hdr_keys() (hdr.c:10-28) extracts from bswap_64 words."""
    d = load_golden("hdr_pin")
    dfs, raw, freq = d["df_headers"], d["valid_idf_sec_epoch_beam"], d["freq"]
    for i in range(dfs.shape[0]):
        w0 = co.bmf_lanes(bytes(dfs[i, 0:8])).view(np.uint16).astype(np.uint64)
        w1 = co.bmf_lanes(bytes(dfs[i, 8:16])).view(np.uint16).astype(np.uint64)
        w2 = co.bmf_lanes(bytes(dfs[i, 16:24])).view(np.uint16).astype(np.uint64)
        idf = int(w0[0]) | (int(w0[1]) << 16)
        sec = (int(w0[2]) | (int(w0[3]) << 16)) & 0x3FFFFFFF
        valid = int(w0[3]) >> 15
        epoch = (int(w1[1]) >> 10) & 0x3F
        beam = int(w2[0])
        assert [valid, idf, sec, epoch, beam] == [int(x) for x in raw[i]]
        assert float(int(w2[1])) == freq[i]


def test_hdr_pin_live_reference_if_present():
    """Re-run the reference's hdr.c (built by `make -C oracle ref`) when it
    exists in this container; on the GPU box the committed pin is used."""
    L = co.ref_hdr_lib()
    if L is None:
        pytest.skip("oracle/_ref/libhdr_ref.so not built (no /root/reference here)")
    d = load_golden("hdr_pin")
    for i in range(0, d["df_headers"].shape[0], 17):
        h = co.HdrT()
        buf = np.ascontiguousarray(d["df_headers"][i])
        L.hdr_keys(buf.ctypes.data, h)
        assert [h.valid, h.idf, h.sec, h.epoch, h.beam] == [int(x) for x in
                                                             d["valid_idf_sec_epoch_beam"][i]]


# ---- the two restatements agree on random layouts (hypothesis) -----------------
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@st.composite
def _layouts(draw):
    nbit = draw(st.sampled_from([8, 16]))
    be = int(draw(st.booleans())) if nbit == 16 else 0
    word = 4 * nbit // 8
    ncc = draw(st.integers(1, 40))
    base = 1
    while (base * ncc * word) % 16:
        base *= 2
    nsdf = base * draw(st.integers(1, 3))
    nchunk = draw(st.integers(1, 12))
    frames = draw(st.integers(1, 12))
    return npo.Geom(nbit=nbit, big_endian=be, nchunk=nchunk, nsamp_df=nsdf, nchan_chunk=ncc,
                    npol_out=draw(st.sampled_from([1, 2])), nsamp_int=frames * nsdf,
                    mean=int(draw(st.booleans()))), draw(st.integers(0, 2 ** 32 - 1))


@settings(max_examples=150, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow])
@given(_layouts())
def test_c_and_numpy_restatements_agree(case):
    g, seed = case
    buf = co.fill_synthetic(g, g.block_bytes, seed, seed % 3, seed % 11)
    assert np.array_equal(buf, npo.fill_synthetic(g, g.block_bytes, seed, seed % 3, seed % 11))
    acc = npo.integrate(g, buf)
    assert np.array_equal(co.integrate(g, buf), acc)
    assert np.array_equal(co.finalize(g, acc).view(np.uint32), npo.finalize(g, acc).view(np.uint32))
