"""BMF data-frame headers and TFTFP placement (CPU).

The decode is pinned by the reference's own hdr.c (tests/golden/hdr_pin.npz:
hdr_keys outputs on random headers, hdr.c:10-28); frame index, reference
advance and chunk-from-IP restate capture.c:562-584 and sync.c:119-125.
"""
import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
from conftest import load_golden
from paf_b2p import dada


def test_decode_matches_reference_hdr_c():
    d = load_golden("hdr_pin")
    for i in range(d["df_headers"].shape[0]):
        h = dada.df_decode(d["df_headers"][i].tobytes())
        assert [h.valid, h.idf, h.sec, h.epoch, h.beam] == [int(x) for x in
                                                             d["valid_idf_sec_epoch_beam"][i]]
        assert h.freq == d["freq"][i]


def test_encode_decode_roundtrip_and_reference():
    rng = np.random.default_rng(7)
    L = co.ref_hdr_lib()
    for _ in range(300):
        f = dict(idf=int(rng.integers(0, 2 ** 32)), sec=int(rng.integers(0, 2 ** 30)),
                 valid=int(rng.integers(0, 2)), epoch=int(rng.integers(0, 64)),
                 beam=int(rng.integers(0, 2 ** 16)), freq=float(rng.integers(0, 2 ** 16)))
        raw = dada.df_encode(**f)
        h = dada.df_decode(raw)
        assert (h.idf, h.sec, h.valid, h.epoch, h.beam, h.freq) == tuple(f.values())
        # the NumPy restatement encodes the same bytes
        assert raw == npo.df_encode(f["idf"], f["sec"], f["valid"], f["epoch"], f["beam"],
                                    int(f["freq"])).tobytes()
        if L is not None:  # and the reference's own decoder reads them back
            r = co.HdrT()
            buf = np.frombuffer(raw, dtype=np.uint8).copy()
            L.hdr_keys(buf.ctypes.data, r)
            assert (r.idf, r.sec, r.valid, r.epoch, r.beam, r.freq) == tuple(f.values())


def _index_restated(idf, sec, ridf, rsec):
    # capture.c:566 in Python floats (IEEE double, as C)
    secdiff = (sec - rsec) % 2 ** 64
    if secdiff >= 2 ** 63:
        secdiff -= 2 ** 64
    v = float(idf) + float(secdiff) / 1.08E-4 - float(ridf)
    return int(v)  # C conversion truncates toward zero


@pytest.mark.parametrize("idf,sec,ridf,rsec", [
    (100, 54, 90, 54), (5, 81, 249990, 54), (249995, 54, 10, 81), (0, 0, 0, 0),
    (7, 27 * 1000, 3, 27 * 999), (12, 3, 0, 0), (0, 54, 249999, 27)])
def test_frame_index_restates_capture(idf, sec, ridf, rsec):
    h, r = dada.DfHdr(1, idf, sec, 0, 0, 0.0), dada.DfHdr(1, ridf, rsec, 0, 0, 0.0)
    assert dada.df_index(h, r) == _index_restated(idf, sec, ridf, rsec)


def test_ref_advance_wraps_period():
    r = dada.DfHdr(1, 249000, 54, 0, 0, 0.0)
    a = dada.df_ref_advance(r, 8192)  # sync.c:119-125
    assert (a.idf, a.sec) == (249000 + 8192 - 250000, 81)
    b = dada.df_ref_advance(dada.DfHdr(1, 10, 54, 0, 0, 0.0), 8192)
    assert (b.idf, b.sec) == (8202, 54)
    # the index of a frame stays the same measured from either reference
    h = dada.DfHdr(1, 7000, 81, 0, 0, 0.0)
    assert dada.df_index(h, r) == dada.df_index(h, a) + 8192


def test_chunk_from_ip_table():
    # capture.c:573-580: BMFs 10.16.X.1..12, X = 1..8; links 1,3,5,... carry chunks
    got = {}
    for x in range(1, 9):
        for y in range(1, 13):
            got[(x, y)] = dada.df_chunk_from_ip(10, 16, x, y)
    assert got[(1, 1)] == 0 and got[(1, 2)] == 0 and got[(1, 12)] == 5
    assert got[(2, 1)] == 6 and got[(8, 11)] == 47
    assert sorted(set(got.values())) == list(range(48))


def test_oracle_assembly_places_and_counts():
    nchunk, block_ndf = 4, 6
    rng = np.random.default_rng(3)
    block = rng.integers(0, 256, block_ndf * nchunk * 7168, dtype=np.uint8)
    ref_idf, ref_sec = 249998, 27  # the block crosses into the next period
    order = rng.permutation(block_ndf * nchunk)[:-3]  # 3 frames lost
    dfs, chunk = npo.df_stream(block, nchunk, ref_idf, ref_sec, order)
    # a late frame (before the block) and a frame from the next block
    extra, echunk = npo.df_stream(block[:nchunk * 7168 * 2], nchunk, ref_idf - 2, ref_sec)
    later, lchunk = npo.df_stream(block[:nchunk * 7168], nchunk, ref_idf + block_ndf, ref_sec)
    dfs = np.concatenate([dfs, extra[:1], later[:1]])
    chunk = np.concatenate([chunk, echunk[:1], np.array([9], np.uint8)])  # bad chunk id too
    out = np.full(block.size, 0xA5, dtype=np.uint8)
    counts = co.assemble(dfs, chunk, ref_idf, ref_sec, out, block_ndf, nchunk)
    got = out.reshape(-1, 7168)
    want = block.reshape(-1, 7168)
    placed = np.zeros(block_ndf * nchunk, bool)
    placed[order] = True
    assert np.array_equal(got[placed], want[placed])
    assert np.all(got[~placed] == 0xA5)
    exp = np.bincount(order % nchunk, minlength=nchunk).tolist() + [1, 0, 1]
    assert counts.tolist() == exp


# ---- paf_dfgen: payload-only DADA file -> raw DF capture stream ------------------

def _run_dfgen(tmp_path, block, nchunk, *args):
    import os
    import subprocess
    src = tmp_path / "in.dada"
    dada.write_dada_file(str(src), "HDR_SIZE 4096\n", block)
    out, chk = tmp_path / "out.df", tmp_path / "chunks.u8"
    subprocess.run([os.path.join(dada.BIN_DIR, "paf_dfgen"), "-i", str(src), "-o", str(out),
                    "-n", str(nchunk), "-c", str(chk), *map(str, args)],
                   check=True, capture_output=True)
    dfs = np.fromfile(out, dtype=np.uint8).reshape(-1, npo.DF_BYTES)
    return dfs, np.fromfile(chk, dtype=np.uint8)


@pytest.mark.parametrize("ref_idf", [1000, 249995])
def test_dfgen_matches_numpy_stream(tmp_path, ref_idf):
    nchunk, nf = 4, 6
    rng = np.random.default_rng(ref_idf)
    block = rng.integers(0, 256, nf * nchunk * npo.DF_PAYLOAD, dtype=np.uint8)
    dfs, chunk = _run_dfgen(tmp_path, block, nchunk, "-x", ref_idf, "-s", 54, "-f", 1300, "-b", 3,
                            "-e", 5)
    want, want_chunk = npo.df_stream(block, nchunk, ref_idf, 54, beam=3, epoch=5, freq0=1300)
    assert np.array_equal(dfs, want) and np.array_equal(chunk, want_chunk)


def test_dfgen_shuffled_lossy_stream_reassembles(tmp_path):
    nchunk, nf = 3, 8
    rng = np.random.default_rng(3)
    block = rng.integers(0, 256, nf * nchunk * npo.DF_PAYLOAD, dtype=np.uint8)
    dfs, chunk = _run_dfgen(tmp_path, block, nchunk, "-x", 249996, "-s", 27, "-r", 11, "-l", 200)
    n = dfs.shape[0]
    assert 0 < n < nf * nchunk  # some frames lost, order shuffled
    out = np.zeros_like(block)
    counts = co.assemble(dfs, chunk, 249996, 27, out, nf, nchunk)
    assert int(counts[:nchunk].sum()) == n
    # every frame that arrived lands where it came from; lost ones stay zero
    got = out.reshape(nf * nchunk, -1)
    src = block.reshape(nf * nchunk, -1)
    hit = np.zeros(nf * nchunk, bool)
    for i in range(n):
        h = npo.df_decode(dfs[i, :64])
        gidf = int(h["idf"][0]) + (int(h["sec"][0]) - 27) // 27 * 250000 - 249996
        hit[gidf * nchunk + chunk[i]] = True
    assert np.array_equal(got[hit], src[hit]) and not got[~hit].any()


def test_single_field_decoders_match_reference_hdr_c():
    # hdr_idf / hdr_sec / hdr_freq (hdr.c:30-55) against our full decode, on
    # random headers -- live, when oracle/_ref holds the reference's hdr.c
    L = co.ref_hdr_lib()
    if L is None:
        pytest.skip("oracle/_ref/libhdr_ref.so not built (no /root/reference here)")
    import ctypes as C
    L.hdr_idf.argtypes = L.hdr_sec.argtypes = L.hdr_freq.argtypes = [C.c_void_p]
    L.hdr_idf.restype = L.hdr_sec.restype = C.c_uint64
    L.hdr_freq.restype = C.c_double
    rng = np.random.default_rng(11)
    for _ in range(500):
        raw = rng.integers(0, 256, 64, dtype=np.uint8)
        h = dada.df_decode(raw.tobytes())
        p = raw.ctypes.data
        assert (L.hdr_idf(p), L.hdr_sec(p), L.hdr_freq(p)) == (h.idf, h.sec, h.freq)


# ---- start time of a capture (acquire_start_time, capture.c:791-843) -------------
EPOCHS = "# epoch  days-from-1970  date\n36 17532.0 2018-01-01\n37 17713.0 2018-07-01\n38 17897.0 2019-01-01\n"


def py_start_time(idf, sec, days):
    """independent restatement of capture.c:819-825 in Python floats (the
    same IEEE doubles); C round() is half away from zero"""
    import math
    import time as _t
    sec_prd = idf * 1.08e-4
    t = int(86400.0 * days + float(sec) + math.floor(sec_prd))
    utc = _t.strftime("%Y-%m-%d-%H:%M:%S", _t.gmtime(t))
    micro = 1.0e6 * (sec_prd - math.floor(sec_prd))
    return utc, int(1e6 * math.floor(micro + 0.5))


@pytest.mark.parametrize("idf,sec,days,utc,ps", [
    (0, 1000, 17713.0, "2018-07-01-00:16:40", 0),
    (12345, 0, 17713.0, "2018-07-01-00:00:01", 333260000000),        # 1.33326 s into the period
    (249999, 27, 17713.5, "2018-07-01-12:00:53", 999892000000),      # last frame of a period
    (0, 0, 0.0, "1970-01-01-00:00:00", 0),
    (1, 0, 17532.0, "2018-01-01-00:00:00", 108000000),               # one frame = 108 us
])
def test_start_time_known_answers(idf, sec, days, utc, ps):
    assert dada.df_start_time(idf, sec, days) == (utc, ps)
    assert py_start_time(idf, sec, days) == (utc, ps)


def test_start_time_matches_restatement():
    rng = np.random.default_rng(5)
    for _ in range(2000):
        idf = int(rng.integers(0, 250000))
        sec = int(rng.integers(0, 1 << 30))
        days = float(rng.integers(0, 40000)) + float(rng.choice([0.0, 0.25, 0.5]))
        assert dada.df_start_time(idf, sec, days) == py_start_time(idf, sec, days), (idf, sec, days)


def test_epoch_file_lookup(tmp_path):
    f = tmp_path / "epoch.txt"
    f.write_text(EPOCHS)
    assert dada.df_epoch_days(str(f), 37) == 17713.0
    assert dada.df_epoch_days(str(f), 36) == 17532.0
    with pytest.raises(KeyError):              # the reference silently used the last line read
        dada.df_epoch_days(str(f), 12)
    with pytest.raises(OSError):               # capture.c:798-805
        dada.df_epoch_days(str(tmp_path / "nope.txt"), 37)
