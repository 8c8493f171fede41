"""UDP capture into a GPU-resident ring, end to end on
one box: paf_dfsend -> loopback UDP on 3 ports -> paf_capture (host sorts
frames by time, GPU assembles them into the dada_db -g ring block) ->
paf_baseband2power (integrates in place) -> paf_dbdisk.  The spectra equal
the oracle's of the blocks placed from the same stream."""
import os
import subprocess
import time

import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
from paf_b2p import dada
from test_capture import make_stream
from test_df import EPOCHS, py_start_time

pytestmark = pytest.mark.gpu
BIN = dada.BIN_DIR


def far_future_copy(df_path, ck_path, ahead):
    """insert, mid-stream, a copy of one frame whose timestamp lies `ahead`
    frames later (a corrupt or far-future header)"""
    dfs = np.fromfile(df_path, np.uint8).reshape(-1, npo.DF_BYTES)
    ck = np.fromfile(ck_path, np.uint8)
    i = len(dfs) // 2
    h = dada.df_decode(dfs[i].tobytes())
    tot = h.idf + ahead
    bad = dfs[i].copy()
    bad[:64] = np.frombuffer(dada.df_encode(tot % 250000, h.sec + 27 * (tot // 250000), h.valid, h.epoch,
                                            h.beam, h.freq), np.uint8)
    np.concatenate([dfs[:i], bad[None], dfs[i:]]).tofile(df_path)
    np.concatenate([ck[:i], ck[i:i + 1], ck[i:]]).tofile(ck_path)


@pytest.mark.parametrize("inject", [False, True])
def test_udp_capture_to_spectra(gpu, tmp_path, inject):
    nchunk, block_ndf, nblk = 8, 64, 4
    g, payload, df, ck = make_stream(tmp_path, nchunk=nchunk, nblk=nblk, block_ndf=block_ndf,
                                     window=block_ndf * nchunk * 3 // 2, seed=11, epoch=37)
    efile = tmp_path / "epoch.txt"
    efile.write_text(EPOCHS)
    if inject:  # one frame 10 blocks (640 frames) ahead, past the far limit 64 + 2 x 256:
        # dropped, no block switch (capture.c:491-508)
        far_future_copy(df, ck, 10 * block_ndf)
    hdr = tmp_path / "hdr.txt"
    hdr.write_text(f"HDR_SIZE 4096\nNBIT 16\nNDIM 2\nNPOL 2\nNCHAN {nchunk * 7}\nNCHUNK {nchunk}\n"
                   "NCHAN_CHUNK 7\nNSAMP_DF 128\nBYTE_ORDER BE\nTSAMP 0.84375\nUTC_START unset\n"
                   "FREQ 0\n")
    kin, kout = 0x7f40 + (os.getpid() % 16) * 4, 0x7f80 + (os.getpid() % 16) * 4
    for k in (kin, kout):
        dada.destroy_ring(k)
    dada.create_ring(kin, 3, g.block_bytes, device=0)
    dada.create_ring(kout, 4, g.nout * 4)
    port = 25000 + (os.getpid() % 500) * 8
    procs = []
    try:
        odir = tmp_path / "files"
        odir.mkdir()
        # the sink names the file by the DADA rule, <UTC_START>_<OBS_OFFSET>.000000.dada
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-D", str(odir)],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b",
                                   f"{kout:x}", "-c", str(tmp_path), "-d", "0"],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([os.path.join(BIN, "paf_capture"), "-a", f"{kin:x}", "-f", str(hdr),
                                   "-c", str(block_ndf), "-n", str(nblk), "-P", str(port), "-N", "3",
                                   "-m", "freq:1300", "-x", "249990", "-s", "54", "-t", "1",
                                   "-g", str(efile), "-i", "1340.5", "-b", "1", "-d", "0"],
                                  stderr=subprocess.PIPE, text=True)]
        time.sleep(3)  # capture opens its context and binds before the sender starts
        snd = subprocess.run([os.path.join(BIN, "paf_dfsend"), "-i", str(df), "-k", str(ck), "-P",
                              str(port), "-N", "3", "-r", "200"], capture_output=True, text=True)
        assert snd.returncode == 0, snd.stderr
        errs = []
        for p in procs[::-1]:
            _, e = p.communicate(timeout=120)
            errs.append(e)
            assert p.returncode == 0, e[-800:]
        cap_log = errs[0]
        files = os.listdir(odir)
        assert len(files) == 1, files
        out = odir / files[0]
        ohdr, data = dada.read_dada_file(str(out))
        sp = data.view(np.float32).reshape(-1, g.nout)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
    dfs = np.fromfile(df, np.uint8).reshape(-1, npo.DF_BYTES)
    chunk = np.fromfile(ck, np.uint8)
    assert sp.shape[0] == nblk, cap_log
    assert f", {int(inject)} far ahead," in cap_log
    idf, sec = 249990, 54
    for b in range(nblk):
        want = np.zeros(g.block_bytes, np.uint8)
        co.assemble(dfs, chunk, idf, sec, want, block_ndf, nchunk)
        assert np.array_equal(want, payload[b * g.block_bytes:(b + 1) * g.block_bytes])
        assert np.array_equal(sp[b].view(np.uint32), co.power(g, want).view(np.uint32)), cap_log
        gi = idf + block_ndf
        idf, sec = gi % 250000, sec + (gi // 250000) * 27
    assert "0.000% lost" in cap_log
    # start time of the first block's reference frame (idf 249990, sec 54,
    # epoch 37 -> 17713 days): capture.c:791-843, then carried through the
    # integrator's output header to the sink's file name
    utc, ps = py_start_time(249990, 54, 17713.0)
    assert (utc, ps) == ("2018-07-01-00:01:20", 998920000000)
    assert dada.header_get(ohdr, "UTC_START", "%s") == utc
    assert dada.header_get(ohdr, "PICOSECONDS", "%llu") == ps
    assert dada.header_get(ohdr, "FREQ", "%f") == 1340.5
    assert files[0] == f"{utc}_0000000000000000.000000.dada"
    assert f"UTC_START {utc}" in cap_log
