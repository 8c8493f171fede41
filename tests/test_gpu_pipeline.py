"""End-to-end drop-in test on the GPU: the three-process DADA pipeline
(paf_diskdb -> paf_baseband2power -> paf_dbdisk, launched like
paf-baseband2power.py) against the oracle run on the input file.
"""
import os
import textwrap

import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
from paf_b2p import dada, pipeline

pytestmark = pytest.mark.gpu
SEED = 20181105


def write_conf(path, ndf, nchk, bytes_per_df, nchan_out, key_in, key_out, hfname):
    path.write_text(textwrap.dedent(f"""\
        [BasicConf]
        NSAMP_DF: 128
        NPOL_SAMP: 2
        NDIM_POL: 2
        NCHK_NIC: {nchk}
        BYTES_PER_DF: {bytes_per_df}
        [DiskdbConf]
        NDF: {ndf}
        NBLK: 3
        KEY: {key_in:x}
        KFNAME_PREFIX: diskdb
        NREADER: 1
        SOD: 1
        HFNAME: {hfname}
        [Baseband2powerConf]
        KEY: {key_out:x}
        KFNAME_PREFIX: baseband2power
        NREADER: 1
        SOD: 1
        NCHAN: {nchan_out}
        NBYTE: 4
        NBLK: 4
        """))


def spectra(path, nout):
    hdr, data = dada.read_dada_file(path)
    return hdr.decode(), data.view(np.float32).reshape(-1, nout)


@pytest.mark.parametrize("npol_out,mean,memcheck", [(1, 0, 0), (2, 1, 0), (1, 0, 1)])
def test_bmf_pipeline(gpu, tmp_path, npol_out, mean, memcheck):
    """memcheck 1: the launcher's -e (the reference's cuda-memcheck run,
    paf-baseband2power.py:89-90) -- the same spectra from the stage on the
    bounds-checked debug build of libpafb2p, which its log names"""
    # BMF-native TFTFP int16 BE, 64 DFs per block (8192 samples per integration),
    # 3 whole integrations + a partial one that must be skipped
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=64 * 128, npol_out=npol_out, mean=mean)
    nblk = 3
    payload = co.fill_synthetic(g, g.block_bytes * nblk + g.block_bytes // 2, SEED, 0, 9)
    src = tmp_path / "bmf.dada"
    dada.write_dada_file(str(src), "NBIT 16\n", payload)
    conf = tmp_path / "p.conf"
    write_conf(conf, 64, 48, 7168, 336, 0x6a10, 0x6b10, "header_baseband2power.txt")
    outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, str(src), npol_out=npol_out,
                        mean=bool(mean), layout="bmf", timeout=600, memcheck=memcheck)
    hdr, sp = spectra(outs[0], g.nout)
    assert sp.shape == (nblk, g.nout)
    for i in range(nblk):
        blk = payload[i * g.block_bytes:(i + 1) * g.block_bytes]
        assert np.array_equal(sp[i].view(np.uint32), co.power(g, blk, nthreads=8).view(np.uint32))
    assert dada.header_get(hdr, "NBIT", "%d") == 32
    assert dada.header_get(hdr, "NPOL", "%d") == npol_out
    assert dada.header_get(hdr, "NCHAN", "%d") == 336
    assert abs(dada.header_get(hdr, "TSAMP", "%lf") - 8192 * 27 / 32) < 1e-6
    log = open(os.path.join(str(tmp_path / "out"), "paf_baseband2power.log")).read()
    assert "partial integration skipped" in log and "FINISH PAF_PROCESS: 3 integrations" in log
    assert ("libpafb2p: debug build" in log) == bool(memcheck)


def test_int8_header_layout_two_subbands(gpu, tmp_path):
    # generic 256-chan int8 described by the input header; two sub-band
    # chains (rings KEY and KEY+0x10), both on the one visible GPU
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 16)
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nUTC_START 2018-11-05-00:00:00\n"
                     "NBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\nTSAMP 0.84375\n")
    files, payloads = [], []
    for r in range(2):
        p = co.fill_synthetic(g, g.block_bytes * 2, SEED, r, 0)
        f = tmp_path / f"sb{r}.dada"
        dada.write_dada_file(str(f), "x 1\n", p)
        files.append(str(f))
        payloads.append(p)
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 16, 1, 1024, 256, 0x6c10, 0x6d10, str(hfile))
    outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, files, nsub=2, timeout=600)
    for r in range(2):
        hdr, sp = spectra(outs[r], 256)
        assert sp.shape == (2, 256)
        for i in range(2):
            blk = payloads[r][i * g.block_bytes:(i + 1) * g.block_bytes]
            assert np.array_equal(sp[i].view(np.uint32), co.power(g, blk).view(np.uint32))
        assert abs(dada.header_get(hdr, "TSAMP", "%lf") - 0.84375 * (1 << 16)) < 1e-6
        assert dada.header_get(hdr, "NCHAN", "%d") == 256


def test_psrdada_mode_host_pipeline(gpu, tmp_path):
    """The PSRDADA-mode hosts (bin/psrdada_api: -DB2P_PSRDADA, compiled
    against the Appendix A declarations, linked against libpafdada) run the
    three-process chain: header read with ipcbuf_get_next_read /
    mark_cleared, ring blocks pinned as first seen, end of data from
    ipcbuf_eod, no libpafdada extension.  Spectra equal the oracle."""
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 16)
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nUTC_START 2018-11-05-00:00:00\n"
                     "NBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\nTSAMP 0.84375\n")
    payload = co.fill_synthetic(g, g.block_bytes * 3 + g.frame_bytes * 7, SEED, 6, 0)
    f = tmp_path / "sb.dada"
    dada.write_dada_file(str(f), "x 1\n", payload)
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 16, 1, 1024, 256, 0x6e40, 0x6e50, str(hfile))
    outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, str(f), timeout=600,
                        bin_dir=os.path.join(dada.BIN_DIR, "psrdada_api"))
    hdr, sp = spectra(outs[0], 256)
    assert sp.shape == (3, 256)
    for i in range(3):
        blk = payload[i * g.block_bytes:(i + 1) * g.block_bytes]
        assert np.array_equal(sp[i].view(np.uint32), co.power(g, blk).view(np.uint32))
    assert dada.header_get(hdr, "NBIT", "%d") == 32
    log = open(os.path.join(str(tmp_path / "out"), "paf_baseband2power.log")).read()
    assert "partial integration skipped" in log and "FINISH PAF_PROCESS: 3 integrations" in log


def test_stage_stops_cleanly_on_sigterm(gpu, tmp_path):
    """SIGTERM while paf_baseband2power waits for its next input block: the
    wait gives up, the stage ends its output transfer (end of data), the
    sink finishes with every spectrum so far, and the stage exits 0"""
    import signal
    import subprocess
    import time

    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 14)
    kin, kout = 0x6f00 + (os.getpid() % 32) * 4, 0x6f80 + (os.getpid() % 32) * 4
    for k in (kin, kout):
        dada.destroy_ring(k)
    dada.create_ring(kin, 3, g.block_bytes)
    dada.create_ring(kout, 4, g.nout * 4)
    out = tmp_path / "power.dada"
    procs = []
    try:
        procs.append(subprocess.Popen([os.path.join(dada.BIN_DIR, "paf_dbdisk"), "-k", f"{kout:x}",
                                       "-o", str(out)], stderr=subprocess.PIPE, text=True))
        stage = subprocess.Popen([os.path.join(dada.BIN_DIR, "paf_baseband2power"), "-a", f"{kin:x}",
                                  "-b", f"{kout:x}", "-c", str(tmp_path), "-d", "0"],
                                 stderr=subprocess.PIPE, text=True)
        procs.append(stage)
        blocks = [co.fill_synthetic(g, g.block_bytes, SEED, 7, k) for k in range(2)]
        log = tmp_path / "paf_baseband2power.log"
        with dada.Hdu(kin, "W") as w:
            w.write_header("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\n"
                           "TSAMP 0.84375\n")
            for b in blocks:
                w.write_block(b.tobytes())
            t_end = time.time() + 120
            while "integration 2:" not in (log.read_text() if log.exists() else ""):
                assert time.time() < t_end and stage.poll() is None, stage.stderr.read()
                time.sleep(0.1)
            time.sleep(0.3)                       # the stage is now waiting for block 3
            stage.send_signal(signal.SIGTERM)
            assert stage.wait(60) == 0, stage.stderr.read()
            assert procs[0].wait(60) == 0, procs[0].stderr.read()
        _, data = dada.read_dada_file(str(out))
        sp = data.view(np.float32).reshape(-1, g.nout)
        assert sp.shape == (2, g.nout)
        for k in range(2):
            assert np.array_equal(sp[k].view(np.uint32), co.power(g, blocks[k]).view(np.uint32))
        text = log.read_text()
        assert "stopped by a signal" in text and "FINISH PAF_PROCESS: 2 integrations" in text
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)


def test_stage_between_psrdada_neighbours(gpu, tmp_path):
    """The drop-in on the wire: paf_baseband2power (libpafdada) between
    PSRDADA processes -- its input ring written, and its output ring drained,
    by tests/psrdada_model.py, the independent statement of the reference's
    libpsrdada protocol.  Two integrations and a short
    block; spectra equal the oracle, the header carries the stage's keys."""
    import subprocess
    import threading

    import psrdada_model as pm

    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 14)
    kin, kout = 0x6f40 + (os.getpid() % 16) * 4, 0x6fc0 + (os.getpid() % 16) * 4
    for k in (kin, kout):
        dada.destroy_ring(k)
    dada.create_ring(kin, 3, g.block_bytes)
    dada.create_ring(kout, 4, g.nout * 4)
    blocks = [co.fill_synthetic(g, g.block_bytes, SEED, 8, k) for k in range(2)]
    got = {}

    def drain():  # a PSRDADA reader on the output ring (dada_dbdisk's role)
        hdr, data = pm.Ring(kout + 1), pm.Ring(kout)
        try:
            hdr.lock_read()
            data.lock_read()
            p, n = hdr.get_next_read()
            got["header"] = pm.C.string_at(p, n).split(b"\0")[0].decode()
            hdr.mark_cleared()
            got["spectra"] = data.read_transfer()
            data.unlock_read()
            hdr.unlock_read()
        finally:
            hdr.close()
            data.close()

    reader = threading.Thread(target=drain)
    reader.start()
    stage = subprocess.Popen([os.path.join(dada.BIN_DIR, "paf_baseband2power"), "-a", f"{kin:x}",
                              "-b", f"{kout:x}", "-c", str(tmp_path), "-d", "0"],
                             stderr=subprocess.PIPE, text=True)
    hdr, data = pm.Ring(kin + 1), pm.Ring(kin)
    try:  # a PSRDADA writer on the input ring (paf_diskdb / capture's role)
        hdr.lock_write()
        data.lock_write()
        hdr.write_block(pm.header_block(hdr, b"HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\n"
                                             b"NCHAN 256\nTSAMP 0.84375\n"))
        for b in blocks:
            data.write_block(b.tobytes())
        data.write_block(b"\1" * 999)  # a short block ends the transfer (skipped by the stage)
        data.unlock_write()
        hdr.unlock_write()
        assert stage.wait(120) == 0, stage.stderr.read()
        reader.join(60)
        assert not reader.is_alive()
    finally:
        hdr.close()
        data.close()
        if stage.poll() is None:
            stage.kill()
            stage.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
    assert len(got["spectra"]) == 2
    for k in range(2):
        sp = np.frombuffer(got["spectra"][k], dtype=np.float32)
        assert np.array_equal(sp.view(np.uint32), co.power(g, blocks[k]).view(np.uint32))
    assert dada.header_get(got["header"], "NBIT", "%d") == 32
    assert dada.header_get(got["header"], "NCHAN", "%d") == 256


def test_stage_on_an_empty_transfer(gpu, tmp_path):
    """a writer that locks, writes the header and no block (libpafdada ends
    such a transfer with one 0-byte end-of-data block): the stage writes its
    output header, no spectrum, ends its output transfer and exits 0"""
    import subprocess

    kin, kout = 0x6e80 + (os.getpid() % 16) * 4, 0x6ec0 + (os.getpid() % 16) * 4
    for k in (kin, kout):
        dada.destroy_ring(k)
    dada.create_ring(kin, 2, 1 << 24)
    dada.create_ring(kout, 2, 256 * 4)
    out = tmp_path / "power.dada"
    try:
        sink = subprocess.Popen([os.path.join(dada.BIN_DIR, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                stderr=subprocess.PIPE, text=True)
        stage = subprocess.Popen([os.path.join(dada.BIN_DIR, "paf_baseband2power"), "-a", f"{kin:x}",
                                  "-b", f"{kout:x}", "-c", str(tmp_path), "-d", "0"],
                                 stderr=subprocess.PIPE, text=True)
        with dada.Hdu(kin, "W") as w:
            w.write_header("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\nTSAMP 0.84375\n")
        assert stage.wait(120) == 0, stage.stderr.read()
        assert sink.wait(60) == 0, sink.stderr.read()
        hdr, data = dada.read_dada_file(str(out))
        assert data.size == 0 and dada.header_get(hdr, "NBIT", "%d") == 32
        assert "FINISH PAF_PROCESS: 0 integrations" in (tmp_path / "paf_baseband2power.log").read_text()
    finally:
        for p in (locals().get("stage"), locals().get("sink")):
            if p is not None and p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
