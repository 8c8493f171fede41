"""GPU-resident DADA rings: data blocks in HBM owned by
a holder process (dada_db -g) and shared through HIP IPC handles.

* bytes written by one process come out of another unchanged;
* the three-process pipeline with the input ring on the GPU
  (paf_diskdb copies into HBM, paf_baseband2power integrates in place)
  matches the oracle;
* paf_dfdb assembles a raw data-frame stream (paf_dfgen) on the GPU straight
  into the ring block, and the spectra match the oracle of the original
  blocks, with and without lost frames; a corrupt far-future frame is left
  out, and a stream that jumps blocks ahead ends at the jump;
* replay mode hands out re-used blocks, spectra match the oracle;
* blocks already queued when the stage gets to them are integrated in one
  launch (b2p_integrate_n), spectra bit-equal to the oracle.
"""
import os
import re
import subprocess
import sys
import time

import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
from conftest import REPO
from paf_b2p import dada, pipeline

pytestmark = pytest.mark.gpu
SEED = 20181105
BIN = dada.BIN_DIR
HDR = os.path.join(os.path.dirname(BIN), "conf", "header_baseband2power.txt")
_next = [0x7a00 + (os.getpid() % 32) * 32]


def fresh_key():
    k = _next[0]
    _next[0] += 2
    dada.destroy_ring(k)
    return k


def _wait(procs, timeout=300):
    t_end = time.time() + timeout
    while any(p.poll() is None for p in procs) and time.time() < t_end:
        if any(p.poll() not in (None, 0) for p in procs):
            break
        time.sleep(0.05)
    bad = [p for p in procs if p.poll() != 0]
    for p in procs:
        if p.poll() is None:
            p.kill()
            p.wait()
    errs = [p.stderr.read().decode(errors="replace") for p in procs]
    msgs = [f"{os.path.basename(p.args[0])} rc={p.returncode}: {e[-600:]}" for p, e in zip(procs, errs)]
    if bad:  # the stage logs to <-c dir>/paf_baseband2power.log, not stderr
        for p in procs:
            a = list(p.args)
            if os.path.basename(a[0]) == "paf_baseband2power" and "-c" in a:
                log = os.path.join(a[a.index("-c") + 1], "paf_baseband2power.log")
                if os.path.exists(log):
                    msgs.append("stage log: " + open(log, errors="replace").read()[-2000:])
    assert not bad, "\n".join(msgs)
    return errs


# 29 952 B (12 frames of 2496 B) once failed in the holder: HIP served the
# block from a sub-allocated chunk and hipIpcGetMemHandle refused it
@pytest.mark.parametrize("bufsz", [1 << 16, 29952, 1040, (3 << 20) + 48])
def test_device_ring_bytes_cross_processes(gpu, tmp_path, bufsz):
    key = fresh_key()
    dada.create_ring(key, 3, bufsz, device=0)
    try:
        out = tmp_path / "o.dada"
        rd = subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{key:x}", "-o", str(out)],
                              stderr=subprocess.PIPE)
        rng = np.random.default_rng(1)
        blocks = [rng.integers(0, 256, bufsz, dtype=np.uint8).tobytes() for _ in range(5)]
        blocks.append(rng.integers(0, 256, bufsz // 3, dtype=np.uint8).tobytes())  # short = EOD
        with dada.Hdu(key, "W") as w:
            assert w.device == 0
            w.write_header("HDR_SIZE 4096\nNBIT 8\n")
            for b in blocks:
                w.write_block(b)
        _wait([rd])
        hdr, data = dada.read_dada_file(str(out))
        assert data.tobytes() == b"".join(blocks)
    finally:
        assert dada.destroy_ring(key)
    with pytest.raises(OSError):  # destroyed: the holder is gone with it
        dada.Hdu(key, "R")


def test_pipeline_with_device_input_ring(gpu, tmp_path):
    from test_gpu_pipeline import spectra, write_conf
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7, nsamp_int=64 * 128)
    nblk = 3  # three whole integrations, then a partial one the consumer must skip
    payload = co.fill_synthetic(g, g.block_bytes * nblk + g.block_bytes // 2, SEED, 0, 11)
    src = tmp_path / "bmf.dada"
    dada.write_dada_file(str(src), "NBIT 16\n", payload)
    conf = tmp_path / "p.conf"
    kin, kout = fresh_key(), fresh_key()
    write_conf(conf, 64, 48, 7168, 336, kin, kout, "header_baseband2power.txt")
    outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, str(src), layout="bmf", timeout=600,
                        device_ring=True)
    _, sp = spectra(outs[0], g.nout)
    assert sp.shape == (nblk, g.nout)
    for i in range(nblk):
        blk = payload[i * g.block_bytes:(i + 1) * g.block_bytes]
        assert np.array_equal(sp[i].view(np.uint32), co.power(g, blk, nthreads=8).view(np.uint32))
    log = open(os.path.join(str(tmp_path / "out"), "paf_baseband2power.log")).read()
    assert "GPU-resident" in log and "two launches in flight" in log
    assert "partial integration skipped" in log and "FINISH PAF_PROCESS: 3 integrations" in log


def _run_chain(tmp_path, kin, kout, producer, layout, nout, nbufs, bufsz, device=0, stage_args=()):
    dada.create_ring(kin, nbufs, bufsz, device=device)
    dada.create_ring(kout, 4, nout * 4)
    try:
        out = tmp_path / "power.dada"
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}",
                                   "-b", f"{kout:x}", "-c", str(tmp_path), "-d", "0", "-f", layout]
                                  + list(stage_args), stderr=subprocess.PIPE),
                 subprocess.Popen(producer, stderr=subprocess.PIPE)]
        msgs = _wait(procs)
        _, data = dada.read_dada_file(str(out))
        return data.view(np.float32).reshape(-1, nout), msgs[2]
    finally:
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)


@pytest.mark.parametrize("lost", [0, 40])
def test_dfdb_assembles_stream_into_device_ring(gpu, tmp_path, lost):
    nchunk, block_ndf, nblk = 48, 64, 4
    g = npo.Geom(nbit=16, big_endian=1, nchunk=nchunk, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=block_ndf * 128)
    payload = co.fill_synthetic(g, g.block_bytes * nblk, SEED, 2, 5)
    src = tmp_path / "bmf.dada"
    dada.write_dada_file(str(src), "NBIT 16\n", payload)
    df, ck = tmp_path / "s.df", tmp_path / "s.chunks"
    ref_idf, ref_sec = 249900, 27 * 40  # the stream crosses a 27-s period
    per_block = block_ndf * nchunk
    subprocess.run([os.path.join(BIN, "paf_dfgen"), "-i", str(src), "-o", str(df), "-n", str(nchunk),
                    "-c", str(ck), "-x", str(ref_idf), "-s", str(ref_sec), "-r", "7",
                    "-w", str(per_block * 3 // 2), "-l", str(lost)], check=True, capture_output=True)
    kin, kout = fresh_key(), fresh_key()
    sp, log = _run_chain(tmp_path, kin, kout,
                         [os.path.join(BIN, "paf_dfdb"), "-a", f"{kin:x}", "-b", HDR, "-c", str(df),
                          "-k", str(ck), "-n", str(nchunk), "-x", str(ref_idf), "-s", str(ref_sec)],
                         "bmf", g.nout, 3, g.block_bytes)
    dfs = np.fromfile(df, dtype=np.uint8).reshape(-1, npo.DF_BYTES)
    chunk = np.fromfile(ck, dtype=np.uint8)
    assert sp.shape[0] == nblk
    idf, sec = ref_idf, ref_sec
    for b in range(nblk):
        want = np.zeros(g.block_bytes, np.uint8)  # lost frames read as zeros
        co.assemble(dfs, chunk, idf, sec, want, block_ndf, nchunk)
        if not lost:
            assert np.array_equal(want, payload[b * g.block_bytes:(b + 1) * g.block_bytes])
        assert np.array_equal(sp[b].view(np.uint32), co.power(g, want, nthreads=8).view(np.uint32))
        gi = idf + block_ndf
        idf, sec = gi % 250000, sec + (gi // 250000) * 27
    assert ("0.000% lost" in log) == (lost == 0)


@pytest.mark.parametrize("case", ["corrupt_frame", "jump"])
def test_dfdb_far_future_frames(gpu, tmp_path, case):
    """A frame more than 2 blocks past the latest block seen is taken as
    corrupt (paf_dfdb.c header; capture.c:491-508 stops the capture at one):
    a single such frame is left out and every block still comes out; a
    stream whose timestamps jump 4 blocks ahead ends its blocks at the jump."""
    nchunk, block_ndf, nblk = 48, 16, 4
    g = npo.Geom(nbit=16, big_endian=1, nchunk=nchunk, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=block_ndf * 128)
    payload = co.fill_synthetic(g, g.block_bytes * nblk, SEED, 6, 1)
    ref_idf, ref_sec = 249_990, 27 * 40  # across a 27-s period
    dfs, chunk = npo.df_stream(payload, nchunk, ref_idf, ref_sec)
    t = np.arange(dfs.shape[0]) // nchunk
    c = np.arange(dfs.shape[0]) % nchunk
    if case == "corrupt_frame":
        sel = np.array([(block_ndf + 3) * nchunk + 5])  # one frame of block 1
        ahead = 5 * block_ndf
    else:
        sel = np.nonzero(t >= 2 * block_ndf)[0]  # blocks 2.. stamped 4 blocks later
        ahead = 4 * block_ndf
    gidf = ref_idf + t[sel] + ahead
    dfs[sel, :npo.DF_HDR] = npo.df_encode(gidf % 250000, ref_sec + (gidf // 250000) * 27, 1, 0, 0, 1300 + c[sel])
    df, ck = tmp_path / "s.df", tmp_path / "s.chunks"
    dfs.tofile(df)
    chunk.tofile(ck)
    kin, kout = fresh_key(), fresh_key()
    sp, log = _run_chain(tmp_path, kin, kout,
                         [os.path.join(BIN, "paf_dfdb"), "-a", f"{kin:x}", "-b", HDR, "-c", str(df),
                          "-k", str(ck), "-n", str(nchunk), "-x", str(ref_idf), "-s", str(ref_sec)],
                         "bmf", g.nout, 3, g.block_bytes)
    want_blocks = nblk if case == "corrupt_frame" else 2
    assert sp.shape[0] == want_blocks, log[-600:]
    idf, sec = ref_idf, ref_sec
    for b in range(want_blocks):
        want = np.zeros(g.block_bytes, np.uint8)
        co.assemble(dfs, chunk, idf, sec, want, block_ndf, nchunk)
        if case == "corrupt_frame" and b == 1:  # the corrupt frame's slot stays zero
            s0 = (3 * nchunk + 5) * npo.DF_PAYLOAD
            assert not want[s0:s0 + npo.DF_PAYLOAD].any()
        assert np.array_equal(sp[b].view(np.uint32), co.power(g, want, nthreads=8).view(np.uint32)), (case, b)
        gi = idf + block_ndf
        idf, sec = gi % 250000, sec + (gi // 250000) * 27
    placed = sum(int(x) for x in re.findall(r"block \d+: (\d+) of", log))
    assert placed == (nblk * block_ndf * nchunk - 1 if case == "corrupt_frame" else 2 * block_ndf * nchunk), log


def test_dfdb_lagging_source_drops_late_frames_only(gpu, tmp_path):
    """One source (chunk 0) arrives 4 blocks behind the others.  Its frames
    are more than one block late when they arrive, so paf_dfdb drops them,
    as the capture drops late frames (capture.c:464-531) -- and they must
    not hold its read-ahead back: before round 5 every batch's lowest block
    stayed 4 blocks back, the 6 batch slots overflowed and the oldest batch,
    holding most of the current block, was evicted (advisor, round 4).  Every
    block comes out with every on-time frame placed and chunk 0 empty."""
    nchunk, block_ndf, nblk, lag = 48, 16, 10, 4
    g = npo.Geom(nbit=16, big_endian=1, nchunk=nchunk, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=block_ndf * 128)
    payload = co.fill_synthetic(g, g.block_bytes * nblk, SEED, 7, 3)
    ref_idf, ref_sec = 1000, 27 * 40
    dfs, chunk = npo.df_stream(payload, nchunk, ref_idf, ref_sec)
    t = np.arange(dfs.shape[0]) // nchunk
    arrival = t + np.where(chunk == 0, lag * block_ndf, 0)
    order = np.argsort(arrival, kind="stable")
    df, ck = tmp_path / "s.df", tmp_path / "s.chunks"
    dfs[order].tofile(df)
    chunk[order].tofile(ck)
    kin, kout = fresh_key(), fresh_key()
    sp, log = _run_chain(tmp_path, kin, kout,
                         [os.path.join(BIN, "paf_dfdb"), "-a", f"{kin:x}", "-b", HDR, "-c", str(df),
                          "-k", str(ck), "-n", str(nchunk), "-x", str(ref_idf), "-s", str(ref_sec)],
                         "bmf", g.nout, 3, g.block_bytes)
    assert sp.shape[0] == nblk, log[-800:]
    placed = [int(x) for x in re.findall(r"block \d+: (\d+) of", log)]
    on_time = (nchunk - 1) * block_ndf
    assert len(placed) == nblk and all(p >= on_time for p in placed), (placed, log[-800:])
    assert "dropped for want of slots" not in log, log[-800:]
    on_time_only = chunk != 0
    idf = ref_idf
    for b in range(nblk - lag):  # the late source's frames of these blocks all came > 1 block late
        assert placed[b] == on_time, (b, placed)
        want = np.zeros(g.block_bytes, np.uint8)
        co.assemble(dfs[on_time_only], chunk[on_time_only], idf, ref_sec, want, block_ndf, nchunk)
        assert np.array_equal(sp[b].view(np.uint32), co.power(g, want, nthreads=8).view(np.uint32)), b
        idf += block_ndf


@pytest.mark.parametrize("device", [0, -1])  # GPU-resident ring, and a host ring for contrast
def test_replay_reuses_blocks(gpu, tmp_path, device):
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    nbufs, nrep = 3, 8
    kin, kout = fresh_key(), fresh_key()
    sp, _ = _run_chain(tmp_path, kin, kout,
                       [os.path.join(BIN, "paf_dfdb"), "-a", f"{kin:x}", "-b", HDR, "-R", str(nrep),
                        "-f", "int8:256", "-r", str(SEED)],
                       "int8:256", g.nout, nbufs, g.block_bytes, device=device)
    assert sp.shape[0] == nrep
    want = [co.power(g, co.fill_synthetic(g, g.block_bytes, SEED, 0, i)) for i in range(nbufs)]
    for i in range(nrep):
        assert np.array_equal(sp[i].view(np.uint32), want[i % nbufs].view(np.uint32))


def test_gathered_subbands_on_device_rings(gpu, tmp_path):
    # paf_baseband2power -n 2 with both input rings GPU-resident (one GPU on
    # the test box: both rings and both contexts on device 0, peer-copy gather)
    from test_gpu_pipeline import write_conf
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 14)
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\nTSAMP 0.84375\n")
    files, payloads = [], []
    for r in range(2):
        p = co.fill_synthetic(g, g.block_bytes * 2, SEED, r, 4)
        f = tmp_path / f"sb{r}.dada"
        dada.write_dada_file(str(f), "x 1\n", p)
        files.append(str(f))
        payloads.append(p)
    kin, kout = fresh_key(), fresh_key()
    dada.destroy_ring(kin + 0x10)
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 14, 1, 1024, 256, kin, kout, str(hfile))
    outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, files, nsub=2, gather=True,
                        device_ring=True, timeout=600)
    _, data = dada.read_dada_file(outs[0])
    sp = data.view(np.float32).reshape(-1, 2, 256)
    assert sp.shape[0] == 2
    for i in range(2):
        for r in range(2):
            blk = payloads[r][i * g.block_bytes:(i + 1) * g.block_bytes]
            assert np.array_equal(sp[i, r].view(np.uint32), co.power(g, blk).view(np.uint32))
    log = open(str(tmp_path / "out" / "paf_baseband2power.log")).read()
    assert log.count("GPU-resident (device 0)") == 2


def test_queued_blocks_are_integrated_in_one_launch(gpu, tmp_path):
    """the input ring is filled (7 whole integrations + the end of data)
    before the stage starts: it takes every queued block into one
    b2p_integrate_n launch, and each spectrum equals the oracle's"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    nblk = 7
    kin, kout = fresh_key(), fresh_key()
    dada.create_ring(kin, nblk + 1, g.block_bytes, device=0)
    dada.create_ring(kout, 4, g.nout * 4)
    try:
        payload = [co.fill_synthetic(g, g.block_bytes, SEED, 0, i) for i in range(nblk)]
        with dada.Hdu(kin, "W") as w:
            w.write_header(open(HDR).read())
            for p in payload:
                w.write_block(p.tobytes())
        out = tmp_path / "power.dada"
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}",
                                   "-b", f"{kout:x}", "-c", str(tmp_path), "-d", "0", "-f", "int8:256"],
                                  stderr=subprocess.PIPE)]
        _wait(procs)
        _, data = dada.read_dada_file(str(out))
        sp = data.view(np.float32).reshape(-1, g.nout)
        assert sp.shape[0] == nblk
        for i in range(nblk):
            assert np.array_equal(sp[i].view(np.uint32), co.power(g, payload[i]).view(np.uint32))
        log = open(str(tmp_path / "paf_baseband2power.log")).read()
        assert "launch 1: 7 integration(s) from 1" in log
        assert "1 integrate launches for 7 integrations, up to 7 queued blocks per launch" in log
    finally:
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)


def test_replaying_producer_keeps_the_stage_batching(gpu, tmp_path):
    """paf_dfdb -R re-hands ring blocks faster than one launch per block
    drains them: with every launch logged (-V) the launches
    add up to every block, several took more than one, none more than
    b2p_blocks_per_launch allows within the ring (6 blocks: 5), and every
    spectrum equals the oracle's of the block it read"""
    import re
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    nbufs, nrep = 6, 60
    kin, kout = fresh_key(), fresh_key()
    dada.create_ring(kin, nbufs, g.block_bytes, device=0)
    dada.create_ring(kout, 4, g.nout * 4)
    try:
        out = tmp_path / "power.dada"
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}",
                                   "-b", f"{kout:x}", "-c", str(tmp_path), "-d", "0", "-f", "int8:256", "-V"],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_dfdb"), "-a", f"{kin:x}", "-b", HDR, "-R", str(nrep),
                                   "-f", "int8:256", "-r", str(SEED)], stderr=subprocess.PIPE)]
        _wait(procs)
        _, data = dada.read_dada_file(str(out))
        sp = data.view(np.float32).reshape(-1, g.nout)
        assert sp.shape[0] == nrep
        want = [co.power(g, co.fill_synthetic(g, g.block_bytes, SEED, 0, i)) for i in range(nbufs)]
        for i in range(nrep):
            assert np.array_equal(sp[i].view(np.uint32), want[i % nbufs].view(np.uint32))
        log = open(str(tmp_path / "paf_baseband2power.log")).read()
        launches = [int(n) for n in re.findall(r"launch \d+: (\d+) integration", log)]
        assert sum(launches) == nrep and max(launches) <= nbufs - 1, launches
        assert sum(n > 1 for n in launches) >= 2, launches
    finally:
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)


def test_gathered_replays_in_batches(gpu, tmp_path):
    """paf_baseband2power -n 2 on two GPU-resident rings fed by replaying
    producers: every round integrates the same number of queued blocks per
    sub-band in one launch each and gathers them in one collective
    (b2p_group_gather_n); rounds add up to every block, several took more
    than one, and every output block holds both sub-bands' spectra of the
    blocks they read, equal to the oracle's"""
    import re
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    nbufs, nrep, nsub = 6, 40, 2
    base, kout = fresh_key(), fresh_key()
    kins = [base + 0x10 * q for q in range(nsub)]
    for k in kins:
        dada.destroy_ring(k)
        dada.create_ring(k, nbufs, g.block_bytes, device=0)
    dada.create_ring(kout, 4, nsub * g.nout * 4)
    try:
        out = tmp_path / "power.dada"
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{base:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp_path), "-d", "0", "-f", "int8:256", "-n", str(nsub), "-V"],
                                  stderr=subprocess.PIPE)]
        procs += [subprocess.Popen([os.path.join(BIN, "paf_dfdb"), "-a", f"{k:x}", "-b", HDR, "-R", str(nrep),
                                    "-f", "int8:256", "-r", str(SEED + q)], stderr=subprocess.PIPE)
                  for q, k in enumerate(kins)]
        _wait(procs)
        _, data = dada.read_dada_file(str(out))
        sp = data.view(np.float32).reshape(-1, nsub, g.nout)
        assert sp.shape[0] == nrep
        want = [[co.power(g, co.fill_synthetic(g, g.block_bytes, SEED + q, 0, i)) for i in range(nbufs)]
                for q in range(nsub)]
        for i in range(nrep):
            for q in range(nsub):
                assert np.array_equal(sp[i, q].view(np.uint32), want[q][i % nbufs].view(np.uint32)), (i, q)
        log = open(str(tmp_path / "paf_baseband2power.log")).read()
        rounds = [int(n) for n in re.findall(r"round \d+: (\d+) integration", log)]
        assert sum(rounds) == nrep and max(rounds) > 1, rounds
    finally:
        for k in kins + [kout]:
            dada.destroy_ring(k)


def test_gathered_rounds_stop_at_the_shorter_transfer(gpu, tmp_path):
    """two GPU-resident rings filled before the stage starts, 5 and 7 whole
    blocks: the gathered stage takes them in rounds of queued blocks, ends
    at the shorter transfer (5 output blocks, both sub-bands' spectra equal
    to the oracle's), counts the unmatched blocks as a skipped integration
    and exits cleanly"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    counts = [5, 7]
    base, kout = fresh_key(), fresh_key()
    kins = [base + 0x10 * q for q in range(2)]
    for k in kins:
        dada.destroy_ring(k)
        dada.create_ring(k, 8, g.block_bytes, device=0)
    dada.create_ring(kout, 8, 2 * g.nout * 4)
    try:
        payload = [[co.fill_synthetic(g, g.block_bytes, SEED + 7, q, i) for i in range(counts[q])]
                   for q in range(2)]
        for q, k in enumerate(kins):
            with dada.Hdu(k, "W") as w:
                w.write_header(open(HDR).read())
                for p in payload[q]:
                    w.write_block(p.tobytes())
        out = tmp_path / "power.dada"
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{base:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp_path), "-d", "0", "-f", "int8:256", "-n", "2"],
                                  stderr=subprocess.PIPE)]
        _wait(procs)
        _, data = dada.read_dada_file(str(out))
        sp = data.view(np.float32).reshape(-1, 2, g.nout)
        assert sp.shape[0] == 5
        for i in range(5):
            for q in range(2):
                want = co.power(g, payload[q][i])
                assert np.array_equal(sp[i, q].view(np.uint32), want.view(np.uint32)), (i, q)
        log = open(str(tmp_path / "paf_baseband2power.log")).read()
        assert "partial integration skipped (a sub-band's transfer ended)" in log
        assert "FINISH PAF_PROCESS: 5 integrations, 1 skipped, ok" in log
    finally:
        for k in kins + [kout]:
            dada.destroy_ring(k)


def _read_with_timeout(hdu, seconds=30):
    import threading
    got = []
    t = threading.Thread(target=lambda: got.append(hdu.read_block()), daemon=True)
    t.start()
    t.join(seconds)
    return got[0] if got else "TIMEOUT"


@pytest.mark.parametrize("nsub", [1, 2])
def test_real_time_spectra_do_not_wait_for_the_next_block(gpu, tmp_path, nsub):
    """a real-time producer: one block at a time, the next only after the
    previous block's spectrum has come out -- which it must, since nothing
    is queued behind it (outputs do not trail by a block / two rounds);
    spectra equal the oracle's"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    base, kout = fresh_key(), fresh_key()
    kins = [base + 0x10 * q for q in range(nsub)]
    for k in kins:
        dada.destroy_ring(k)
        dada.create_ring(k, 4, g.block_bytes, device=0)
    dada.create_ring(kout, 4, nsub * g.nout * 4)
    proc = None
    ws = []
    try:
        ws = [dada.Hdu(k, "W") for k in kins]
        for w in ws:
            w.write_header(open(HDR).read())
        proc = subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{base:x}", "-b", f"{kout:x}",
                                 "-c", str(tmp_path), "-d", "0", "-f", "int8:256"]
                                + (["-n", str(nsub)] if nsub > 1 else []), stderr=subprocess.PIPE)
        with dada.Hdu(kout, "R") as r:
            r.read_header()
            for i in range(4):
                blocks = [co.fill_synthetic(g, g.block_bytes, SEED + 11, q, i) for q in range(nsub)]
                for w, b in zip(ws, blocks):
                    w.write_block(b.tobytes())
                got = _read_with_timeout(r)
                assert got != "TIMEOUT", f"spectrum {i} did not come out before block {i + 1}"
                sp = np.frombuffer(got, np.float32).reshape(nsub, g.nout)
                for q in range(nsub):
                    assert np.array_equal(sp[q].view(np.uint32), co.power(g, blocks[q]).view(np.uint32))
            for w in ws:
                w.close()
            ws = []
            assert _read_with_timeout(r) is None
        assert proc.wait(timeout=60) == 0, proc.stderr.read().decode(errors="replace")[-800:]
    finally:
        for w in ws:
            w.close()
        if proc and proc.poll() is None:
            proc.kill()
            proc.wait()
        for k in kins + [kout]:
            dada.destroy_ring(k)


def _holder_pids(key):
    """pids of this ring's holder: the forked `dada_db -k KEY ... -g` process"""
    pids = []
    for d in os.listdir("/proc"):
        if d.isdigit():
            try:
                args = open(f"/proc/{d}/cmdline", "rb").read().split(b"\0")
            except OSError:
                continue
            if args and args[0].endswith(b"dada_db") and f"{key:x}".encode() in args and b"-g" in args:
                pids.append(int(d))
    return pids


def test_holder_frees_blocks_only_after_importers_detach(gpu):
    """the ordering rule of a device ring (dada_internal.h): while a process
    still has the blocks' IPC handles open, destroying the ring does not
    free them -- dada_db_destroy reports the attached importer (EBUSY, text
    in dada_device_error) and the holder keeps the memory; the moment the
    importer detaches, the holder frees the blocks and exits.  An importer
    that is killed counts as detached (the kernel drops its attachment)."""
    key = fresh_key()
    dada.create_ring(key, 2, 1 << 16, device=0)
    assert len(_holder_pids(key)) == 1
    v = dada.Hdu(key, "r")  # a viewer: connected, every block's handle imported
    try:
        t0 = time.time()
        assert not dada.destroy_ring(key)
        assert time.time() - t0 > 5  # it waited for the holder first
        assert "still have the blocks open" in dada.device_error(), dada.device_error()
        assert len(_holder_pids(key)) == 1  # memory still held for the importer
    finally:
        v.close()
    t_end = time.time() + 10
    while _holder_pids(key) and time.time() < t_end:
        time.sleep(0.05)
    assert not _holder_pids(key), "holder did not exit once the importer detached"
    # a killed importer: a child process attaches and is killed
    dada.create_ring(key, 2, 1 << 16, device=0)
    code = ("import sys, time; sys.path.insert(0, %r); from paf_b2p import dada; "
            "h = dada.Hdu(%d, 'r'); print('attached', flush=True); time.sleep(60)") % (
        os.path.join(REPO, "paf-baseband2power_amd"), key)
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
    try:
        assert child.stdout.readline().strip() == "attached"
        child.kill()
        child.wait()
        t0 = time.time()
        assert dada.destroy_ring(key), dada.device_error()
        assert time.time() - t0 < 5
    finally:
        if child.poll() is None:
            child.kill()
            child.wait()
    assert not _holder_pids(key)


def test_device_ring_info_reports_the_holder(gpu):
    """dada_device_ring_info on a real HIP holder: serving, its pid live, no
    ring block exported after a retry; a process that opens the blocks is
    counted as an importer within a holder tick; after destroy the ring is
    gone (ENOENT) and so is the holder"""
    key = fresh_key()
    dada.create_ring(key, 3, 1 << 20, device=0)
    try:
        info = dada.device_ring_info(key)
        assert info["device"] == 0 and info["holder_state"] == 1 and info["export_retries"] == 0, info
        assert os.path.exists(f"/proc/{info['holder_pid']}")
        assert _holder_pids(key) == [info["holder_pid"]]
        v = dada.Hdu(key, "r")
        try:
            t_end = time.time() + 5
            while dada.device_ring_info(key)["importers"] < 1 and time.time() < t_end:
                time.sleep(0.05)
            assert dada.device_ring_info(key)["importers"] == 1
        finally:
            v.close()
    finally:
        assert dada.destroy_ring(key), dada.device_error()
    with pytest.raises(OSError):
        dada.device_ring_info(key)
    assert not _holder_pids(key)
