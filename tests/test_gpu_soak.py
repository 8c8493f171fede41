"""Soak: the GPU-resident ring stage under a replaying producer for many
thousands of blocks, every output spectrum checked bit for bit.

The short ring tests (test_gpu_device_ring.py) cover each mechanism once.
Here the same mechanisms run for tens of thousands of launches back to back,
so that a rare ordering fault would show as a wrong spectrum:

* the replica banks that alternate between batched launches;
* the finalize that one launch carries for the previous one;
* the fences that release ring blocks;
* the gathered rounds of `-n 2`, and the time-split reduce of `-t 2`.

Small blocks (16 MiB, a 2-3 us kernel) put the semaphore / fence / launch
machinery at its highest rate, on device rings and on a host ring.
Full-size configs[1] blocks (1 GiB) run the production launch shape. `paf_dfdb -R` fills ring buffer i with synthetic
block i once and re-hands it, so output k must equal the oracle of block
k mod nbufs.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
from paf_b2p import dada
from test_gpu_device_ring import BIN, HDR, SEED, _wait, fresh_key

pytestmark = pytest.mark.gpu


def _soak(tmp_path, g, nbufs, nrep, nsub=1, timeout=300, device=0, stage_args=()):
    base, kout = fresh_key(), fresh_key()
    kins = [base + 0x10 * q for q in range(nsub)]
    for k in kins:
        dada.destroy_ring(k)
        dada.create_ring(k, nbufs, g.block_bytes, device=device)
    dada.create_ring(kout, 16, nsub * g.nout * 4)
    try:
        out = tmp_path / "power.dada"
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{base:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp_path), "-d", "0", "-f", f"int8:{g.nchan_chunk}"]
                                  + (["-n", str(nsub)] if nsub > 1 else []) + list(stage_args),
                                  stderr=subprocess.PIPE)]
        procs += [subprocess.Popen([os.path.join(BIN, "paf_dfdb"), "-a", f"{k:x}", "-b", HDR, "-R", str(nrep),
                                    "-f", f"int8:{g.nchan_chunk}", "-r", str(SEED + q)], stderr=subprocess.PIPE)
                  for q, k in enumerate(kins)]
        _wait(procs, timeout=timeout)
        _, data = dada.read_dada_file(str(out))
        sp = data.view(np.uint32).reshape(-1, nsub, g.nout)
        assert sp.shape[0] == nrep
        want = np.stack([np.stack([co.power(g, co.fill_synthetic(g, g.block_bytes, SEED + q, 0, i),
                                            nthreads=16).view(np.uint32) for q in range(nsub)])
                         for i in range(nbufs)])                       # [nbufs, nsub, nout]
        exp = want[np.arange(nrep) % nbufs]
        bad = np.nonzero(np.any(sp != exp, axis=(1, 2)))[0]
        assert bad.size == 0, f"{bad.size} of {nrep} outputs differ, first at {bad[:8].tolist()}"
        return open(str(tmp_path / "paf_baseband2power.log")).read()
    finally:
        for k in kins + [kout]:
            dada.destroy_ring(k)


def test_soak_small_blocks_one_subband(gpu, tmp_path):
    """300 000 blocks of 16 MiB through an 8-block device ring"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    log = _soak(tmp_path, g, nbufs=8, nrep=300000)
    m = re.search(r"FINISH PAF_PROCESS: (\d+) integrations", log)
    assert m and int(m.group(1)) == 300000


def test_soak_small_blocks_gathered(gpu, tmp_path):
    """-n 2: 100 000 gathered rounds of two sub-bands (different seeds)"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    _soak(tmp_path, g, nbufs=6, nrep=100000, nsub=2)


def test_soak_small_blocks_host_ring(gpu, tmp_path):
    """a host ring: 50 000 16-MiB blocks copied H2D through the stage's double-
    buffered staging, each one released only after its copy"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    _soak(tmp_path, g, nbufs=4, nrep=50000, device=-1)


def test_soak_time_split_host_ring(gpu, tmp_path):
    """-t 2: 20 000 host-ring blocks, each cut by time over two contexts
    (both on the one test GPU) whose exact partial sums are reduced"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    log = _soak(tmp_path, g, nbufs=4, nrep=20000, device=-1, stage_args=["-t", "2"])
    assert "reduce of 2 time shares" in log


def test_soak_full_size_configs1_blocks(gpu, tmp_path):
    """10 000 configs[1] blocks (1 GiB each, 10 TiB read) through an 8-block
    device ring: the production launch shapes, queued blocks batched"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256)
    log = _soak(tmp_path, g, nbufs=8, nrep=10000)
    m = re.search(r"(\d+) integrate launches for (\d+) integrations", log)
    assert m and int(m.group(2)) == 10000 and int(m.group(1)) <= 10000


def test_soak_udp_capture_many_blocks(gpu, tmp_path):
    """paf_dfsend -> loopback UDP on 3 ports -> paf_capture (GPU assembly into
    a device ring) -> paf_baseband2power, 120 blocks of 64 frames x 8 chunks
    with arrival shuffled within 1.5 blocks and the 27-s frame-counter wrap
    crossed: every spectrum equals the oracle of the block assembled from the
    same stream, and no frame is lost"""
    import time
    from test_capture import make_stream
    nchunk, block_ndf, nblk = 8, 64, 120
    g, payload, df, ck = make_stream(tmp_path, nchunk=nchunk, nblk=nblk, block_ndf=block_ndf,
                                     window=block_ndf * nchunk * 3 // 2, seed=29)
    hdr = tmp_path / "hdr.txt"
    hdr.write_text(f"HDR_SIZE 4096\nNBIT 16\nNDIM 2\nNPOL 2\nNCHAN {nchunk * 7}\nNCHUNK {nchunk}\n"
                   "NCHAN_CHUNK 7\nNSAMP_DF 128\nBYTE_ORDER BE\nTSAMP 0.84375\n")
    kin, kout = fresh_key(), fresh_key()
    dada.create_ring(kin, 4, g.block_bytes, device=0)
    dada.create_ring(kout, 8, g.nout * 4)
    port = 26000 + (os.getpid() % 500) * 8
    out = tmp_path / "power.dada"
    procs = []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b",
                                   f"{kout:x}", "-c", str(tmp_path), "-d", "0"], stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([os.path.join(BIN, "paf_capture"), "-a", f"{kin:x}", "-f", str(hdr),
                                   "-c", str(block_ndf), "-n", str(nblk), "-P", str(port), "-N", "3",
                                   "-m", "freq:1300", "-x", "249990", "-s", "54", "-t", "1", "-d", "0"],
                                  stderr=subprocess.PIPE, text=True)]
        time.sleep(3)  # capture opens its context and binds before the sender starts
        snd = subprocess.run([os.path.join(BIN, "paf_dfsend"), "-i", str(df), "-k", str(ck), "-P",
                              str(port), "-N", "3", "-r", "100"], capture_output=True, text=True)
        assert snd.returncode == 0, snd.stderr
        errs = []
        for p in procs[::-1]:
            _, e = p.communicate(timeout=180)
            errs.append(e)
            assert p.returncode == 0, e[-800:]
        cap_log = errs[0]
        _, data = dada.read_dada_file(str(out))
        sp = data.view(np.float32).reshape(-1, g.nout)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
    assert "0.000% lost" in cap_log, cap_log[-600:]
    assert sp.shape[0] == nblk, cap_log[-600:]
    dfs = np.fromfile(df, np.uint8).reshape(-1, npo.DF_BYTES)
    chunk = np.fromfile(ck, np.uint8)
    idf, sec = 249990, 54
    want = np.zeros(g.block_bytes, np.uint8)
    for b in range(nblk):
        want[:] = 0
        co.assemble(dfs, chunk, idf, sec, want, block_ndf, nchunk)
        assert np.array_equal(want, payload[b * g.block_bytes:(b + 1) * g.block_bytes]), b
        assert np.array_equal(sp[b].view(np.uint32), co.power(g, want).view(np.uint32)), b
        gi = idf + block_ndf
        idf, sec = gi % 250000, sec + (gi // 250000) * 27
