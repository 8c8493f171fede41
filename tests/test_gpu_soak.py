"""Soak: the GPU-resident ring stage under a replaying producer for many
thousands of blocks, every output spectrum checked bit for bit.

The short ring tests (test_gpu_device_ring.py) cover each mechanism once.
Here the same mechanisms run for tens of thousands of launches back to back,
so that a rare ordering fault would show as a wrong spectrum:

* the replica banks that alternate between batched launches;
* the finalize that one launch carries for the previous one;
* the fences that release ring blocks;
* the gathered rounds of `-n 2`, and the time-split reduce of `-t 2`.

Small blocks (16 KiB, a 5 us kernel) put the semaphore / fence / launch
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
    """300 000 blocks of 16 KiB through an 8-block device ring"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    log = _soak(tmp_path, g, nbufs=8, nrep=300000)
    m = re.search(r"FINISH PAF_PROCESS: (\d+) integrations", log)
    assert m and int(m.group(1)) == 300000


def test_soak_small_blocks_gathered(gpu, tmp_path):
    """-n 2: 100 000 gathered rounds of two sub-bands (different seeds)"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=256, nsamp_int=1 << 14)
    _soak(tmp_path, g, nbufs=6, nrep=100000, nsub=2)


def test_soak_small_blocks_host_ring(gpu, tmp_path):
    """a host ring: 50 000 blocks copied H2D through the stage's double-
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
