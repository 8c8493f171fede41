"""The drop-in C stage at the BASELINE multi-sub-band sizes (and configs[0]
from a file, last test).

configs[3] (4 sub-bands x 256 ch x 2 pol int8) and configs[4] (8 sub-bands x
1024 ch x 2 pol int8) run through `paf_baseband2power -n N`, the process the
reference's launcher would spawn per stage (paf-baseband2power.py:88-92,
114-115): N GPU-resident input rings of full 1024x1024-sample blocks (1 GiB /
4 GiB), filled by one `paf_dfdb -R` producer each (the counter-based
synthetic stream of sub-band r, block b), the stage gathering each round's
N spectra into one output block (-G copy: the members share the test box's
one GPU, which RCCL refuses), drained by `paf_dbdisk`.  Two blocks per ring
keep configs[4] inside one GPU's HBM (8 rings x 3 slots x 4 GiB).  Every N x NCHAN
output block is checked against the C oracle of the same bytes, bit for
bit, and the output header's NSUBBAND equals N."""
import os
import subprocess

import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
import paf_b2p
from paf_b2p import dada
from test_gpu_device_ring import BIN, _wait, fresh_key

pytestmark = pytest.mark.gpu
SEED = 20181105
NBLK = 2


def _oracle_of_device_block(it, scratch, g, subband, block):
    """regenerate block `block` of sub-band `subband` on the GPU (the same
    b2p_fill_synthetic call paf_dfdb made), download it in 256 MiB chunks of
    whole frames and sum it with the C oracle"""
    it.fill_synthetic(scratch, SEED, subband, block)
    it.sync()
    step = max(1, (256 << 20) // g.frame_bytes) * g.frame_bytes
    acc = np.zeros(g.nout, dtype=np.uint64)
    for off in range(0, g.block_bytes, step):
        n = min(step, g.block_bytes - off)
        co.integrate(g, it.download(scratch, nbytes=n, offset=off), nthreads=16, acc=acc)
    return co.finalize(g, acc)


@pytest.mark.parametrize("nsub,nchan", [pytest.param(4, 256, id="configs3_4x256ch_1GiB"),
                                        pytest.param(8, 1024, id="configs4_8x1024ch_4GiB")])
def test_c_stage_gathers_full_size_subbands(gpu, tmp_path, nsub, nchan):
    g = npo.Geom(nbit=8, nchan_chunk=nchan, nsamp_int=1 << 20)  # 1 GiB (256 ch) / 4 GiB (1024 ch)
    kout = fresh_key()
    base = fresh_key()
    keys = [base + 0x10 * r for r in range(nsub)]
    hdr = tmp_path / "hdr.txt"
    hdr.write_text(f"HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN {nchan}\nTSAMP 0.84375\n")
    for k in keys + [kout]:
        dada.destroy_ring(k)
    procs = []
    try:
        # NBLK blocks + the end-of-data block fit each ring, so every producer
        # finishes before the stage starts: with the 8 ring holders, at most
        # 11 processes use the box's GPU at once (its limit is 16)
        for k in keys:
            dada.create_ring(k, NBLK + 1, g.block_bytes, device=0)
        dada.create_ring(kout, 4, nsub * g.nout * 4)
        for r, k in enumerate(keys):
            _wait([subprocess.Popen([os.path.join(BIN, "paf_dfdb"), "-a", f"{k:x}", "-b", str(hdr), "-R",
                                     str(NBLK), "-f", f"int8:{nchan}", "-r", str(SEED), "-u", str(r)],
                                    stderr=subprocess.PIPE)], timeout=120)
        out = tmp_path / "power.dada"
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{base:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp_path), "-d", "0", "-f", f"int8:{nchan}", "-n", str(nsub),
                                   "-G", "copy"], stderr=subprocess.PIPE)]
        _wait(procs, timeout=600)
        ohdr, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in keys + [kout]:
            dada.destroy_ring(k)
    log = open(str(tmp_path / "paf_baseband2power.log")).read()
    sp = data.view(np.uint32).reshape(-1, nsub, g.nout)
    assert sp.shape[0] == NBLK, log[-800:]
    assert dada.header_get(ohdr, "NSUBBAND", "%d") == nsub
    assert dada.header_get(ohdr, "NBIT", "%d") == 32
    with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict())) as it:
        scratch = it.alloc(g.block_bytes)
        # the GPU generator is the oracle's generator: a prefix of sub-band 1,
        # block 1 regenerated on the host matches the GPU's bytes
        it.fill_synthetic(scratch, SEED, 1, 1)
        it.sync()
        assert np.array_equal(it.download(scratch, nbytes=1 << 20),
                              co.fill_synthetic(g, 1 << 20, SEED, 1, 1))
        for b in range(NBLK):
            for r in range(nsub):
                want = _oracle_of_device_block(it, scratch, g, r, b)
                assert np.array_equal(sp[b, r], want.view(np.uint32)), (nsub, nchan, b, r)
        scratch.free()
    # distinct sub-bands really are distinct (a mixed-up gather would show)
    assert len({sp[0, r].tobytes() for r in range(nsub)}) == nsub


def test_c_stage_configs0_file_through_host_ring(gpu, tmp_path):
    """configs[0], the reference's own CPU-runnable case, through the GPU
    drop-in: a DADA file of two full 1024x1024-sample integrations (256 ch x
    2 pol int8, 1 GiB each) and half of a third -> `paf_diskdb` -> a HOST
    ring of 1 GiB blocks (paf-baseband2power.py:114's shape) -> the stage
    (push from the registered ring block through the staging chunks) ->
    `paf_dbdisk`.  Both spectra equal the C oracle's of the file's bytes, bit
    for bit; the half integration at the end of the file is skipped."""
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 20)   # 1 GiB
    nblk = 2
    payload = co.fill_synthetic(g, nblk * g.block_bytes + g.block_bytes // 2, SEED, 0, 0)
    src = tmp_path / "c1.dada"
    dada.write_dada_file(str(src), "FILE_HEADER_IS_SKIPPED 1\n", payload)
    want = [co.power(g, payload[b * g.block_bytes:(b + 1) * g.block_bytes], nthreads=16) for b in range(nblk)]
    del payload
    hdr = tmp_path / "hdr.txt"
    hdr.write_text("HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\nTSAMP 0.84375\n")
    kin, kout = fresh_key(), fresh_key()
    dada.create_ring(kin, 2, g.block_bytes)
    dada.create_ring(kout, 4, g.nout * 4)
    out = tmp_path / "power.dada"
    procs = []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp_path), "-d", "0", "-f", "int8:256"], stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_diskdb"), "-a", f"{kin:x}", "-b", str(tmp_path), "-c",
                                   "c1.dada", "-d", str(hdr), "-e", "1", "-T", "4"], stderr=subprocess.PIPE)]
        _wait(procs, timeout=300)
        ohdr, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
    log = open(str(tmp_path / "paf_baseband2power.log")).read()
    sp = data.view(np.uint32).reshape(-1, g.nout)
    assert sp.shape[0] == nblk, log[-800:]
    for b in range(nblk):
        assert np.array_equal(sp[b], want[b].view(np.uint32)), b
    assert "partial integration skipped" in log and f"FINISH PAF_PROCESS: {nblk} integrations" in log, log[-800:]
    assert dada.header_get(ohdr, "NBIT", "%d") == 32 and dada.header_get(ohdr, "NCHAN", "%d") == 256
