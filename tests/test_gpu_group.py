"""Multi-GPU gather on the one-GPU test box: RCCL with one
member, peer copies with members sharing the device, and the multi-sub-band
C host (one process, one thread per sub-band, spectra gathered)."""
import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
import paf_b2p
from paf_b2p import dada, pipeline

pytestmark = pytest.mark.gpu
SEED = 20181105


def _members(n, g):
    its = [paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict())) for _ in range(n)]
    bufs, specs = [], []
    for r, it in enumerate(its):
        d = it.alloc(g.block_bytes)
        it.fill_synthetic(d, SEED, r, 0)
        s = it.alloc(g.nout * 4)
        it.push(d)
        it.finish_async(s.ptr, True)  # deferred: the gather must flush it
        bufs.append(d)
        specs.append(s)
    return its, bufs, specs


@pytest.mark.parametrize("n,mode", [(1, 0), (3, 1)])
def test_group_gather(gpu, n, mode):
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 14, npol_out=2)
    its, bufs, specs = _members(n, g)
    root = its[0].alloc(n * g.nout * 4)
    with paf_b2p.Group(its, mode=mode) as grp:
        grp.gather([s.ptr for s in specs], root.ptr)
    got = its[0].download(root).view(np.float32).reshape(n, g.nout)
    for r in range(n):
        host = its[r].download(bufs[r])
        assert np.array_equal(got[r].view(np.uint32), co.power(g, host).view(np.uint32))
    for it, d, s in zip(its, bufs, specs):
        d.free()
        s.free()
    root.free()
    for it in its:
        it.close()


@pytest.mark.parametrize("n,mode", [(1, 0), (2, 1)])
def test_group_gather_async_behind_fences(gpu, n, mode):
    """b2p_group_gather_async: each member integrates 3 blocks in one launch
    (finalize left pending), then a second batch whose launch finalizes the
    first; the gather of batch 1 waits on the tickets fenced after that
    second launch, runs on the group's streams, lands member-major on the
    root and in pinned host memory; every spectrum equals the oracle's"""
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 14)
    nb = 3
    its = [paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict())) for _ in range(n)]
    blocks = [[its[r].alloc(g.block_bytes) for _ in range(2 * nb)] for r in range(n)]
    for r in range(n):
        for i, b in enumerate(blocks[r]):
            its[r].fill_synthetic(b, SEED, r, i)
    slots = [[its[r].alloc(nb * g.nout * 4) for _ in range(2)] for r in range(n)]
    root = its[0].alloc(n * nb * g.nout * 4)
    host = np.zeros(n * nb * g.nout, np.float32)
    with paf_b2p.Group(its, mode=mode) as grp:
        for r in range(n):
            its[r].integrate_n(blocks[r][:nb], slots[r][0].ptr, True)   # batch 1, finalize pending
        tickets = []
        for r in range(n):
            its[r].integrate_n(blocks[r][nb:], slots[r][1].ptr, True)   # finalizes batch 1
            tickets.append(its[r].fence())
        gt = grp.gather_async([slots[r][0].ptr for r in range(n)], nb, root.ptr, tickets,
                              host.ctypes.data)
        grp.wait(gt)
        got_root = its[0].download(root).view(np.float32).reshape(n, nb, g.nout)
        for r in range(n):
            for i in range(nb):
                want = co.power(g, its[r].download(blocks[r][i]))
                assert np.array_equal(got_root[r, i].view(np.uint32), want.view(np.uint32)), (r, i)
                assert np.array_equal(host.reshape(n, nb, g.nout)[r, i].view(np.uint32), want.view(np.uint32))
        for it in its:
            it.sync()
    for r in range(n):
        for b in blocks[r] + slots[r]:
            b.free()
    root.free()
    for it in its:
        it.close()


def test_multi_subband_c_host_gathered(gpu, tmp_path):
    from test_gpu_pipeline import write_conf
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 15)
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\n"
                     "TSAMP 0.84375\n")
    files, payloads = [], []
    for r in range(3):
        p = co.fill_synthetic(g, g.block_bytes * 2, SEED, r, 1)
        f = tmp_path / f"sb{r}.dada"
        dada.write_dada_file(str(f), "x 1\n", p)
        files.append(str(f))
        payloads.append(p)
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 15, 1, 1024, 256, 0x7a10, 0x7b10, str(hfile))
    outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, files, nsub=3, gather=True,
                        timeout=600)
    hdr, data = dada.read_dada_file(outs[0])
    sp = data.view(np.float32).reshape(-1, 3, 256)
    assert sp.shape[0] == 2
    assert dada.header_get(hdr, "NCHAN", "%d") == 768
    assert dada.header_get(hdr, "NSUBBAND", "%d") == 3
    for i in range(2):
        for r in range(3):
            blk = payloads[r][i * g.block_bytes:(i + 1) * g.block_bytes]
            assert np.array_equal(sp[i, r].view(np.uint32), co.power(g, blk).view(np.uint32))
    log = open(str(tmp_path / "out" / "paf_baseband2power.log")).read()
    assert "gather of 3 sub-bands" in log


def test_c_host_reports_rccl_setup_failure(gpu, tmp_path):
    """-n 2 on the one-GPU box with -G rccl: RCCL refuses two members on one
    device.  The stage must log the b2p_group_open failure and exit non-zero
    within its -T limit -- never hang (the first real multi-rank RCCL run is
    the driver's, so its failure has to be loud and bounded)."""
    import time
    from test_gpu_pipeline import write_conf
    if paf_b2p.device_count() != 1:
        pytest.skip("needs members that share one GPU")
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 12)
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\n"
                     "TSAMP 0.84375\n")
    files = []
    for r in range(2):
        f = tmp_path / f"sb{r}.dada"
        dada.write_dada_file(str(f), "x 1\n", co.fill_synthetic(g, g.block_bytes, SEED, r, 0))
        files.append(str(f))
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 12, 1, 1024, 256, 0x7c10, 0x7d10, str(hfile))
    t0 = time.time()
    with pytest.raises(RuntimeError) as e:
        pipeline.run(str(conf), str(tmp_path / "out"), 0, files, nsub=2, gather=True, timeout=120,
                     stage_args=["-G", "rccl", "-T", "20"])
    assert time.time() - t0 < 100
    assert "paf_baseband2power: rc=1" in str(e.value)
    log = open(str(tmp_path / "out" / "paf_baseband2power.log")).read()
    assert "b2p_group_open" in log and "member 1: GPU 0 (PCI" in log


@pytest.mark.parametrize("device", [False, True], ids=["host_ring", "device_ring"])
def test_c_host_rccl_gather_at_world_size_one(gpu, tmp_path, device):
    """`paf_baseband2power -n 1 -G rccl`: the C host's collective path with
    one RCCL member -- ncclCommInitRankConfig (non-blocking, inside one group
    call), then an ncclGather per integration (-S / host ring) or per round
    of queued blocks (GPU-resident ring), polled against the -T limit
    (csrc/b2p_group.hip, rccl.h:745) -- executed on the hardware, every
    spectrum equal to the oracle's.  The one multi-rank step this box cannot
    run is two RCCL members on distinct GPUs."""
    import os
    import subprocess
    from test_gpu_device_ring import BIN, _wait, fresh_key
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 14)  # 16 MiB blocks
    nblk = 3
    blocks = [co.fill_synthetic(g, g.block_bytes, SEED, 0, b) for b in range(nblk)]
    kin, kout = fresh_key(), fresh_key()
    hdr = "HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 256\nTSAMP 0.84375\n"
    (tmp_path / "hdr.txt").write_text(hdr)
    dada.create_ring(kin, nblk + 1, g.block_bytes, device=0 if device else -1)
    dada.create_ring(kout, 4, g.nout * 4)
    out = tmp_path / "power.dada"
    procs = []
    try:
        if device:  # the blocks and their end of data fit: the producer is done first
            _wait([subprocess.Popen([os.path.join(BIN, "paf_dfdb"), "-a", f"{kin:x}", "-b",
                                     str(tmp_path / "hdr.txt"), "-R", str(nblk), "-f", "int8:256", "-r",
                                     str(SEED), "-u", "0"], stderr=subprocess.PIPE)], timeout=120)
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp_path), "-d", "0", "-f", "int8:256", "-n", "1", "-G", "rccl",
                                   "-T", "60"], stderr=subprocess.PIPE)]
        if not device:
            with dada.Hdu(kin, "W") as w:
                w.write_header(hdr)
                for b in blocks:
                    w.write_block(b.tobytes())
        _wait(procs, timeout=180)
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
    log = open(str(tmp_path / "paf_baseband2power.log")).read()
    assert "gather of 1 sub-bands to GPU 0 via RCCL ncclGather" in log, log[-800:]
    sp = data.view(np.uint32).reshape(-1, g.nout)
    assert sp.shape[0] == nblk, log[-800:]
    for b in range(nblk):
        assert np.array_equal(sp[b], co.power(g, blocks[b], nthreads=8).view(np.uint32)), b


# ---- time-split mode (second mode) -----------------------------

@pytest.mark.parametrize("npol_out,mean", [(1, 0), (2, 1)])
def test_partial_sums_and_finalize(gpu, npol_out, mean):
    # exact sums out of one context, fp32 from them = the normal finish
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=128 * 32, npol_out=npol_out, mean=mean)
    block = co.fill_synthetic(g, g.block_bytes, SEED, 0, 3)
    with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict())) as it:
        d = it.upload(block)
        it.push(d)
        sums = it.finish_partial()                      # host, blocking
        assert np.array_equal(sums, co.integrate(g, block))
        ds, out = it.alloc(g.nout * 8 * 2), it.alloc(g.nout * 4 * 2)
        for k in range(2):                              # async, device rows
            it.push(d)
            it.finish_partial(ds.ptr + k * g.nout * 8, True)
        it.finalize_sums(ds.ptr, 2, out.ptr)
        it.sync()
        got = it.download(out).view(np.float32).reshape(2, g.nout)
        for b in (d, ds, out):
            b.free()
    want = co.power(g, block)
    assert all(np.array_equal(got[k].view(np.uint32), want.view(np.uint32)) for k in range(2))


@pytest.mark.parametrize("n,mode", [(1, 0), (4, 1)])
def test_group_time_split_equals_one_gpu(gpu, n, mode):
    # one BMF integration cut into n time shares, one member each; the
    # reduced exact sums round to the single-GPU spectrum bit for bit
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=128 * 64, mean=1)
    block = co.fill_synthetic(g, g.block_bytes, SEED, 5, 2)
    share = npo.Geom(**{**g.asdict(), "nsamp_int": g.nsamp_int // n})
    its = [paf_b2p.Integrator(paf_b2p.make_geom(**share.asdict())) for _ in range(n)]
    bufs, sums = [], []
    for r, it in enumerate(its):
        d = it.upload(block[r * share.block_bytes:(r + 1) * share.block_bytes])
        s = it.alloc(g.nout * 8)
        it.push(d)
        it.finish_partial(s.ptr, True)                  # deferred: reduce flushes it
        bufs.append(d)
        sums.append(s)
    root_sum, root_out = its[0].alloc(g.nout * 8), its[0].alloc(g.nout * 4)
    with paf_b2p.Group(its, mode=mode) as grp:
        grp.reduce([s.ptr for s in sums], g.nout, root_sum.ptr)
    its[0].finalize_sums(root_sum.ptr, 1, root_out.ptr, g.nsamp_int)
    its[0].sync()
    tot = its[0].download(root_sum).view(np.uint64)
    got = its[0].download(root_out).view(np.float32)
    assert np.array_equal(tot, co.integrate(g, block))
    assert np.array_equal(got.view(np.uint32), co.power(g, block).view(np.uint32))
    for b in bufs + sums + [root_sum, root_out]:
        b.free()
    for it in its:
        it.close()


@pytest.mark.parametrize("split,mean", [(3, 0), (2, 1)])
def test_c_host_time_split(gpu, tmp_path, split, mean):
    # paf_baseband2power -t N: one host ring, each integration cut by time over
    # N contexts (all on the one test GPU: peer-copy reduce), same spectra
    from test_gpu_pipeline import spectra, write_conf
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=128 * 48, mean=mean)
    nblk = 2
    payload = co.fill_synthetic(g, g.block_bytes * nblk + g.block_bytes // 3, SEED, 0, 21)
    src = tmp_path / "bmf.dada"
    dada.write_dada_file(str(src), "NBIT 16\n", payload)
    conf = tmp_path / "p.conf"
    write_conf(conf, 48, 48, 7168, 336, 0x7c30 + 0x40 * split, 0x7d30 + 0x40 * split,
               "header_baseband2power.txt")
    outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, str(src), layout="bmf", mean=bool(mean),
                        split=split, timeout=600)
    hdr, sp = spectra(outs[0], g.nout)
    assert sp.shape == (nblk, g.nout)
    for i in range(nblk):
        blk = payload[i * g.block_bytes:(i + 1) * g.block_bytes]
        assert np.array_equal(sp[i].view(np.uint32), co.power(g, blk, nthreads=8).view(np.uint32))
    assert dada.header_get(hdr, "NSPLIT", "%d") == split
    assert dada.header_get(hdr, "NSAMP_INT", "%d") == g.nsamp_int
    log = open(str(tmp_path / "out" / "paf_baseband2power.log")).read()
    assert f"reduce of {split} time shares" in log and "partial integration skipped" in log
