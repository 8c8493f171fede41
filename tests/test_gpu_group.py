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
