"""N>1 path on CPU: world_size-2 gloo processes, one sub-band each, spectra
gathered to rank 0 in sub-band order, max-over-ranks timing (the same
functions bench.py uses with RCCL)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ORACLE, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    import b2p_oracle as npo
    from paf_b2p import distributed as D

    r, w, _ = D.env_ranks()
    D.init("gloo", r)
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=64)
    steps = 3
    spec = []
    for k in range(steps):  # this rank's sub-band, 3 integrations
        buf = npo.fill_synthetic(g, g.block_bytes, 20181105, D.subband_of(r), k)
        spec.append(npo.power(g, buf))
    local = torch.from_numpy(np.stack(spec))
    got = D.gather_spectra(local)
    got2 = D.all_gather_spectra(local)      # the fallback keeps the same contract
    assert (got2 is None) == (r != 0)
    if r == 0:
        assert all(torch.equal(a, b) for a, b in zip(got, got2))
    el = D.max_over_ranks(0.5 + r)
    # what ran, read back: the live group and every rank's identity record
    seen = D.observed_world()
    assert seen == {"backend": "gloo", "world_size": w, "rccl_ranks": 0}
    ids = D.gather_identities({"rank": r, "host": "h", "pci_bus_id": f"0000:{r % 2:02x}:00.0"})
    assert [i["rank"] for i in ids] == list(range(w))
    assert D.distinct_gpus(ids) == min(2, w)
    if r == 0:
        q.put(("gather", [t.numpy() for t in got], el))
    else:
        q.put(("peer", got, el))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_gather_and_max(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    sys.path.insert(0, ORACLE)
    import b2p_oracle as npo
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=64)
    root = [x for x in res if x[0] == "gather"][0]
    assert all(x[2] == world - 0.5 for x in res)          # max over ranks
    assert [x[1] for x in res if x[0] == "peer"] == [None] * (world - 1)
    for sb, arr in enumerate(root[1]):                    # rank order == sub-band order
        for k in range(3):
            buf = npo.fill_synthetic(g, g.block_bytes, 20181105, sb, k)
            assert np.array_equal(arr[k], npo.power(g, buf))


def test_aggregate_rate_formula():
    sys.path.insert(0, PKG)
    from paf_b2p import distributed as D
    # 8 ranks x 10 steps x 2^29 samples in 1 s
    assert D.aggregate_rate(8, 10, 1 << 29, 1.0) == 8 * 10 * (1 << 29) / 1e6


def _split_worker(rank, world, port, q):
    # SURVEY.md 8e second mode: one integration cut along time, exact
    # partial sums reduced to rank 0, rounded once there
    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    import b2p_oracle as npo
    from paf_b2p import distributed as D

    r, w, _ = D.env_ranks()
    D.init("gloo", r)
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7, nsamp_int=128 * 8)
    first, nf = D.time_share(r, w, g.nsamp_int // g.nsamp_df)
    parts = []
    for k in range(2):
        full = npo.fill_synthetic(g, g.block_bytes, 20181105, 0, k)
        mine = full[first * g.frame_bytes:(first + nf) * g.frame_bytes]
        parts.append(npo.integrate(g, mine).view(np.int64))
    # large values near the exactness limit travel unchanged too
    parts.append(np.full(g.nout, (1 << 52) // w + r, dtype=np.int64))
    tot = D.reduce_sums(torch.from_numpy(np.stack(parts)))
    q.put((r, None if tot is None else tot.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_time_split_reduce_is_exact():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    sys.path.insert(0, ORACLE)
    import b2p_oracle as npo
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7, nsamp_int=128 * 8)
    assert res[1] is None
    tot = res[0].view(np.uint64)
    for k in range(2):
        full = npo.fill_synthetic(g, g.block_bytes, 20181105, 0, k)
        assert np.array_equal(tot[k], npo.integrate(g, full))
        assert np.array_equal(npo.finalize(g, tot[k]), npo.power(g, full))
    assert np.all(tot[2] == (1 << 52) // world * world + sum(range(world)))


def test_time_share_rules():
    sys.path.insert(0, PKG)
    from paf_b2p import distributed as D
    assert [D.time_share(r, 4, 8192) for r in range(4)] == [(0, 2048), (2048, 2048),
                                                             (4096, 2048), (6144, 2048)]
    with pytest.raises(ValueError):
        D.time_share(0, 3, 8192)


def test_device_of_wraps_to_visible_devices(monkeypatch):
    sys.path.insert(0, PKG)
    from paf_b2p import distributed as D
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert [D.device_of(r) for r in (0, 3, 7)] == [0, 3, 7]
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert D.device_of(5) == 0          # one visible GPU per process
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert D.device_of(2) == 0
