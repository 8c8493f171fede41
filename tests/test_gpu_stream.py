"""The integrator on a caller's HIP stream (b2p_set_stream), as bench.py's
RCCL path runs it: torch tensors in and out, everything ordered on one torch
stream, no b2p_sync between the last integration and torch's use of the
spectra.  Spectra must equal the oracle bit for bit.
"""
import numpy as np
import pytest
import torch

import b2p_oracle as npo
import oracle_c as co
import paf_b2p

pytestmark = pytest.mark.gpu

SEED = 20181105


def test_integrate_on_torch_stream_matches_oracle(gpu):
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 14)  # 16 MiB blocks
    nblk, k = 3, 5
    blocks = [co.fill_synthetic(g, g.block_bytes, SEED, 0, b) for b in range(nblk)]
    ref = [co.power(g, b) for b in blocks]
    ts = torch.cuda.Stream()
    with torch.cuda.stream(ts):
        with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict()), device=0) as it:
            it.set_stream(ts.cuda_stream)
            dev = [torch.from_numpy(b).to("cuda", non_blocking=False) for b in blocks]
            out = torch.full((k, g.nout), -1.0, dtype=torch.float32, device="cuda")
            it.set_timing(2)
            for i in range(k):
                it.push(dev[i % nblk].data_ptr(), g.block_bytes, True)
                it.finish_async(out[i].data_ptr(), True)
            it.set_timing(0)  # flushes the last finalize onto ts, returns without waiting
            total = out.sum(dim=1)  # torch work on the same stream, behind the finalize
            ts.synchronize()
            st = it.stats()
            got = out.cpu().numpy()
            it.set_stream(None)
    assert st["launches"] == k
    for i in range(k):
        assert np.array_equal(got[i].view(np.uint32), ref[i % nblk].view(np.uint32)), i
    assert np.allclose(total.cpu().numpy(), got.sum(axis=1))


def test_fused_integrate_on_torch_stream(gpu):
    g = npo.Geom(nbit=8, nchan_chunk=1024, nsamp_int=1 << 12)
    blocks = [co.fill_synthetic(g, g.block_bytes, SEED, 1, b) for b in range(2)]
    ts = torch.cuda.Stream()
    with torch.cuda.stream(ts):
        with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict()), device=0) as it:
            it.set_stream(ts.cuda_stream)
            dev = [torch.from_numpy(b).cuda() for b in blocks]
            out = torch.zeros((4, g.nout), dtype=torch.float32, device="cuda")
            for i in range(4):
                it.integrate((dev[i % 2].data_ptr(), g.block_bytes), out[i].data_ptr(), True)
            it.sync()
            got = out.cpu().numpy()
    for i in range(4):
        assert np.array_equal(got[i].view(np.uint32), co.power(g, blocks[i % 2]).view(np.uint32)), i
