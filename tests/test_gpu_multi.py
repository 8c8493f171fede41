"""b2p_integrate_n: several whole integrations in one launch must give the
same bits as one b2p_integrate per block, and as the oracle, whatever the
layout, block count, output placement and the calls around it."""
import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
import paf_b2p
from paf_b2p import _lib as L

pytestmark = pytest.mark.gpu
SEED = 20181105

LAYOUTS = {
    "int8_64": dict(nbit=8, nchan_chunk=64, nsamp_int=1 << 14),
    "int8_256_p2": dict(nbit=8, nchan_chunk=256, nsamp_int=1 << 13, npol_out=2, mean=1),
    "bmf_small": dict(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7, nsamp_int=128 * 16),
    "tftfp_8x8": dict(nbit=16, big_endian=1, nchunk=8, nsamp_df=128, nchan_chunk=8, nsamp_int=128 * 32),
    # the planner's other branches: a period split into whole-wave columns,
    # and a frame with no whole-wave divisor (rows of lcm(frame, 64))
    "int8_336": dict(nbit=8, nchan_chunk=336, nsamp_int=1 << 12),
    "int8_odd": dict(nbit=8, nchunk=11, nsamp_df=4, nchan_chunk=99, nsamp_int=4 * 64),
}


def same(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


@pytest.mark.parametrize("name", sorted(LAYOUTS))
@pytest.mark.parametrize("k", [1, 2, 5, 8])
def test_integrate_n_equals_separate_and_oracle(gpu, name, k):
    g = npo.Geom(**LAYOUTS[name])
    hosts = [co.fill_synthetic(g, g.block_bytes, SEED, 4, b) for b in range(k)]
    with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict())) as it:
        ds = [it.upload(h) for h in hosts]
        multi = it.integrate_n(ds)                         # host output, blocking
        single = np.stack([it.integrate(d) for d in ds])
        for d in ds:
            d.free()
    assert multi.shape == (k, g.nout)
    for b in range(k):
        assert same(multi[b], single[b]), b
        assert same(multi[b], co.power(g, hosts[b])), b


def test_integrate_n_back_to_back_device_output(gpu):
    """three multi launches and single integrations interleaved without a
    host sync: each launch's deferred finalize rides on the next, the two
    replica banks alternate, every spectrum lands in its own device row"""
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 14)
    hosts = [co.fill_synthetic(g, g.block_bytes, SEED, 6, b) for b in range(6)]
    with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict())) as it:
        ds = [it.upload(h) for h in hosts]
        out = it.alloc(15 * g.nout * 4)
        row = 0
        plan = [[0, 1, 2], "s3", [3, 4, 5, 0], [1, 2], "s4", "s5", [5, 4, 3]]
        want = []
        for step in plan:
            if isinstance(step, str):
                b = int(step[1:])
                it.integrate(ds[b], out.ptr + row * g.nout * 4, True)
                want.append(b)
                row += 1
            else:
                it.integrate_n([ds[b] for b in step], out.ptr + row * g.nout * 4, True)
                want += step
                row += len(step)
        it.sync()
        got = it.download(out, nbytes=row * g.nout * 4).view(np.float32).reshape(row, g.nout)
        for d in ds:
            d.free()
        out.free()
    for r, b in enumerate(want):
        assert same(got[r], co.power(g, hosts[b])), (r, b)


def test_integrate_n_refusals(gpu):
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 12)
    with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict())) as it:
        d = it.alloc(g.block_bytes)
        it.fill_synthetic(d, SEED, 0, 0)
        with pytest.raises(paf_b2p.B2PError) as e:
            it.integrate_n([d] * 9)                    # more than B2P_MAX_BLOCKS
        assert e.value.code == L.B2P_EINVAL
        it.push((d, 0, g.frame_bytes))
        with pytest.raises(paf_b2p.B2PError):
            it.integrate_n([d, d])                     # a push is pending
        it.finish(allow_partial=True)
        with pytest.raises(paf_b2p.B2PError) as e:
            it.integrate_n([(d.ptr + 4, g.block_bytes)])   # misaligned block
        assert e.value.code == L.B2P_EALIGN
        out = it.integrate_n([d, d])
        assert same(out[0], out[1])
        d.free()


def test_fused_integrate_into_an_output_still_pending(gpu):
    """launch variant fuse=1: b2p_integrate emits its spectrum from the last
    workgroup of its own launch, while the extra workgroup of that launch
    finalizes the previous, deferred integration.  With both aimed at the
    same output (reused before b2p_sync) the newer spectrum must win -- the
    older one once landed last (tests/test_gpu_api_model.py found it)."""
    g = npo.Geom(nbit=16, nchunk=2, nsamp_df=2, nchan_chunk=12, nsamp_int=4)
    hosts = [co.fill_synthetic(g, g.block_bytes, SEED, 9, b) for b in range(2)]
    want = [co.power(g, h).view(np.uint32) for h in hosts]
    with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict()), tuning={"fuse": 1}) as it:
        ds = [it.upload(h) for h in hosts]
        out = it.alloc(6 * g.nout * 4)
        for _ in range(20):
            it.integrate_n([ds[0]] * 6, out.ptr, True)      # deferred: slots 0..5 <- block 0
            it.integrate(ds[1], out.ptr, True)               # fused: slot 0 <- block 1
            it.sync()
            got = it.download(out).view(np.uint32).reshape(6, g.nout)
            assert np.array_equal(got[0], want[1])
            for s in range(1, 6):
                assert np.array_equal(got[s], want[0])
        for d in ds + [out]:
            d.free()
