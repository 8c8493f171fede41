"""GPU parity: the HIP path (through the C ABI) against the oracle.

Bar: bit-identical fp32 output (exact integer accumulate, one RNE rounding).
Small cases compare with the committed fixtures and with the oracle on the
same seeded inputs; full BASELINE sizes compare with the multi-threaded C
oracle on the downloaded block and through size-independent properties
(chunking/order invariance, determinism, back-to-back integrations).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
import paf_b2p
from conftest import REPO, golden_geom, load_golden
from paf_b2p import _lib as L

pytestmark = pytest.mark.gpu

SEED = 20181105


def to_b2p(g: npo.Geom) -> L.Geom:
    return paf_b2p.make_geom(**g.asdict())


def gpu_power(g: npo.Geom, buf: np.ndarray, splits=None, host=False, register=False,
              tuning=None) -> np.ndarray:
    with paf_b2p.Integrator(to_b2p(g), device=0, tuning=tuning) as it:
        bounds = [0] + list(splits or []) + [buf.size]
        if host:
            hb = np.ascontiguousarray(buf)
            if register and hb.nbytes:
                it.register_host(hb)
            for a, b in zip(bounds[:-1], bounds[1:]):
                it.push(hb[a:b])
            if register and hb.nbytes:
                it.unregister_host(hb)
        else:
            d = it.upload(buf)
            for a, b in zip(bounds[:-1], bounds[1:]):
                it.push((d, a, b - a))
            out = it.finish(allow_partial=True)
            d.free()
            return out
        return it.finish(allow_partial=True)


def same_bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32),
                          np.asarray(b, np.float32).view(np.uint32))


@pytest.mark.parametrize("name", ["bmf_small", "int8_256", "int16le_48"])
@pytest.mark.parametrize("npol_out", [1, 2])
@pytest.mark.parametrize("mean", [0, 1])
def test_golden_fixtures(gpu, name, npol_out, mean):
    d = load_golden(name)
    g = golden_geom(d, npol_out=npol_out, mean=mean)
    out = gpu_power(g, d["input"])
    assert same_bits(out, d[f"power_p{npol_out}_m{mean}"])


@pytest.mark.parametrize("name", ["bmf_small", "int8_256", "int16le_48"])
def test_golden_host_push(gpu, name):
    d = load_golden(name)
    g = golden_geom(d)
    fb = g.frame_bytes
    nf = d["input"].size // fb
    splits = [fb * (nf // 3), fb * (2 * nf // 3)]
    assert same_bits(gpu_power(g, d["input"], host=True), d["power_p1_m0"])
    assert same_bits(gpu_power(g, d["input"], host=True, register=True, splits=splits),
                     d["power_p1_m0"])


# launch-shape branches of plan_launch(): NC=1 with whole waves, partial last
# wave, multi-column frames, non-64-multiple workgroup
GEOMS = {
    "int8_256": npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=4096),
    "int8_1024": npo.Geom(nbit=8, nchan_chunk=1024, nsamp_int=2048),
    "int16le_336": npo.Geom(nbit=16, nchan_chunk=336, nsamp_int=1024),        # B = 1008
    "bmf_8": npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7,
                      nsamp_int=128 * 8),                                      # NC = 21
    "bmf_3chunk": npo.Geom(nbit=16, big_endian=1, nchunk=3, nsamp_df=128, nchan_chunk=7,
                           nsamp_int=128 * 40),                                # B = 448
    "int8_odd": npo.Geom(nbit=8, nchunk=11, nsamp_df=4, nchan_chunk=99,
                         nsamp_int=4 * 64),                                    # B = 363
    "int8_3ch": npo.Geom(nbit=8, nchunk=1, nsamp_df=4, nchan_chunk=3, nsamp_int=4 * 999),
    "int16be_5x3": npo.Geom(nbit=16, big_endian=1, nchunk=5, nsamp_df=16, nchan_chunk=3,
                            nsamp_int=16 * 77),
    "tftfp_8x8": npo.Geom(nbit=16, big_endian=1, nchunk=8, nsamp_df=128, nchan_chunk=8,
                          nsamp_int=128 * 12),                                 # B = 512, NC = 8
}


@pytest.mark.parametrize("name", sorted(GEOMS))
@pytest.mark.parametrize("npol_out", [1, 2])
def test_layouts_vs_oracle(gpu, name, npol_out):
    g = npo.Geom(**{**GEOMS[name].asdict(), "npol_out": npol_out})
    buf = npo.fill_synthetic(g, g.block_bytes, SEED, 5, 7)
    assert same_bits(gpu_power(g, buf), npo.power(g, buf))


@pytest.mark.parametrize("name", sorted(GEOMS))
def test_chunked_pushes_equal_single(gpu, name):
    g = GEOMS[name]
    buf = co.fill_synthetic(g, g.block_bytes, SEED, 1, 2)
    nf = g.block_bytes // g.frame_bytes
    rng = np.random.default_rng(nf)
    cuts = sorted(set(int(x) * g.frame_bytes for x in rng.integers(1, nf, size=min(5, nf - 1))))
    whole = gpu_power(g, buf)
    assert same_bits(gpu_power(g, buf, splits=cuts), whole)
    assert same_bits(whole, co.power(g, buf))


@pytest.mark.parametrize("name", sorted(GEOMS))
def test_synthetic_generator_matches_oracle(gpu, name):
    g = GEOMS[name]
    n = min(g.block_bytes, 1 << 20) // 16 * 16
    eb = g.nbit // 8
    with paf_b2p.Integrator(to_b2p(g)) as it:
        d = it.alloc(n)
        for elem0 in (0, 16 // eb * 12345):
            it.fill_synthetic(d, SEED, 3, 11, elem0=elem0)
            assert np.array_equal(it.download(d), co.fill_synthetic(g, n, SEED, 3, 11, elem0))
        d.free()


def test_extreme_int8_long_lane_runs(gpu):
    # -128 everywhere, one workgroup row-group => every lane integrates all
    # 65536 rows: exercises the 32768-row widening and uint32 wrap (2^32/lane)
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 20, npol_out=2)
    buf = np.full(g.block_bytes, 0x80, dtype=np.uint8)
    out = gpu_power(g, buf, tuning={"row_groups": 1})
    assert np.all(out == np.float32((1 << 20) * 2 * 16384))
    out1 = gpu_power(npo.Geom(**{**g.asdict(), "npol_out": 1}), buf, tuning={"row_groups": 2})
    assert np.all(out1 == np.float32((1 << 20) * 4 * 16384))


def test_extreme_int16_be_full_bmf_block(gpu):
    # every component -32768 over a full 2.625 GiB BMF integration: 2^52/chan
    g = npo.BMF
    buf = np.tile(np.array([0x80, 0x00], dtype=np.uint8), g.block_bytes // 2)
    out = gpu_power(g, buf)
    assert np.all(out == np.float32(2.0 ** 52))
    del buf


def test_full_config2_block_vs_c_oracle(gpu):
    # BASELINE configs[1]: 256 ch x 2 pol int8, 1024x1024 samples (1 GiB)
    for npol_out in (1, 2):
        g = npo.Geom(nbit=8, nchan_chunk=256, npol_out=npol_out)
        with paf_b2p.Integrator(to_b2p(g)) as it:
            d = it.alloc(g.block_bytes)
            it.fill_synthetic(d, SEED, 0, 0)
            it.push(d)
            out = it.finish()
            host = it.download(d)
            d.free()
        assert same_bits(out, co.power(g, host, nthreads=16))


def test_full_config3_pinned_host_vs_c_oracle(gpu):
    """BASELINE configs[2]: 1024 ch x 2 pol int8 (4 GiB per integration) from
    a registered (pinned) host buffer, H2D overlapped with the kernel through
    the staging pair, pushed in three ragged frame-whole pieces; then the
    same context integrates the next block from the device (the fused
    path), so host and device spans share one context"""
    g = npo.Geom(nbit=8, nchan_chunk=1024)
    with paf_b2p.Integrator(to_b2p(g)) as it:
        d = it.alloc(g.block_bytes)
        it.fill_synthetic(d, SEED, 3, 0)
        host = it.download(d)
        it.register_host(host)
        try:
            cuts = [0, 777 * g.frame_bytes, g.block_bytes - 5 * g.frame_bytes, g.block_bytes]
            for a, b in zip(cuts, cuts[1:]):
                it.push(host[a:b])
            out = it.finish()
        finally:
            it.unregister_host(host)
        it.fill_synthetic(d, SEED, 3, 1)
        nxt = it.integrate(d)
        host2 = it.download(d)
        d.free()
    assert same_bits(out, co.power(g, host, nthreads=16))
    assert same_bits(nxt, co.power(g, host2, nthreads=16))


def test_full_bmf_block_vs_c_oracle(gpu):
    # reference-native: 8192 DF x 48 chunks x 7168 B = 2818572288 B
    g = npo.BMF
    with paf_b2p.Integrator(paf_b2p.bmf_geom()) as it:
        d = it.alloc(g.block_bytes)
        it.fill_synthetic(d, SEED, 0, 1)
        it.push(d)
        out = it.finish()
        host = it.download(d)
        d.free()
    assert out.shape == (336,)
    assert same_bits(out, co.power(g, host, nthreads=16))


def test_full_tftfp_8x8_block_vs_c_oracle(gpu):
    """int16 BE TFTFP, 8 chunks x 8 channels, a full 2^20-sample integration
    (512 MiB): the power-of-two frame runs as 8 columns of 512 threads"""
    g = npo.Geom(nbit=16, big_endian=1, nchunk=8, nsamp_df=128, nchan_chunk=8)
    with paf_b2p.Integrator(to_b2p(g)) as it:
        assert (it.info.threads, it.info.columns) == (512, 8)
        d = it.alloc(g.block_bytes)
        it.fill_synthetic(d, SEED, 2, 3)
        out = it.integrate(d)
        host = it.download(d)
        d.free()
    assert same_bits(out, co.power(g, host, nthreads=16))


def test_full_1024ch_int16_8gib_vs_c_oracle(gpu):
    # configs 3/5 at int16 = 8 GiB per integration (more than
    # 2^32 bytes and 2^29 16-B vectors in one launch), X and Y kept apart
    g = npo.Geom(nbit=16, nchan_chunk=1024, npol_out=2)
    assert g.block_bytes == 8 << 30
    with paf_b2p.Integrator(to_b2p(g)) as it:
        d = it.alloc(g.block_bytes)
        it.fill_synthetic(d, SEED, 6, 0)
        it.push(d)
        out = it.finish()
        host = it.download(d)
        d.free()
    assert out.shape == (2048,)
    assert same_bits(out, co.power(g, host, nthreads=16))
    del host


def test_full_1024ch_properties(gpu):
    # configs 3/5 layout at full size: push order / chunking invariance and
    # run-to-run determinism (exact integer sums), plus two back-to-back
    # integrations on one context
    g = paf_b2p.generic_geom(1024)
    bb = paf_b2p.block_bytes(g)
    with paf_b2p.Integrator(g) as it:
        d = it.alloc(bb)
        it.fill_synthetic(d, SEED, 4, 0)
        it.push(d)
        whole = it.finish()
        half = bb // 2
        it.push((d, half, bb - half))
        it.push((d, 0, half))
        rev = it.finish()
        it.push(d)
        again = it.finish()
        sample = it.download(d, nbytes=64 << 20)
        d.free()
    assert same_bits(whole, rev) and same_bits(whole, again)
    # the first 64 MiB alone, against the oracle
    gs = npo.Geom(nbit=8, nchan_chunk=1024, nsamp_int=(64 << 20) // 4096)
    with paf_b2p.Integrator(to_b2p(gs)) as it2:
        dd = it2.upload(sample)
        it2.push(dd)
        part = it2.finish()
        dd.free()
    assert same_bits(part, co.power(gs, sample, nthreads=16))


def test_error_codes(gpu):
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=64)
    with paf_b2p.Integrator(to_b2p(g)) as it:
        d = it.alloc(g.block_bytes + 64)
        with pytest.raises(paf_b2p.B2PError) as e:
            it.push((d, 0, g.frame_bytes + 16))
        assert e.value.code == L.B2P_ERAGGED
        with pytest.raises(paf_b2p.B2PError) as e:
            it.push((d, 0, g.block_bytes + g.frame_bytes))
        assert e.value.code == L.B2P_EOVERFLOW
        with pytest.raises(paf_b2p.B2PError) as e:
            it.push((d, 8, g.frame_bytes))
        assert e.value.code == L.B2P_EALIGN
        it.push((d, 0, 0))  # empty span: no-op
        assert it.samples_pending() == 0
        it.fill_synthetic(d, SEED, 0, 0, nbytes=g.block_bytes)
        it.push((d, 0, g.frame_bytes * 10))
        assert it.samples_pending() == 10
        with pytest.raises(paf_b2p.B2PError) as e:
            it.finish()
        assert e.value.code == L.B2P_EPARTIAL
        # partial result is still emitted, and the context is reset
        it.push((d, 0, g.frame_bytes * 10))
        part = it.finish(allow_partial=True)
        buf = it.download(d, nbytes=g.frame_bytes * 10)
        gp = npo.Geom(**{**g.asdict(), "nsamp_int": 10})
        assert same_bits(part, npo.power(gp, buf))
        assert it.samples_pending() == 0
        d.free()


def test_empty_integration_is_zero(gpu):
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=64)
    with paf_b2p.Integrator(to_b2p(g)) as it:
        out = it.finish(allow_partial=True)
    assert np.all(out == 0)


def test_device_index_fallback(gpu):
    # paf_baseband2power.cu:89-90: with one visible device any index maps to 0
    if paf_b2p.device_count() != 1:
        pytest.skip("more than one device visible")
    with paf_b2p.Integrator(paf_b2p.generic_geom(256), device=5) as it:
        assert it.info.device == 0


@pytest.mark.parametrize("name", sorted(GEOMS))
@pytest.mark.parametrize("npol_out,mean", [(1, 0), (2, 1)])
def test_integrate_fused_equals_push_finish(gpu, name, npol_out, mean):
    # b2p_integrate: one launch, last workgroup finalizes; three back-to-back
    # integrations on one context (the arrival ticket must re-arm) and both
    # row mappings
    g = npo.Geom(**{**GEOMS[name].asdict(), "npol_out": npol_out, "mean": mean})
    bufs = [npo.fill_synthetic(g, g.block_bytes, SEED, 2, k) for k in range(3)]
    for inter in (0, 1):
        with paf_b2p.Integrator(to_b2p(g), tuning={"interleave": inter}) as it:
            for b in bufs:
                d = it.upload(b)
                fused = it.integrate(d)
                it.push(d)
                pf = it.finish()
                d.free()
                assert same_bits(fused, pf)
                assert same_bits(fused, npo.power(g, b))


def test_integrate_host_span_and_errors(gpu):
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=4096)
    buf = co.fill_synthetic(g, g.block_bytes, SEED, 0, 0)
    with paf_b2p.Integrator(to_b2p(g)) as it:
        assert same_bits(it.integrate(buf), co.power(g, buf))   # host span
        d = it.upload(buf)
        with pytest.raises(paf_b2p.B2PError) as e:
            it.integrate((d, 0, g.block_bytes - g.frame_bytes))
        assert e.value.code == L.B2P_EINVAL
        it.push((d, 0, g.frame_bytes))
        with pytest.raises(paf_b2p.B2PError):
            it.integrate(d)                                      # a push is pending
        it.finish(allow_partial=True)
        assert same_bits(it.integrate(d), co.power(g, buf))
        d.free()


def test_full_size_fused_vs_oracle(gpu):
    # configs[1] and the BMF block through the one-launch path
    for g, pg in ((npo.Geom(nbit=8, nchan_chunk=256), paf_b2p.generic_geom(256)),
                  (npo.BMF, paf_b2p.bmf_geom())):
        with paf_b2p.Integrator(pg) as it:
            d = it.alloc(g.block_bytes)
            it.fill_synthetic(d, SEED, 7, 7)
            out = it.integrate(d)
            host = it.download(d)
            d.free()
        assert same_bits(out, co.power(g, host, nthreads=16))


def test_timing_modes(gpu):
    g = paf_b2p.generic_geom(256)
    with paf_b2p.Integrator(g) as it:
        d = it.alloc(it.block_bytes)
        it.fill_synthetic(d, SEED, 0, 0)
        it.set_timing(1)
        for _ in range(3):
            it.push(d)
            it.finish()
        s1 = it.stats()
        assert s1["launches"] == 3 and s1["finalizes"] == 3 and s1["bytes"] == 3 * it.block_bytes
        per = s1["kernel_ms"] / 3
        assert 0.05 < per < 5.0  # ms; 1 GiB at 0.2-20 TB/s
        it.set_timing(0)
        it.reset_stats()
        it.set_timing(2)
        for _ in range(4):
            it.integrate(d, None)
        it.set_timing(0)
        s2 = it.stats()
        assert s2["launches"] == 4 and s2["finalizes"] in (0, 4)  # fused or not (tuning.fuse)
        assert s2["kernel_ms"] / 4 > 0.5 * per
        d.free()


def test_integrate_device_span_is_one_launch(gpu):
    # a device span must be read in place: one integrate launch (+ finalize),
    # no staging copies
    g = paf_b2p.generic_geom(256)
    with paf_b2p.Integrator(g) as it:
        d = it.alloc(it.block_bytes)
        it.fill_synthetic(d, SEED, 0, 0)
        it.set_timing(1)
        it.integrate(d)
        s = it.stats()
        assert s["launches"] == 1 and s["bytes"] == it.block_bytes
        d.free()


@pytest.mark.parametrize("fuse", [0, 1])
def test_back_to_back_async_integrations(gpu, fuse):
    # 7 integrations enqueued without a host sync: the two replica sets
    # alternate and every finalize overlaps the next integrate (or runs in
    # the last workgroup with tuning fuse=1); each spectrum must be exact
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=1 << 16)
    with paf_b2p.Integrator(to_b2p(g), tuning={"fuse": fuse}) as it:
        blocks = []
        for k in range(3):
            d = it.alloc(g.block_bytes)
            it.fill_synthetic(d, SEED, 9, k)
            blocks.append(d)
        out = it.alloc(7 * g.nout * 4)
        for k in range(7):
            it.integrate(blocks[k % 3], out.ptr + k * g.nout * 4, True)
        it.sync()
        got = it.download(out).view(np.float32).reshape(7, g.nout).copy()
        # the push / finish_async form, also unsynchronised
        for k in range(7):
            it.push(blocks[k % 3])
            it.finish_async(out.ptr + k * g.nout * 4, True)
        it.sync()
        got2 = it.download(out).view(np.float32).reshape(7, g.nout)
        assert same_bits(got, got2)
        hosts = [it.download(b) for b in blocks]
        for b in blocks:
            b.free()
        out.free()
    for k in range(7):
        assert same_bits(got[k], co.power(g, hosts[k % 3])), k


def test_push_failure_part_way_marks_context_failed(gpu):
    """A host-span push that fails after its first staging chunk was summed
    leaves the integration unknown: the call reports the failure and every
    later call on the context returns B2P_EFAILED until b2p_close (the
    reference would have exit(-1)ed, cudautil.cuh:29-41).  The failure is
    injected at staging chunk 2 of a 4-chunk span by the TEST build of the
    library (lib/hooks/libpafb2p.so, -DB2P_TEST_HOOKS), loaded in a child
    process; the release library has no injection entry at all."""
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "tests", "hooks_push_fail.py")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "push-fail hook: ok" in r.stdout


def test_fused_host_output_after_finish_async_host(gpu):
    """tuning fuse=1: a fused integrate whose spectrum goes to the host follows
    a finish_async to the host; the carried finalize of the first and the
    fused finalize of the second must not share the staging output"""
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=8192)
    bufs = [co.fill_synthetic(g, g.block_bytes, SEED, 5, k) for k in range(3)]
    with paf_b2p.Integrator(to_b2p(g), tuning={"fuse": 1}) as it:
        ds = [it.upload(b) for b in bufs]
        outs = [np.zeros(g.nout, np.float32) for _ in range(3)]
        it.push(ds[0])
        it.finish_async(outs[0].ctypes.data, False)
        it.integrate(ds[1], outs[1].ctypes.data, False)
        it.integrate(ds[2], outs[2].ctypes.data, False)
        it.sync()
        for d in ds:
            d.free()
    for b, o in zip(bufs, outs):
        assert same_bits(o, co.power(g, b))
