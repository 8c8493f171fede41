"""Child process of the debug-build GPU tests (tests/test_gpu_random_layouts.py).

Loads the DEBUG build of the library (lib/debug/libpafb2p.so: -DB2P_DEBUG
-DB2P_TEST_HOOKS) instead of the release one.  In it every span load of the
integrate kernel is checked against its span and every output slot against
nout -- an out-of-bounds access is recorded, not made, and fails the next
sync with its index, workgroup and lane -- and push_host checks every
staging chunk against the staging size, the span and its host
registration.  Kept out of the pytest process, which only maps the release
library.

  python3 tests/debug_build_checks.py checks          the detector and the lifetime rules
  python3 tests/debug_build_checks.py staging N [SEED] the host-staging property, N examples

Prints "debug build checks: ok" / "staging under debug build: N examples ok";
any failed check raises (exit 1).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "paf-baseband2power_amd"), os.path.join(REPO, "oracle"), HERE]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process)

from paf_b2p import _lib as L  # noqa: E402

L.LIB_PATH = os.path.join(L.PKG_DIR, "lib", "debug", "libpafb2p.so")

import b2p_oracle as npo  # noqa: E402
import oracle_c as co  # noqa: E402
import paf_b2p  # noqa: E402
import staging_case  # noqa: E402

# one layout per launch-shape branch of plan_shape (b2p_plan.h)
SHAPES = [
    dict(nbit=8, nchan_chunk=256, nsamp_int=1 << 14),                      # one-column int8 row
    dict(nbit=8, nchan_chunk=336, nsamp_int=1 << 13),                      # period split into columns
    dict(nbit=16, big_endian=1, nchunk=48, nchan_chunk=7, nsamp_df=128, nsamp_int=1 << 10),  # BMF frame split
    dict(nbit=16, nchunk=8, nchan_chunk=8, nsamp_df=64, nsamp_int=1 << 10),  # power-of-two frame, 512 columns
    dict(nbit=8, nchunk=61, nchan_chunk=44, nsamp_df=1, nsamp_int=333),    # no whole-wave divisor
]


def same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def checks():
    lib = L.lib()
    assert hasattr(lib, "b2p_debug_build") and lib.b2p_debug_build() == 1, "not the debug build"
    # 1. clean runs report nothing: device spans cut at odd frames, every branch
    for kw in SHAPES:
        g = npo.Geom(**kw)
        buf = co.fill_synthetic(g, g.block_bytes, 20181105, 1, 0)
        with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict())) as it:
            d = it.upload(buf)
            nf = g.block_bytes // g.frame_bytes
            cut = max(1, nf // 3) * g.frame_bytes if nf > 1 else g.block_bytes
            it.push((d, 0, cut))
            if cut < g.block_bytes:
                it.push((d, cut, g.block_bytes - cut))
            out = it.finish()
            d.free()
        assert same(out, co.power(g, buf, nthreads=8)), kw
    # 2. a lowered load bound: the detector names the first offending load
    g = npo.Geom(**SHAPES[0])
    buf = co.fill_synthetic(g, g.block_bytes, 7, 0, 0)
    it = paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict()))
    d = it.upload(buf)
    assert lib.b2p_test_debug_shrink_bound(it._ctx, 64) == 0
    it.push(d)
    try:
        it.finish()
        raise AssertionError("lowered bound not reported")
    except paf_b2p.B2PError as e:
        msg = str(e)
        assert e.code == L.B2P_EHIP and "B2P_DEBUG" in msg and "out-of-bounds span loads" in msg, msg
        nvec = g.block_bytes // 16
        assert f"of {nvec - 64}," in msg, msg              # the bound it was checked against
        first = int(msg.split("first: index ")[1].split()[0])
        assert nvec - 64 <= first < nvec, msg               # an index in the cut-off tail
    try:
        it.sync()
        raise AssertionError("context not failed")
    except paf_b2p.B2PError as e:
        assert e.code == L.B2P_EFAILED, e
    d.free()
    it.close()
    # 3. a push from registered memory that fails part-way, then unregister and
    #    free at once: b2p_push drained the copies of the span before it
    #    returned, so nothing reads the freed pages (repeated; a copy left in
    #    flight would fault the GPU, and every later call would fail)
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=4096)   # 4 MiB, 4 staging chunks of 1 MiB
    pg = paf_b2p.make_geom(**g.asdict())
    for rep in range(8):
        host = co.fill_synthetic(g, g.block_bytes, 11, 0, rep)
        it = paf_b2p.Integrator(pg, tuning={"stage_mib": 1})
        it.register_host(host)
        assert lib.b2p_test_inject_push_fail(it._ctx, 1 + rep % 3) == 0
        try:
            it.push(host)
            raise AssertionError("injected failure did not surface")
        except paf_b2p.B2PError as e:
            assert "injected" in str(e), e
        it.unregister_host(host)   # must succeed on a failed context (cleanup)
        del host                   # freed now
        it.close()
    # 4. close releases what its context registered and the caller left:
    #    the same array registers again in a fresh context (HIP would refuse
    #    a range that is still registered)
    host = co.fill_synthetic(g, g.block_bytes, 12, 0, 0)
    it = paf_b2p.Integrator(pg)
    it.register_host(host)
    it.close()
    with paf_b2p.Integrator(pg, tuning={"stage_mib": 1}) as it2:
        it2.register_host(host)
        try:
            it3 = paf_b2p.Integrator(pg)
            try:  # an overlapping registration is refused up front
                it3.register_host(host[4096:])
                raise AssertionError("overlapping registration accepted")
            except paf_b2p.B2PError as e:
                assert e.code == L.B2P_EINVAL and "shares pages" in str(e), e
            it3.close()
            it2.push(host)
            out = it2.finish()
        finally:
            it2.unregister_host(host)
    assert same(out, co.power(g, host, nthreads=8))
    print("debug build checks: ok", flush=True)


def staging(n, seed):
    from hypothesis import HealthCheck, given, settings
    from hypothesis import seed as hseed
    from hypothesis import strategies as st

    done = []

    @hseed(seed)
    @settings(max_examples=n, deadline=None, database=None,
              suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
    @given(st.sampled_from(staging_case.LAYOUTS), st.integers(1, 3), st.integers(2, 24),
           st.lists(st.floats(0.0, 1.0), max_size=4), st.booleans(), st.integers(0, 2 ** 31))
    def prop(layout, stage_mib, mib, cut_fracs, register, s):
        staging_case.run_case(layout, stage_mib, mib, cut_fracs, register, s)
        done.append(1)

    assert L.lib().b2p_debug_build() == 1, "not the debug build"
    prop()
    print(f"staging under debug build: {len(done)} examples ok", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "checks":
        checks()
    else:
        staging(int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 5005)
