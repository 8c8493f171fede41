"""Child process of test_push_failure_part_way_marks_context_failed (GPU).

Loads the TEST build of the library (lib/hooks/libpafb2p.so, compiled with
-DB2P_TEST_HOOKS) instead of the release one, then injects a failure at
staging chunk 2 of a 4-chunk host span through b2p_test_inject_push_fail.
Kept out of the pytest process so that process only ever maps the release
library.  Prints "push-fail hook: ok" on success; any failed check raises.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "paf-baseband2power_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process)

from paf_b2p import _lib as L  # noqa: E402

L.LIB_PATH = os.path.join(L.PKG_DIR, "lib", "hooks", "libpafb2p.so")

import b2p_oracle as npo  # noqa: E402
import oracle_c as co  # noqa: E402
import paf_b2p  # noqa: E402


def main():
    lib = L.lib()
    assert hasattr(lib, "b2p_test_inject_push_fail"), "not the test build"
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=4096)      # 4 MiB per integration
    buf = co.fill_synthetic(g, g.block_bytes, 20181105, 0, 0)
    pg = paf_b2p.make_geom(**g.asdict())
    it = paf_b2p.Integrator(pg, tuning={"stage_mib": 1})       # 4 staging chunks
    assert lib.b2p_test_inject_push_fail(it._ctx, 2) == 0
    try:
        it.push(buf)
        raise AssertionError("injected failure did not surface")
    except paf_b2p.B2PError as e:
        assert e.code == L.B2P_EHIP and "injected" in str(e), e
    for call in (lambda: it.push(buf), lambda: it.finish(allow_partial=True), it.sync,
                 lambda: it.set_timing(2), it.fence):
        try:
            call()
            raise AssertionError("call on a failed context succeeded")
        except paf_b2p.B2PError as e:
            assert e.code == L.B2P_EFAILED, e
    assert "injected" in lib.b2p_last_error(it._ctx).decode()   # the first failure's text
    it.close()
    with paf_b2p.Integrator(pg, tuning={"stage_mib": 1}) as it2:   # a fresh context is fine
        it2.push(buf)
        out = it2.finish()
    want = co.power(g, buf)
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))
    print("push-fail hook: ok", flush=True)


if __name__ == "__main__":
    main()
