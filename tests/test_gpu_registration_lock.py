"""b2p_unregister_host drains its context's streams before it takes the
process-wide registration lock (advisor, round 5): while one context waits
for ~100 ms of queued launches to finish, another context's registration
call is answered at once instead of queueing behind that drain.

The probe call needs no HIP work: registering a range that shares pages with
a live registration is refused under the lock (B2P_EINVAL) before any HIP
call, so its latency is the lock's wait and nothing else."""
import threading
import time

import numpy as np
import pytest

import paf_b2p
from paf_b2p import _lib as L

pytestmark = pytest.mark.gpu


def test_unregister_drain_does_not_hold_the_registration_lock(gpu):
    a = paf_b2p.Integrator(nbit=8, nchan_chunk=256, nsamp_int=1 << 20)  # configs[1]: 1 GiB per integration
    b = paf_b2p.Integrator(nbit=8, nchan_chunk=256, nsamp_int=1 << 20)
    host = np.zeros(1 << 20, dtype=np.uint8)
    blk = a.alloc(a.block_bytes)
    out = a.alloc(a.nout * 4)
    try:
        a.fill_synthetic(blk, 20181105, 0, 0)
        a.sync()
        a.register_host(host)
        for _ in range(640):  # ~96 ms of integrate launches queued on a's stream
            a.integrate(blk, out.ptr, True)
        t_drain, t_probe, errs = [], [], []

        def drain():
            t0 = time.perf_counter()
            a.unregister_host(host)  # waits for a's stream first
            t_drain.append(time.perf_counter() - t0)

        def probe():
            time.sleep(0.01)  # a is inside its drain by now
            t0 = time.perf_counter()
            try:
                b.register_host(host)  # shares pages with a's live registration: refused
            except L.B2PError as e:
                errs.append((e.code, str(e)))
            t_probe.append(time.perf_counter() - t0)
        th = [threading.Thread(target=drain), threading.Thread(target=probe)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        a.sync()
    finally:
        out.free()
        blk.free()
        a.close()
        b.close()
    assert t_drain and t_probe, (t_drain, t_probe)
    assert t_drain[0] > 0.04, t_drain  # the drain really waited for the queued launches
    assert errs and errs[0][0] == L.B2P_EINVAL and "shares pages" in errs[0][1], errs  # refused under the lock
    assert t_probe[0] < 0.25 * t_drain[0], (t_probe, t_drain)  # not queued behind the drain
