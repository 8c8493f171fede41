#!/usr/bin/env python3
"""How long does one context's registration call wait while another context
unregisters a range and drains ~100 ms of queued launches?  (The advisor's
round-5 finding: b2p_unregister_host held the process-wide registration lock
across that drain.)  The probe registers a range that shares pages with the
live registration: the library refuses it under the lock before any HIP
call, so its latency is the lock's wait alone.

  python3 tools/reglock_probe.py [--lib path/to/libpafb2p.so] [--runs 5]

One JSON line: the library, its code objects' sha256, per run the drain's and
the probe's seconds and whether the probe was refused (a probe that waited
out the drain finds the range released, and is accepted).
tests/test_gpu_registration_lock.py asserts the product library's
behaviour; this tool also runs an older build beside it.
"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "paf-baseband2power_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib")
    ap.add_argument("--runs", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    from paf_b2p import _lib as L
    if a.lib:
        L.LIB_PATH = os.path.abspath(a.lib)
    import bench
    import paf_b2p
    runs = []
    ia = paf_b2p.Integrator(nbit=8, nchan_chunk=256, nsamp_int=1 << 20)
    ib = paf_b2p.Integrator(nbit=8, nchan_chunk=256, nsamp_int=1 << 20)
    blk, out = ia.alloc(ia.block_bytes), ia.alloc(ia.nout * 4)
    ia.fill_synthetic(blk, 20181105, 0, 0)
    ia.sync()
    host = np.zeros(1 << 20, dtype=np.uint8)
    for _ in range(a.runs):
        ia.register_host(host)
        for _ in range(640):
            ia.integrate(blk, out.ptr, True)
        res = {}

        def drain():
            t0 = time.perf_counter()
            ia.unregister_host(host)
            res["drain_s"] = round(time.perf_counter() - t0, 5)

        def probe():
            time.sleep(0.01)
            t0 = time.perf_counter()
            try:
                ib.register_host(host)  # answered only after the drain released the range: accepted
                res["refused"] = False
            except L.B2PError as e:
                res["refused"] = e.code == L.B2P_EINVAL
            res["probe_s"] = round(time.perf_counter() - t0, 5)
            if not res["refused"]:
                ib.unregister_host(host)
        th = [threading.Thread(target=drain), threading.Thread(target=probe)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        ia.sync()
        runs.append(res)
    out.free()
    blk.free()
    ia.close()
    ib.close()
    print(json.dumps({"lib": os.path.relpath(L.LIB_PATH, REPO), "device_code_sha256": bench.device_code_sha(L.LIB_PATH),
                      "runs": runs}), flush=True)


if __name__ == "__main__":
    main()
