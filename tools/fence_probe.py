"""How much host-side waiting costs between back-to-back integrations (BMF
blocks, HBM-resident): no wait, b2p_fence_wait on the previous launch, or a
full b2p_sync per block; spectra to pinned host or device memory."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "paf-baseband2power_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import paf_b2p  # noqa: E402

it = paf_b2p.Integrator(paf_b2p.bmf_geom())
blocks = [it.alloc(it.block_bytes) for _ in range(2)]
for b, d in enumerate(blocks):
    it.fill_synthetic(d, 20181105, 0, b)
host = np.zeros((3, it.nout), np.float32)
it.register_host(host)
dev = it.alloc(3 * it.nout * 4)
K = 100
for mode in ("none", "fence_prev", "sync_each"):
    for out in ("host", "device"):
        it.sync()
        t = [0, 0]
        t0 = time.perf_counter()
        for k in range(K):
            if out == "host":
                it.integrate(blocks[k % 2], host[k % 3].ctypes.data, False)
            else:
                it.integrate(blocks[k % 2], dev.ptr + (k % 3) * it.nout * 4, True)
            if mode == "fence_prev":
                t[k & 1] = it.fence()
                if k:
                    it.fence_wait(t[(k - 1) & 1])
            elif mode == "sync_each":
                it.sync()
        it.sync()
        el = time.perf_counter() - t0
        print(json.dumps({"wait": mode, "out": out, "ms_per_block": round(el / K * 1e3, 4)}), flush=True)
it.unregister_host(host)
