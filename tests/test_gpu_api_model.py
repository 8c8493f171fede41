"""Model-based test of the integrator's C ABI (include/b2p.h) on the GPU.

A hypothesis state machine drives one context through random sequences of
the calls a consumer makes -- b2p_push of device or host spans of whole
frames, b2p_finish (blocking), b2p_finish_async and b2p_finish_partial_async
into device slots, b2p_integrate and b2p_integrate_n into device slots,
b2p_flush, b2p_fence / b2p_fence_wait, b2p_sync -- with slots reused before
a sync, pushes while an output is still pending, and calls that must be
refused (b2p_integrate with a push pending, pushes past the integration).
Host memory lifetime (round 5): the input blocks and a host output array
are registered and unregistered at random; a second registration of a
range is refused; b2p_finish_async lands spectra in the registered host
output, and unregistering it while they may still be landing must drain
them first; b2p_close releases what the context left registered (the same
memory registers again in a fresh context at teardown).
A NumPy model keeps the exact uint64 sums of the frames pushed (the C
oracle's integrate over each span) and what every slot must hold after
b2p_sync; every check compares bit for bit.  The geometry and the launch
variant (finalize carried by the next launch, or fused into the last
workgroup, tuning.fuse) are drawn per run.

B2P_HYPOTHESIS_SCALE scales the run; B2P_HYPOTHESIS_SEED (any value) draws a
fresh random set instead of the fixed one."""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, settings
from hypothesis import strategies as st
from hypothesis.stateful import RuleBasedStateMachine, initialize, invariant, precondition, rule

import b2p_oracle as npo
import oracle_c as co
import paf_b2p
from paf_b2p import _lib as L

pytestmark = pytest.mark.gpu
_SCALE = int(os.environ.get("B2P_HYPOTHESIS_SCALE", "1"))
_SEED = os.environ.get("B2P_HYPOTHESIS_SEED")
NBLK, NSLOT = 3, 6
CALLS = {}  # rule -> times run (printed by the test: the machine really ran)

LAYOUTS = [dict(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=64),
           dict(nbit=16, big_endian=1, nchunk=4, nsamp_df=128, nchan_chunk=7),
           dict(nbit=16, nchunk=2, nsamp_df=2, nchan_chunk=12),
           dict(nbit=8, nchunk=3, nsamp_df=4, nchan_chunk=5)]


class ApiModel(RuleBasedStateMachine):
    @initialize(layout=st.sampled_from(LAYOUTS), nframes=st.integers(2, 12), npol_out=st.sampled_from([1, 2]),
                mean=st.booleans(), fuse=st.sampled_from([-1, 1]), seed=st.integers(0, 2 ** 31))
    def setup(self, layout, nframes, npol_out, mean, fuse, seed):
        self.g = npo.Geom(**layout, npol_out=npol_out, mean=int(mean), nsamp_int=nframes * layout["nsamp_df"])
        self.nframes = nframes
        self.it = paf_b2p.Integrator(paf_b2p.make_geom(**self.g.asdict()), tuning={"fuse": fuse})
        fb = self.g.frame_bytes
        # page-aligned, page-padded host arrays (a page is pinned by one
        # registration only): the blocks, then a host output array
        pg = 4096
        span = (self.g.block_bytes + pg - 1) // pg * pg
        hspan = (NSLOT * self.g.nout * 4 + pg - 1) // pg * pg
        self._hmem = np.zeros(NBLK * span + hspan + pg, np.uint8)
        a0 = (-self._hmem.ctypes.data) % pg
        self.host = []
        for b in range(NBLK):
            v = self._hmem[a0 + b * span: a0 + b * span + self.g.block_bytes]
            co.fill_synthetic(self.g, self.g.block_bytes, seed, 1, b, out=v)
            self.host.append(v)
        self.hout = self._hmem[a0 + NBLK * span: a0 + NBLK * span + NSLOT * self.g.nout * 4].view(np.float32)
        self.registered = set()            # host blocks registered (index), "out" for the output
        self.want_host = {}                # host slot -> expected fp32 bits (after sync)
        self.it.register_host(self.hout)   # the host output starts registered (finish_async_host)
        self.registered.add("out")
        self.dev = [self.it.upload(h) for h in self.host]
        # per block, exact sums of each frame (the model adds them up)
        g1 = npo.Geom(**{**self.g.asdict(), "nsamp_int": layout["nsamp_df"]})
        self.fsum = [[self._sums(g1, h[f * fb:(f + 1) * fb]) for f in range(nframes)] for h in self.host]
        self.bsum = [np.sum(np.stack(s), axis=0, dtype=np.uint64) for s in self.fsum]
        self.out = self.it.alloc(NSLOT * self.g.nout * 4)
        self.raw = self.it.alloc(NSLOT * self.g.nout * 8)
        self.acc = np.zeros(self.g.nout, np.uint64)
        self.pend = 0                      # frames in the running integration
        self.want = {}                     # slot -> expected fp32 bits (after sync)
        self.want_raw = {}                 # slot -> expected uint64 sums
        self.log = [f"setup {layout} nframes={nframes} npol_out={npol_out} mean={mean} fuse={fuse}"]

    @staticmethod
    def _sums(g, span):
        acc = np.zeros(g.nout, np.uint64)
        co.integrate(g, span, nthreads=1, acc=acc)
        return acc

    def _spectrum(self, acc):
        return co.finalize(self.g, acc).view(np.uint32)

    def teardown(self):
        if hasattr(self, "it"):
            try:
                self.check()
            finally:
                for d in self.dev + [self.out, self.raw]:
                    d.free()
                self.it.close()   # releases what is still registered
            if self.registered:   # ... so the same memory registers again
                with paf_b2p.Integrator(paf_b2p.make_geom(**self.g.asdict())) as it2:
                    for r in self.registered:
                        arr = self.hout if r == "out" else self.host[r]
                        it2.register_host(arr)
                        it2.unregister_host(arr)

    # ---- host memory ----------------------------------------------------------
    @rule(r=st.sampled_from([0, 1, 2, "out"]))
    def register(self, r):
        CALLS["register"] = CALLS.get("register", 0) + 1
        self.log.append(f"register {r}")
        arr = self.hout if r == "out" else self.host[r]
        if r in self.registered:   # a second registration of the range is refused
            with pytest.raises(L.B2PError) as e:
                self.it.register_host(arr)
            assert e.value.code == L.B2P_EINVAL
            return
        self.it.register_host(arr)
        self.registered.add(r)

    @precondition(lambda self: bool(self.registered))
    @rule(data=st.data())
    def unregister(self, data):
        CALLS["unregister"] = CALLS.get("unregister", 0) + 1
        r = data.draw(st.sampled_from(sorted(self.registered, key=str)))
        self.log.append(f"unregister {r}")
        # the output may still be landing (finish_async_host): unregister drains it
        self.it.unregister_host(self.hout if r == "out" else self.host[r])
        self.registered.discard(r)
        if r == "out":   # every spectrum enqueued into it has landed
            got = self.hout.view(np.uint32).reshape(NSLOT, self.g.nout)
            for s_, w in self.want_host.items():
                assert np.array_equal(got[s_], w), ("host slot after unregister", s_, "\n".join(self.log[-60:]))

    @precondition(lambda self: "out" in self.registered)
    @rule(slot=st.integers(0, NSLOT - 1))
    def finish_async_host(self, slot):
        CALLS["finish_async_host"] = CALLS.get("finish_async_host", 0) + 1
        self.log.append(f"finish_async_host slot={slot}")
        rc = self.it.finish_async(self.hout.ctypes.data + slot * self.g.nout * 4, False)
        assert rc == (L.B2P_OK if self.pend == self.nframes else L.B2P_EPARTIAL)
        self.want_host[slot] = self._spectrum(self.acc)
        self._reset()

    # ---- pushes ---------------------------------------------------------------
    @rule(data=st.data())
    def push_device(self, data):
        CALLS["push_device"] = CALLS.get("push_device", 0) + 1
        self.log.append("push_device " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        b = data.draw(st.integers(0, NBLK - 1))
        f0 = data.draw(st.integers(0, self.nframes - 1))
        n = data.draw(st.integers(1, self.nframes - f0))
        self.log.append(f"  push_device b={b} f0={f0} n={n} pend={self.pend}")
        fb = self.g.frame_bytes
        if self.pend + n > self.nframes:   # past the integration: refused, nothing changes
            with pytest.raises(L.B2PError) as e:
                self.it.push((self.dev[b], f0 * fb, n * fb))
            assert e.value.code == L.B2P_EOVERFLOW
            return
        self.it.push((self.dev[b], f0 * fb, n * fb))
        self.acc += np.sum(np.stack(self.fsum[b][f0:f0 + n]), axis=0, dtype=np.uint64)
        self.pend += n

    @rule(data=st.data())
    def push_host(self, data):
        CALLS["push_host"] = CALLS.get("push_host", 0) + 1
        self.log.append("push_host " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        b = data.draw(st.integers(0, NBLK - 1))
        f0 = data.draw(st.integers(0, self.nframes - 1))
        n = data.draw(st.integers(1, min(self.nframes - f0, self.nframes - self.pend) or 1))
        self.log.append(f"  push_host b={b} f0={f0} n={n} pend={self.pend}")
        if self.pend + n > self.nframes:
            return
        fb = self.g.frame_bytes
        self.it.push(np.ascontiguousarray(self.host[b][f0 * fb:(f0 + n) * fb]))
        self.acc += np.sum(np.stack(self.fsum[b][f0:f0 + n]), axis=0, dtype=np.uint64)
        self.pend += n

    # ---- outputs --------------------------------------------------------------
    def _reset(self):
        self.acc = np.zeros(self.g.nout, np.uint64)
        self.pend = 0

    @rule()
    def finish_blocking(self):
        CALLS["finish_blocking"] = CALLS.get("finish_blocking", 0) + 1
        self.log.append("finish_blocking " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        out = self.it.finish(allow_partial=True)
        assert np.array_equal(out.view(np.uint32), self._spectrum(self.acc))
        self._reset()

    @rule(slot=st.integers(0, NSLOT - 1))
    def finish_async(self, slot):
        CALLS["finish_async"] = CALLS.get("finish_async", 0) + 1
        self.log.append("finish_async " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        rc = self.it.finish_async(self.out.ptr + slot * self.g.nout * 4, True)
        assert rc == (L.B2P_OK if self.pend == self.nframes else L.B2P_EPARTIAL)
        self.want[slot] = self._spectrum(self.acc)
        self._reset()

    @rule(slot=st.integers(0, NSLOT - 1))
    def finish_partial(self, slot):
        CALLS["finish_partial"] = CALLS.get("finish_partial", 0) + 1
        self.log.append("finish_partial " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        self.it.finish_partial(self.raw.ptr + slot * self.g.nout * 8, True, allow_partial=True)
        self.want_raw[slot] = self.acc.copy()
        self._reset()

    @rule(b=st.integers(0, NBLK - 1), slot=st.integers(0, NSLOT - 1))
    def integrate(self, b, slot):
        CALLS["integrate"] = CALLS.get("integrate", 0) + 1
        self.log.append("integrate " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        dst = self.out.ptr + slot * self.g.nout * 4
        if self.pend:
            with pytest.raises(L.B2PError) as e:
                self.it.integrate(self.dev[b], dst, True)
            assert e.value.code == L.B2P_EINVAL
            return
        self.it.integrate(self.dev[b], dst, True)
        self.want[slot] = self._spectrum(self.bsum[b])

    @rule(data=st.data())
    def integrate_n(self, data):
        CALLS["integrate_n"] = CALLS.get("integrate_n", 0) + 1
        self.log.append("integrate_n " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        k = data.draw(st.integers(1, NSLOT))
        slot0 = data.draw(st.integers(0, NSLOT - k))
        bs = data.draw(st.lists(st.integers(0, NBLK - 1), min_size=k, max_size=k))
        self.log.append(f"  integrate_n slot0={slot0} blocks={bs} pend={self.pend}")
        dst = self.out.ptr + slot0 * self.g.nout * 4
        if self.pend:
            with pytest.raises(L.B2PError):
                self.it.integrate_n([self.dev[b] for b in bs], dst, True)
            return
        self.it.integrate_n([self.dev[b] for b in bs], dst, True)
        for j, b in enumerate(bs):
            self.want[slot0 + j] = self._spectrum(self.bsum[b])

    @rule()
    def flush(self):
        CALLS["flush"] = CALLS.get("flush", 0) + 1
        self.log.append("flush " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        L.check(L.lib().b2p_flush(self.it._ctx), self.it._ctx)

    @rule()
    def fence(self):
        CALLS["fence"] = CALLS.get("fence", 0) + 1
        self.log.append("fence " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        self.it.fence_wait(self.it.fence())

    @precondition(lambda self: bool(self.want or self.want_raw or self.want_host))
    @rule()
    def check(self):
        CALLS["check"] = CALLS.get("check", 0) + 1
        self.log.append("check " + repr({k: v for k, v in locals().items() if k not in ("self", "data")}))
        self.it.sync()
        got = self.it.download(self.out).view(np.uint32).reshape(NSLOT, self.g.nout)
        for s, w in self.want.items():
            assert np.array_equal(got[s], w), ("slot", s, "\n".join(self.log[-60:]))
        raw = self.it.download(self.raw).view(np.uint64).reshape(NSLOT, self.g.nout)
        for s, w in self.want_raw.items():
            assert np.array_equal(raw[s], w), ("raw slot", s, "\n".join(self.log[-60:]))
        hgot = self.hout.view(np.uint32).reshape(NSLOT, self.g.nout)
        for s, w in self.want_host.items():
            assert np.array_equal(hgot[s], w), ("host slot", s, "\n".join(self.log[-60:]))

    @invariant()
    def pending_matches(self):
        if hasattr(self, "it"):
            assert self.it.samples_pending() == self.pend * self.g.nsamp_df


def test_api_model(gpu):
    from hypothesis.stateful import run_state_machine_as_test
    run_state_machine_as_test(ApiModel, settings=settings(
        max_examples=25 * _SCALE, stateful_step_count=30, deadline=None,
        derandomize=_SEED is None,  # B2P_HYPOTHESIS_SEED: a fresh random set instead
        suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large]))
    print("api model calls:", dict(sorted(CALLS.items())))
    assert CALLS.get("check", 0) >= 10 and CALLS.get("integrate_n", 0) >= 10
    assert CALLS.get("finish_async_host", 0) >= 5 and CALLS.get("unregister", 0) >= 3
