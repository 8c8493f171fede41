"""Python host-side mirror of the integrator's C ABI (include/b2p.h).

``Integrator`` is the per-sub-band object the reference intended to build in
baseband2power.cu (empty, baseband2power.cu:1-16) around conf_t
(baseband2power.cuh:18-23): open on a device, push ring blocks, emit one
power spectrum per 1024x1024-sample integration (README.md:2).  Every call
goes through libpafb2p.so; errors raise ``B2PError`` with the library's
status code (the reference printed and called exit(-1), cudautil.cuh:29-41).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .geometry import make_geom


@dataclass
class DeviceBuffer:
    """Device memory owned by an Integrator (hipMalloc through the C ABI)."""
    ptr: int
    nbytes: int
    owner: "Integrator"

    def free(self) -> None:
        if self.ptr:
            L.check(L.lib().b2p_dev_free(self.owner._ctx, C.c_void_p(self.ptr)), self.owner._ctx)
            self.ptr = 0


class Integrator:
    def __init__(self, geom=None, device: int = 0, tuning: dict | None = None, **geom_kw):
        """tuning: b2p_tuning_t fields (tools/tune.py); None = the measured
        defaults (b2p_open)"""
        g = geom if isinstance(geom, L.Geom) else make_geom(**(geom or {}), **geom_kw)
        self.geom = g
        self._ctx = C.c_void_p()
        self._registered: dict[int, np.ndarray] = {}  # base -> the array, kept alive while registered
        lib = L.lib()
        if tuning:
            t = L.Tuning.make(**tuning)
            L.check(lib.b2p_open_tuned(C.byref(self._ctx), C.byref(g), device, C.byref(t)), None)
        else:
            L.check(lib.b2p_open(C.byref(self._ctx), C.byref(g), device), None)
        info = L.Info()
        L.check(lib.b2p_get_info(self._ctx, C.byref(info)), self._ctx)
        self.info = info
        self.nout = info.nout
        self.frame_bytes = info.frame_bytes
        self.block_bytes = info.block_bytes

    # ---- lifecycle ---------------------------------------------------------
    def close(self) -> None:
        if self._ctx:
            L.check(L.lib().b2p_close(self._ctx))  # also releases what it registered
            self._ctx = C.c_void_p()
        self._registered.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- hot path ------------------------------------------------------------
    def push(self, buf, nbytes: int | None = None, is_device: bool | None = None) -> None:
        """Accumulate a whole number of frames.  ``buf``: numpy uint8 array
        (host), ``DeviceBuffer`` / ``(DeviceBuffer, offset, nbytes)`` /
        ``(device pointer, nbytes)`` (device), or a raw pointer int with
        ``nbytes`` and ``is_device``."""
        ptr, n, dev = self._span(buf, nbytes, is_device)
        L.check(L.lib().b2p_push(self._ctx, C.c_void_p(ptr), n, int(dev)), self._ctx)

    def finish(self, allow_partial: bool = False) -> np.ndarray:
        out = np.zeros(self.nout, dtype=np.float32)
        rc = L.lib().b2p_finish(self._ctx, out.ctypes.data_as(C.c_void_p))
        L.check(rc, self._ctx, allow=(L.B2P_EPARTIAL,) if allow_partial else ())
        return out

    def finish_partial(self, out_ptr: int | None = None, out_is_device: bool = False,
                       allow_partial: bool = False):
        """b2p_finish_partial_async: the integration's exact uint64 sums (a
        member's share of a time-split integration).  With out_ptr None the
        sums are returned (blocking)."""
        if out_ptr is None:
            out = np.zeros(self.nout, dtype=np.uint64)
            rc = L.lib().b2p_finish_partial_async(self._ctx, out.ctypes.data_as(C.c_void_p), 0)
            L.check(rc, self._ctx, allow=(L.B2P_EPARTIAL,) if allow_partial else ())
            self.sync()
            return out
        rc = L.lib().b2p_finish_partial_async(self._ctx, C.c_void_p(out_ptr), int(out_is_device))
        return L.check(rc, self._ctx, allow=(L.B2P_EPARTIAL,) if allow_partial else ())

    def finalize_sums(self, sums_ptr: int, nspec: int, out_ptr: int, nsamp_total: int = 0) -> None:
        """b2p_finalize_sums: fp32 (one RNE rounding) from nspec x nout exact
        sums in device memory, stream-ordered."""
        L.check(L.lib().b2p_finalize_sums(self._ctx, C.c_void_p(sums_ptr), nspec, nsamp_total,
                                          C.c_void_p(out_ptr)), self._ctx)

    def fence(self) -> int:
        """b2p_fence: ticket for everything enqueued so far"""
        t = C.c_uint64()
        L.check(L.lib().b2p_fence(self._ctx, C.byref(t)), self._ctx)
        return t.value

    def fence_wait(self, ticket: int) -> None:
        L.check(L.lib().b2p_fence_wait(self._ctx, ticket), self._ctx)

    def finish_async(self, out_ptr: int, out_is_device: bool) -> int:
        rc = L.lib().b2p_finish_async(self._ctx, C.c_void_p(out_ptr), int(out_is_device))
        return L.check(rc, self._ctx, allow=(L.B2P_EPARTIAL,))

    def integrate(self, buf, out_ptr: int | None = None, out_is_device: bool = False):
        """One whole integration in one call (fused finalize for device spans).
        With out_ptr None the spectrum is returned (blocking)."""
        ptr, n, dev = self._span(buf, None, None)
        if out_ptr is None:
            out = np.zeros(self.nout, dtype=np.float32)
            L.check(L.lib().b2p_integrate(self._ctx, C.c_void_p(ptr), n, int(dev),
                                          out.ctypes.data_as(C.c_void_p), 0), self._ctx)
            self.sync()
            return out
        L.check(L.lib().b2p_integrate(self._ctx, C.c_void_p(ptr), n, int(dev), C.c_void_p(out_ptr),
                                      int(out_is_device)), self._ctx)
        return None

    def integrate_n(self, bufs, out_ptr: int | None = None, out_is_device: bool = False):
        """b2p_integrate_n: len(bufs) whole integrations (device buffers) in ONE
        launch.  With out_ptr None the spectra are returned (blocking)."""
        ptrs = [self._span(b, None, None)[0] for b in bufs]
        arr = (C.c_void_p * len(ptrs))(*ptrs)
        if out_ptr is None:
            out = np.zeros((len(ptrs), self.nout), dtype=np.float32)
            L.check(L.lib().b2p_integrate_n(self._ctx, arr, len(ptrs), out.ctypes.data_as(C.c_void_p), 0),
                    self._ctx)
            self.sync()
            return out
        L.check(L.lib().b2p_integrate_n(self._ctx, arr, len(ptrs), C.c_void_p(out_ptr), int(out_is_device)),
                self._ctx)
        return None

    def sync(self) -> None:
        L.check(L.lib().b2p_sync(self._ctx), self._ctx)

    def samples_pending(self) -> int:
        return int(L.lib().b2p_samples_pending(self._ctx))

    def set_stream(self, hip_stream: int | None) -> None:
        L.check(L.lib().b2p_set_stream(self._ctx, C.c_void_p(hip_stream or 0)), self._ctx)

    # ---- host memory -----------------------------------------------------------
    def register_host(self, arr: np.ndarray) -> None:
        """Pin ``arr`` for full-rate copies (b2p_register_host).  The array is
        kept alive until unregister_host or close: memory must never be
        freed while it is registered, or HIP would go on copying from the
        stale pinned pages of its address."""
        L.check(L.lib().b2p_register_host(self._ctx, C.c_void_p(arr.ctypes.data), arr.nbytes),
                self._ctx)
        self._registered[arr.ctypes.data] = arr

    def unregister_host(self, arr: np.ndarray) -> None:
        L.check(L.lib().b2p_unregister_host(self._ctx, C.c_void_p(arr.ctypes.data)), self._ctx)
        self._registered.pop(arr.ctypes.data, None)

    # ---- device buffers / synthetic data ----------------------------------------
    def alloc(self, nbytes: int) -> DeviceBuffer:
        p = C.c_void_p()
        L.check(L.lib().b2p_dev_alloc(self._ctx, C.byref(p), nbytes), self._ctx)
        return DeviceBuffer(p.value or 0, nbytes, self)

    def upload(self, arr: np.ndarray) -> DeviceBuffer:
        arr = np.ascontiguousarray(arr)
        d = self.alloc(max(arr.nbytes, 16))
        if arr.nbytes:
            L.check(L.lib().b2p_memcpy(self._ctx, C.c_void_p(d.ptr), C.c_void_p(arr.ctypes.data),
                                       arr.nbytes, 1), self._ctx)
        d.nbytes = arr.nbytes
        return d

    def upload_into(self, d: DeviceBuffer, arr: np.ndarray, offset: int = 0) -> None:
        """arr (host) -> d + offset, synchronous (b2p_memcpy: hipMemcpy)"""
        if arr.nbytes:
            L.check(L.lib().b2p_memcpy(self._ctx, C.c_void_p(d.ptr + offset), C.c_void_p(arr.ctypes.data),
                                       arr.nbytes, 1), self._ctx)

    def download(self, d: DeviceBuffer, nbytes: int | None = None, offset: int = 0) -> np.ndarray:
        n = d.nbytes - offset if nbytes is None else nbytes
        out = np.empty(n, dtype=np.uint8)
        if n:
            L.check(L.lib().b2p_memcpy(self._ctx, C.c_void_p(out.ctypes.data),
                                       C.c_void_p(d.ptr + offset), n, 2), self._ctx)
        return out

    def fill_synthetic(self, d: DeviceBuffer, seed: int, subband: int, block: int,
                       nbytes: int | None = None, offset: int = 0, elem0: int = 0) -> None:
        n = d.nbytes - offset if nbytes is None else nbytes
        L.check(L.lib().b2p_fill_synthetic(self._ctx, C.c_void_p(d.ptr + offset), n, seed, subband,
                                           block, elem0), self._ctx)

    def assemble(self, dfs: DeviceBuffer, ndf: int, chunk_of_df: DeviceBuffer, ref_idf: int,
                 ref_sec: int, block: DeviceBuffer, block_ndf: int, nchunk: int,
                 counts: DeviceBuffer) -> None:
        """b2p_assemble: scatter raw 7232-B data frames into a TFTFP block."""
        L.check(L.lib().b2p_assemble(self._ctx, C.c_void_p(dfs.ptr), ndf, 7232,
                                     C.c_void_p(chunk_of_df.ptr), ref_idf, ref_sec,
                                     C.c_void_p(block.ptr), block_ndf, nchunk,
                                     C.c_void_p(counts.ptr)), self._ctx)

    # ---- measurement -------------------------------------------------------------
    def set_timing(self, mode: int | bool) -> None:
        """0 off, 1 per-launch events, 2 one event pair around a region."""
        L.check(L.lib().b2p_set_timing(self._ctx, int(mode)), self._ctx)

    def stats(self) -> dict:
        s = L.Stats()
        L.check(L.lib().b2p_get_stats(self._ctx, C.byref(s)), self._ctx)
        return {"launches": s.launches, "bytes": s.bytes, "kernel_ms": s.kernel_ms,
                "finalize_ms": s.finalize_ms, "finalizes": s.finalizes}

    def reset_stats(self) -> None:
        L.check(L.lib().b2p_reset_stats(self._ctx), self._ctx)

    # ---- helpers -------------------------------------------------------------------
    def _span(self, buf, nbytes, is_device):
        if isinstance(buf, DeviceBuffer):
            return buf.ptr, buf.nbytes if nbytes is None else nbytes, True
        if isinstance(buf, tuple) and len(buf) == 2 and isinstance(buf[0], int):
            return buf[0], buf[1], True  # (device pointer, nbytes), e.g. a torch tensor's
        if isinstance(buf, tuple):
            d, off, n = buf
            return d.ptr + off, n, True
        if isinstance(buf, np.ndarray):
            if not buf.flags.c_contiguous:
                raise ValueError("host span must be contiguous")
            return buf.ctypes.data, buf.nbytes if nbytes is None else nbytes, False
        if isinstance(buf, int):
            if nbytes is None or is_device is None:
                raise ValueError("raw pointer needs nbytes and is_device")
            return buf, nbytes, is_device
        raise TypeError(f"unsupported span type {type(buf)}")


def device_count() -> int:
    n = C.c_int(0)
    rc = L.lib().b2p_device_count(C.byref(n))
    return n.value if rc == L.B2P_OK else 0


def pci_bus_id(device: int) -> str:
    """b2p_device_pci_bus_id: the physical GPU behind a device index"""
    buf = C.create_string_buffer(32)
    L.check(L.lib().b2p_device_pci_bus_id(device, buf, 32))
    return buf.value.decode()


class Group:
    """b2p_group: gather the spectra of N Integrators (one per GPU /
    sub-band) to the first one's device -- RCCL (mode 0) or peer copies
    (mode 1, members sharing a device)."""

    def __init__(self, members: list[Integrator], mode: int = 0, timeout_ms: int = 60000):
        self.members = members
        arr = (C.c_void_p * len(members))(*[m._ctx.value for m in members])
        self._g = C.c_void_p()
        rc = L.lib().b2p_group_open_timed(C.byref(self._g), arr, len(members), mode, timeout_ms)
        if rc != L.B2P_OK:
            raise L.B2PError(rc, L.lib().b2p_group_last_error(None).decode(errors="replace"))

    def gather(self, spectra_ptrs: list[int], root_out_ptr: int) -> None:
        arr = (C.c_void_p * len(spectra_ptrs))(*spectra_ptrs)
        rc = L.lib().b2p_group_gather(self._g, arr, C.c_void_p(root_out_ptr))
        if rc != L.B2P_OK:
            raise L.B2PError(rc, L.lib().b2p_group_last_error(self._g).decode(errors="replace"))
        self.sync()

    def gather_async(self, spectra_ptrs: list[int], nspec: int, root_out_ptr: int, tickets: list[int],
                     host_out_ptr: int | None = None) -> int:
        """b2p_group_gather_async: nspec spectra per member, read once member
        r's fence ticket tickets[r] has passed, on the group's own streams;
        returns the ticket for wait()"""
        arr = (C.c_void_p * len(spectra_ptrs))(*spectra_ptrs)
        tk = (C.c_uint64 * len(tickets))(*tickets)
        gt = C.c_uint64()
        rc = L.lib().b2p_group_gather_async(self._g, arr, nspec, C.c_void_p(root_out_ptr), tk,
                                            C.c_void_p(host_out_ptr) if host_out_ptr else None, C.byref(gt))
        if rc != L.B2P_OK:
            raise L.B2PError(rc, L.lib().b2p_group_last_error(self._g).decode(errors="replace"))
        return gt.value

    def wait(self, gticket: int) -> None:
        rc = L.lib().b2p_group_wait(self._g, gticket)
        if rc != L.B2P_OK:
            raise L.B2PError(rc, L.lib().b2p_group_last_error(self._g).decode(errors="replace"))

    def sync(self) -> None:
        rc = L.lib().b2p_group_sync(self._g)
        if rc != L.B2P_OK:
            raise L.B2PError(rc, L.lib().b2p_group_last_error(self._g).decode(errors="replace"))

    def reduce(self, sums_ptrs: list[int], count: int, root_sum_ptr: int) -> None:
        """b2p_group_reduce: exact uint64 sum of every member's partial sums
        (time-split mode) into root_sum on the first member's device."""
        arr = (C.c_void_p * len(sums_ptrs))(*sums_ptrs)
        rc = L.lib().b2p_group_reduce(self._g, arr, count, C.c_void_p(root_sum_ptr))
        if rc != L.B2P_OK:
            raise L.B2PError(rc, L.lib().b2p_group_last_error(self._g).decode(errors="replace"))
        self.sync()

    def close(self) -> None:
        if self._g:
            L.lib().b2p_group_close(self._g)
            self._g = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
