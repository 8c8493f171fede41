"""ctypes binding of include/b2p.h (lib/libpafb2p.so).

The product path is the HIP library; this module only marshals arguments.
If the library is missing or fails to load, every call raises -- there is no
CPU fallback (the CPU restatement lives in oracle/ and is test-only).

One HIP runtime per process: torch (when installed) ships its own
libamdhip64 with the same SONAME, so torch is imported BEFORE the library is
loaded; the dynamic loader then binds libpafb2p.so to that one runtime
instead of mapping a second copy.
"""
from __future__ import annotations

import ctypes as C
import os

try:  # see module docstring: load order decides which HIP runtime is shared
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C-ABI path
    torch = None

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libpafb2p.so")

B2P_OK = 0
B2P_EINVAL = -1
B2P_ERAGGED = -2
B2P_EOVERFLOW = -3
B2P_EPARTIAL = -4
B2P_ENODEV = -5
B2P_EHIP = -6
B2P_ENOMEM = -7
B2P_EALIGN = -8
B2P_EFAILED = -9
B2P_ETIMEDOUT = -10
ABI_VERSION = 2


class B2PError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"b2p error {code}: {msg}")
        self.code = code


class Geom(C.Structure):
    """b2p_geom_t (include/b2p.h)."""
    _fields_ = [("nbit", C.c_uint32), ("big_endian", C.c_uint32), ("nchunk", C.c_uint32),
                ("nsamp_df", C.c_uint32), ("nchan_chunk", C.c_uint32), ("npol", C.c_uint32),
                ("ndim", C.c_uint32), ("npol_out", C.c_uint32), ("nsamp_int", C.c_uint64),
                ("mean", C.c_uint32), ("reserved", C.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class Info(C.Structure):
    _fields_ = [("nchan", C.c_uint32), ("nout", C.c_uint32), ("frame_bytes", C.c_uint64),
                ("block_bytes", C.c_uint64), ("threads", C.c_uint32), ("columns", C.c_uint32),
                ("row_groups", C.c_uint32), ("row_vectors", C.c_uint32), ("replicas", C.c_uint32),
                ("device", C.c_uint32), ("unroll", C.c_uint32), ("nontemporal", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("launches", C.c_uint64), ("bytes", C.c_uint64), ("kernel_ms", C.c_double),
                ("finalize_ms", C.c_double), ("finalizes", C.c_uint64)]


class Tuning(C.Structure):
    """b2p_tuning_t (include/b2p.h): an explicit launch variant for tuning
    sweeps; 0 / -1 fields keep the measured defaults."""
    _fields_ = [("size", C.c_uint32), ("max_threads", C.c_int32), ("threads", C.c_int32),
                ("wg_per_cu", C.c_int32), ("row_groups", C.c_int32), ("replicas", C.c_int32),
                ("unroll", C.c_int32), ("nontemporal", C.c_int32), ("interleave", C.c_int32),
                ("fuse", C.c_int32), ("stage_mib", C.c_int32), ("assemble_grid", C.c_int32)]

    @classmethod
    def make(cls, **kw) -> "Tuning":
        t = cls()
        lib().b2p_tuning_init(C.byref(t))
        for k, v in kw.items():
            if k not in dict(cls._fields_) or k == "size":
                raise KeyError(f"no tuning field {k!r}")
            setattr(t, k, int(v))
        return t


# name -> (restype, argtypes); must match include/b2p.h exactly
_P = C.c_void_p
PROTOTYPES = {
    "b2p_abi_version": (C.c_int, []),
    "b2p_strerror": (C.c_char_p, [C.c_int]),
    "b2p_last_error": (C.c_char_p, [_P]),
    "b2p_geom_bmf": (C.c_int, [C.POINTER(Geom)]),
    "b2p_geom_check": (C.c_int, [C.POINTER(Geom)]),
    "b2p_frame_bytes": (C.c_uint64, [C.POINTER(Geom)]),
    "b2p_block_bytes": (C.c_uint64, [C.POINTER(Geom)]),
    "b2p_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "b2p_open": (C.c_int, [C.POINTER(_P), C.POINTER(Geom), C.c_int]),
    "b2p_open_tuned": (C.c_int, [C.POINTER(_P), C.POINTER(Geom), C.c_int, C.POINTER(Tuning)]),
    "b2p_tuning_init": (None, [C.POINTER(Tuning)]),
    "b2p_device_pci_bus_id": (C.c_int, [C.c_int, C.c_char_p, C.c_int]),
    "b2p_close": (C.c_int, [_P]),
    "b2p_get_info": (C.c_int, [_P, C.POINTER(Info)]),
    "b2p_set_stream": (C.c_int, [_P, _P]),
    "b2p_register_host": (C.c_int, [_P, _P, C.c_size_t]),
    "b2p_unregister_host": (C.c_int, [_P, _P]),
    "b2p_push": (C.c_int, [_P, _P, C.c_size_t, C.c_int]),
    "b2p_finish": (C.c_int, [_P, _P]),
    "b2p_finish_async": (C.c_int, [_P, _P, C.c_int]),
    "b2p_sync": (C.c_int, [_P]),
    "b2p_integrate": (C.c_int, [_P, _P, C.c_size_t, C.c_int, _P, C.c_int]),
    "b2p_integrate_n": (C.c_int, [_P, C.POINTER(_P), C.c_uint32, _P, C.c_int]),
    "b2p_blocks_per_launch": (C.c_uint32, [C.c_uint64]),
    "b2p_samples_pending": (C.c_uint64, [_P]),
    "b2p_set_timing": (C.c_int, [_P, C.c_int]),
    "b2p_get_stats": (C.c_int, [_P, C.POINTER(Stats)]),
    "b2p_reset_stats": (C.c_int, [_P]),
    "b2p_fill_synthetic": (C.c_int, [_P, _P, C.c_size_t, C.c_uint64, C.c_uint32, C.c_uint64,
                                     C.c_uint64]),
    "b2p_dev_alloc": (C.c_int, [_P, C.POINTER(_P), C.c_size_t]),
    "b2p_assemble": (C.c_int, [_P, _P, C.c_uint64, C.c_uint32, _P, C.c_uint64, C.c_uint64, _P,
                               C.c_uint64, C.c_uint32, _P]),
    "b2p_dev_free": (C.c_int, [_P, _P]),
    "b2p_memcpy": (C.c_int, [_P, _P, _P, C.c_size_t, C.c_int]),
    "b2p_memset": (C.c_int, [_P, _P, C.c_int, C.c_size_t]),
    "b2p_finish_partial_async": (C.c_int, [_P, _P, C.c_int]),
    "b2p_fence": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "b2p_fence_wait": (C.c_int, [_P, C.c_uint64]),
    "b2p_fence_done": (C.c_int, [_P, C.c_uint64]),
    "b2p_flush": (C.c_int, [_P]),
    "b2p_finalize_sums": (C.c_int, [_P, _P, C.c_uint64, C.c_uint64, _P]),
    "b2p_group_reduce": (C.c_int, [_P, _P, C.c_uint64, _P]),
    "b2p_group_open": (C.c_int, [C.POINTER(_P), C.POINTER(_P), C.c_int, C.c_int]),
    "b2p_group_open_timed": (C.c_int, [C.POINTER(_P), C.POINTER(_P), C.c_int, C.c_int, C.c_int]),
    "b2p_group_gather": (C.c_int, [_P, C.POINTER(_P), _P]),
    "b2p_group_gather_n": (C.c_int, [_P, C.POINTER(_P), C.c_uint32, _P]),
    "b2p_group_gather_async": (C.c_int, [_P, C.POINTER(_P), C.c_uint32, _P, C.POINTER(C.c_uint64), _P,
                                         C.POINTER(C.c_uint64)]),
    "b2p_group_wait": (C.c_int, [_P, C.c_uint64]),
    "b2p_group_done": (C.c_int, [_P, C.c_uint64]),
    "b2p_group_sync": (C.c_int, [_P]),
    "b2p_group_last_error": (C.c_char_p, [_P]),
    "b2p_group_close": (C.c_int, [_P]),
}

# the test builds' extra entries (lib/hooks/libpafb2p.so, -DB2P_TEST_HOOKS;
# lib/debug/libpafb2p.so, -DB2P_DEBUG -DB2P_TEST_HOOKS)
HOOK_PROTOTYPES = {"b2p_test_inject_push_fail": (C.c_int, [_P, C.c_long]),
                   "b2p_test_debug_shrink_bound": (C.c_int, [_P, C.c_long]),
                   "b2p_debug_build": (C.c_int, [])}

_lib = None


def lib() -> C.CDLL:
    """Load libpafb2p.so; raise loudly if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                              "or `make -C paf-baseband2power_amd` (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        for name, (res, args) in HOOK_PROTOTYPES.items():
            f = getattr(L, name, None)
            if f is not None:
                f.restype = res
                f.argtypes = args
        if L.b2p_abi_version() != ABI_VERSION:
            raise ImportError("libpafb2p ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, ctx=None, allow=()) -> int:
    if rc == B2P_OK or rc in allow:
        return rc
    L = lib()
    detail = L.b2p_last_error(ctx).decode(errors="replace")
    raise B2PError(rc, f"{L.b2p_strerror(rc).decode()}: {detail}")
