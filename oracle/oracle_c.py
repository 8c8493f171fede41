"""oracle/oracle_c.py -- TEST INFRASTRUCTURE ONLY.

ctypes binding of the C restatement (oracle/b2p_oracle.c) for tests/,
``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from b2p_oracle import Geom  # noqa: E402  (oracle/ is put on sys.path by callers)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "liboracle_b2p.so")
_REF_HDR = os.path.join(_HERE, "_ref", "libhdr_ref.so")


class OrcGeom(C.Structure):
    _fields_ = [("nbit", C.c_uint32), ("big_endian", C.c_uint32), ("nchunk", C.c_uint32),
                ("nsamp_df", C.c_uint32), ("nchan_chunk", C.c_uint32), ("npol", C.c_uint32),
                ("ndim", C.c_uint32), ("npol_out", C.c_uint32), ("nsamp_int", C.c_uint64),
                ("mean", C.c_uint32), ("reserved", C.c_uint32)]

    @classmethod
    def of(cls, g: Geom) -> "OrcGeom":
        return cls(g.nbit, g.big_endian, g.nchunk, g.nsamp_df, g.nchan_chunk, g.npol, g.ndim,
                   g.npol_out, g.nsamp_int, g.mean, 0)


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.orc_integrate.argtypes = [C.POINTER(OrcGeom), P, C.c_size_t, P]
        L.orc_integrate_mt.argtypes = [C.POINTER(OrcGeom), P, C.c_size_t, P, C.c_int]
        L.orc_finalize.argtypes = [C.POINTER(OrcGeom), P, P]
        L.orc_fill_synthetic.argtypes = [C.POINTER(OrcGeom), P, C.c_size_t, C.c_uint64,
                                         C.c_uint32, C.c_uint64, C.c_uint64]
        L.orc_bmf_lanes.argtypes = [P, P]
        L.orc_splitmix64.argtypes = [C.c_uint64]
        L.orc_splitmix64.restype = C.c_uint64
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def integrate(g: Geom, buf: np.ndarray, nthreads: int = 1, acc: np.ndarray | None = None) -> np.ndarray:
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    if acc is None:
        acc = np.zeros(g.nout, dtype=np.uint64)
    og = OrcGeom.of(g)
    if nthreads > 1:
        rc = lib().orc_integrate_mt(C.byref(og), _ptr(buf), buf.size, _ptr(acc), nthreads)
    else:
        rc = lib().orc_integrate(C.byref(og), _ptr(buf), buf.size, _ptr(acc))
    if rc != 0:
        raise ValueError("oracle rejected input (ragged or unsupported geometry)")
    return acc


def finalize(g: Geom, acc: np.ndarray) -> np.ndarray:
    acc = np.ascontiguousarray(acc, dtype=np.uint64)
    out = np.zeros(g.nout, dtype=np.float32)
    lib().orc_finalize(C.byref(OrcGeom.of(g)), _ptr(acc), _ptr(out))
    return out


def power(g: Geom, buf: np.ndarray, nthreads: int = 1) -> np.ndarray:
    return finalize(g, integrate(g, buf, nthreads))


def fill_synthetic(g: Geom, nbytes: int, seed: int, subband: int, block: int,
                   elem0: int = 0, out: np.ndarray | None = None) -> np.ndarray:
    if out is None:
        out = np.empty(nbytes, dtype=np.uint8)
    lib().orc_fill_synthetic(C.byref(OrcGeom.of(g)), _ptr(out), nbytes, seed, subband, block, elem0)
    return out


def bmf_lanes(word: bytes) -> np.ndarray:
    w = np.frombuffer(word, dtype=np.uint8).copy()
    lanes = np.zeros(4, dtype=np.int16)
    lib().orc_bmf_lanes(_ptr(w), _ptr(lanes))
    return lanes


class HdrT(C.Structure):
    """struct hdr_t of the reference (hdr.h:6-14)."""
    _fields_ = [("valid", C.c_int), ("idf", C.c_uint64), ("sec", C.c_uint64),
                ("epoch", C.c_int), ("beam", C.c_int), ("freq", C.c_double)]


def ref_hdr_lib():
    """The reference's own hdr.c built by `make -C oracle ref` (None if absent)."""
    if not os.path.exists(_REF_HDR):
        return None
    L = C.CDLL(_REF_HDR)
    L.hdr_keys.argtypes = [C.c_void_p, C.POINTER(HdrT)]
    L.hdr_keys.restype = C.c_int
    return L


def assemble(dfs: np.ndarray, chunk_of_df: np.ndarray, ref_idf: int, ref_sec: int,
             block: np.ndarray, block_ndf: int, nchunk: int, counts: np.ndarray | None = None):
    """orc_assemble (capture.c:527-547 placement) into `block` in place."""
    L = lib()
    L.orc_assemble.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_uint64,
                               C.c_uint64, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]
    dfs = np.ascontiguousarray(dfs, dtype=np.uint8)
    chunk_of_df = np.ascontiguousarray(chunk_of_df, dtype=np.uint8)
    if counts is None:
        counts = np.zeros(nchunk + 3, dtype=np.uint64)
    ndf = dfs.size // 7232
    L.orc_assemble(_ptr(dfs), ndf, 7232, _ptr(chunk_of_df), ref_idf, ref_sec, _ptr(block),
                   block_ndf, nchunk, _ptr(counts))
    return counts


# ---- the tuned CPU port (oracle/b2p_cpu_port.c): bench.py's cpu_baseline --
_PORT_PATH = os.path.join(_HERE, "lib", "libb2p_cpuport.so")
ISA = {"auto": 0, "scalar": 1, "avx2": 2, "avx512bw": 3, "avx512vnni": 4}
_port = None


def port_lib():
    global _port
    if _port is None:
        if not os.path.exists(_PORT_PATH):
            build()
        L = C.CDLL(_PORT_PATH)
        L.cpp_integrate.argtypes = [C.POINTER(OrcGeom), C.c_void_p, C.c_size_t, C.c_void_p, C.c_int,
                                    C.c_int]
        L.cpp_isa_name.argtypes = [C.c_int]
        L.cpp_isa_name.restype = C.c_char_p
        _port = L
    return _port


def port_isa(isa: str = "auto") -> str:
    """the ISA the port runs for a request ("auto": the best this CPU has)"""
    return port_lib().cpp_isa_name(ISA[isa]).decode()


def port_integrate(g: Geom, buf: np.ndarray, nthreads: int = 1, acc: np.ndarray | None = None,
                   isa: str = "auto") -> np.ndarray:
    """exact uint64 sums from the tuned port (equal to integrate())"""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    if acc is None:
        acc = np.zeros(g.nout, dtype=np.uint64)
    rc = port_lib().cpp_integrate(C.byref(OrcGeom.of(g)), _ptr(buf), buf.size, _ptr(acc),
                                  nthreads, ISA[isa])
    if rc != 0:
        raise ValueError("cpu port rejected input (ragged or unsupported geometry)")
    return acc
