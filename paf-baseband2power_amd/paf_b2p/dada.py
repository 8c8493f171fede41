"""ctypes binding of include/b2p_dada.h (lib/libpafdada.so): DADA ASCII
headers and SysV ring buffers, used by the launcher and the tests.

Mirrors the PSRDADA calls the reference makes (diskdb.cu:24-130,
capture.c:590-781) plus the reader half.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import PKG_DIR

DADA_LIB = os.path.join(PKG_DIR, "lib", "libpafdada.so")
BIN_DIR = os.path.join(PKG_DIR, "bin")
HDR_SIZE = 4096

_dl = None


def dlib():
    global _dl
    if _dl is None:
        if not os.path.exists(DADA_LIB):
            raise ImportError(f"{DADA_LIB} not built (make -C paf-baseband2power_amd)")
        L = C.CDLL(DADA_LIB, use_errno=True)
        P = C.c_void_p
        L.ascii_header_get.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, P]
        L.ascii_header_set.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p]
        L.ascii_header_del.argtypes = [C.c_char_p, C.c_char_p]
        L.dada_db_create.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint, C.c_uint64, C.c_uint64]
        L.dada_db_destroy.argtypes = [C.c_int]
        L.dada_hdu_create.restype = P
        L.dada_hdu_create.argtypes = [P]
        L.dada_hdu_set_key.argtypes = [P, C.c_int]
        for n in ("dada_hdu_connect", "dada_hdu_disconnect", "dada_hdu_lock_write",
                  "dada_hdu_unlock_write", "dada_hdu_lock_read", "dada_hdu_unlock_read",
                  "dada_hdu_open_read", "dada_hdu_open_view", "dada_hdu_close_view"):
            getattr(L, n).argtypes = [P]
        L.dada_hdu_destroy.argtypes = [P]
        L.dada_hdu_destroy.restype = None
        L.ipcio_open_block_write.restype = P
        L.ipcio_open_block_write.argtypes = [P, C.POINTER(C.c_uint64)]
        L.ipcio_close_block_write.argtypes = [P, C.c_uint64]
        L.ipcio_open_block_read.restype = P
        L.ipcio_open_block_read.argtypes = [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.ipcio_close_block_read.argtypes = [P, C.c_uint64]
        L.ipcio_close_block_read.restype = C.c_ssize_t
        L.ipcbuf_get_next_write.restype = P
        L.ipcbuf_get_next_write.argtypes = [P]
        L.ipcbuf_mark_filled.argtypes = [P, C.c_uint64]
        L.ipcbuf_get_bufsz.restype = C.c_uint64
        L.ipcbuf_get_bufsz.argtypes = [P]
        L.ipcbuf_get_nbufs.restype = C.c_uint64
        L.ipcbuf_get_nbufs.argtypes = [P]
        L.ipcbuf_eod.argtypes = [P]
        L.ipcbuf_enable_eod.argtypes = [P]
        L.ipcbuf_get_write_count.restype = C.c_uint64
        L.ipcbuf_get_read_count.restype = C.c_uint64
        L.ipcbuf_get_read_count.argtypes = [P]
        L.ipcbuf_get_write_count.argtypes = [P]
        L.ipcbuf_get_device.argtypes = [P]
        L.ipcbuf_set_read_depth.argtypes = [P, C.c_int]
        L.ipcbuf_copy_in.argtypes = [P, P, P, C.c_uint64]
        L.dada_device_error.restype = C.c_char_p
        L.dada_device_error.argtypes = []
        L.ipcbuf_copy_out.argtypes = [P, P, P, C.c_uint64]
        for n in ("ipcbuf_get_nfull", "ipcbuf_get_nclear", "ipcbuf_get_sodack", "ipcbuf_get_eodack"):
            getattr(L, n).restype = C.c_uint64
            getattr(L, n).argtypes = [P]
            getattr(L, n + "_iread").restype = C.c_uint64
            getattr(L, n + "_iread").argtypes = [P, C.c_int]
        L.ipcbuf_get_reader_conn_iread.argtypes = [P, C.c_int]
        L.ipcbuf_get_read_semaphore_count.argtypes = [P]
        L.ipcio_read.restype = C.c_ssize_t
        L.ipcio_read.argtypes = [P, P, C.c_size_t]
        L.ipcio_write.restype = C.c_ssize_t
        L.ipcio_write.argtypes = [P, P, C.c_size_t]
        L.dada_db_create_work.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint, C.c_uint64,
                                          C.c_uint64, C.c_int]
        L.dada_device_ring_info.argtypes = [C.c_int, C.POINTER(DeviceInfo)]
        _dl = L
    return _dl


class DeviceInfo(C.Structure):
    """dada_device_info_t (include/b2p_dada.h)"""
    _fields_ = [(n, C.c_int) for n in ("device", "holder_pid", "holder_state", "importers", "export_retries",
                                        "primer_refused")]


class HduStruct(C.Structure):
    """struct dada_hdu (include/b2p_dada.h)"""
    _fields_ = [("log", C.c_void_p), ("data_block", C.c_void_p), ("header_block", C.c_void_p),
                ("header", C.c_void_p), ("header_size", C.c_uint64), ("data_block_key", C.c_int),
                ("header_block_key", C.c_int)]


# ---- ASCII header -------------------------------------------------------------

def header_get(header: bytes | str, key: str, fmt: str = "%1023s"):
    """Value of `key` (string by default), or None when absent."""
    h = header.encode() if isinstance(header, str) else header
    if fmt in ("%d", "%i"):
        v = C.c_int()
    elif fmt in ("%lf", "%f"):
        v, fmt = C.c_double(), "%lf"
    elif fmt in ("%lu", "%llu", "%" "lu"):
        v = C.c_uint64()
    else:
        v = C.create_string_buffer(1024)
    rc = dlib().ascii_header_get(h, key.encode(), fmt.encode(), C.byref(v))
    if rc < 1:
        return None
    return v.value.decode() if isinstance(v, C.Array) else v.value


def header_set(header: bytes | str, key: str, value, size: int = HDR_SIZE) -> bytes:
    h = header.encode() if isinstance(header, str) else header
    buf = C.create_string_buffer(h, max(size, len(h) + 256))
    rc = dlib().ascii_header_set(buf, key.encode(), b"%s", str(value).encode())
    if rc != 0:
        raise ValueError(f"ascii_header_set {key}")
    return buf.value


def header_del(header: bytes | str, key: str) -> bytes:
    h = header.encode() if isinstance(header, str) else header
    buf = C.create_string_buffer(h, len(h) + 1)
    dlib().ascii_header_del(buf, key.encode())
    return buf.value


def header_block(text: bytes | str, size: int = HDR_SIZE) -> bytes:
    """NUL-padded fixed-size header block."""
    t = text.encode() if isinstance(text, str) else text
    if len(t) >= size:
        raise ValueError("header longer than the header block")
    return t + b"\0" * (size - len(t))


# ---- rings --------------------------------------------------------------------------

def create_ring(key: int, nbufs: int, bufsz: int, nreaders: int = 1, hdr_nbufs: int = 8,
                hdr_bufsz: int = HDR_SIZE, device: int = -1, page: bool = False) -> None:
    """device >= 0: data blocks in that GPU's memory (dada_db -g).  That ring
    is made by the dada_db executable, never in this process: its holder is
    forked, and forking a process that runs threads (torch) is not safe.
    page=True: the host blocks' pages are allocated now (dada_db -p, as the
    reference's launcher creates its rings, paf-baseband2power.py:114-115),
    not by the first write of the first block."""
    if device >= 0 or page:
        import subprocess
        r = subprocess.run([os.path.join(BIN_DIR, "dada_db"), "-k", f"{key:x}", "-b", str(bufsz),
                            "-n", str(nbufs), "-r", str(nreaders), "-H", str(hdr_bufsz)]
                           + (["-g", str(device)] if device >= 0 else ["-p"]),
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise OSError(f"dada_db {'-g %d' % device if device >= 0 else '-p'} {key:x}: {r.stderr.strip()}")
        if device >= 0:
            DEVICE_RINGS.append(dict(key=key, nbufs=nbufs, bufsz=bufsz, **device_ring_info(key)))
        return
    if dlib().dada_db_create(key, nbufs, bufsz, nreaders, hdr_nbufs, hdr_bufsz) != 0:
        raise OSError(C.get_errno(), f"dada_db_create {key:x}")


# every GPU-resident ring create_ring made in this process, with its holder's
# export record (device_ring_info) as it stood once the ring was ready: the
# GPU tests assert export_retries == 0 for each (tests/conftest.py)
DEVICE_RINGS: list[dict] = []


def device_ring_info(key: int) -> dict:
    """the holder of GPU-resident ring `key` (dada_device_ring_info): pid,
    state (1 serving, 2 blocks freed), importers it last counted, ring
    blocks exported only after a retry, and whether its primer allocation's
    export was refused"""
    info = DeviceInfo()
    if dlib().dada_device_ring_info(key, C.byref(info)) != 0:
        e = C.get_errno()
        raise OSError(e, f"dada_device_ring_info {key:x}: {os.strerror(e)}")
    return {n: getattr(info, n) for n, _ in DeviceInfo._fields_}


def device_error() -> str:
    """why this thread's last device-ring call failed (dada_device_error)"""
    return (dlib().dada_device_error() or b"").decode(errors="replace")


def destroy_ring(key: int) -> bool:
    return dlib().dada_db_destroy(key) == 0


class Hdu:
    """A dada_hdu_t as writer ('W'), reader ('R') or viewer of the data ring
    ('r': follows the writer without taking blocks, dada_hdu_open_view)."""

    def __init__(self, key: int, mode: str):
        L = dlib()
        self.mode = mode
        self._held, self._eod_held = 0, False  # read depth > 1: blocks held, EOD block behind them
        self.h = L.dada_hdu_create(None)
        L.dada_hdu_set_key(self.h, key)
        if L.dada_hdu_connect(self.h) != 0:
            L.dada_hdu_destroy(self.h)
            why = device_error()
            raise OSError(f"no ring at key {key:x}" + (f" ({why})" if why else ""))
        lock = {"W": L.dada_hdu_lock_write, "R": L.dada_hdu_lock_read, "r": L.dada_hdu_open_view}[mode]
        if lock(self.h) != 0:
            L.dada_hdu_destroy(self.h)
            raise OSError(f"cannot lock ring {key:x} for {mode}")
        s = HduStruct.from_address(self.h)
        self.data = s.data_block        # ipcio_t* (its first member is the ipcbuf_t)
        self.hdr = s.header_block       # ipcbuf_t*
        self.bufsz = L.ipcbuf_get_bufsz(self.data)
        self.device = L.ipcbuf_get_device(self.data)  # -1: host ring

    # writer ----------------------------------------------------------------------
    def write_header(self, text: bytes | str) -> None:
        L = dlib()
        p = L.ipcbuf_get_next_write(self.hdr)
        hsz = L.ipcbuf_get_bufsz(self.hdr)
        blk = header_block(text, hsz)
        C.memmove(p, blk, hsz)
        if L.ipcbuf_mark_filled(self.hdr, hsz) != 0:
            raise OSError("mark_filled header")

    def write_block(self, data: bytes | memoryview) -> None:
        L = dlib()
        bid = C.c_uint64()
        p = L.ipcio_open_block_write(self.data, C.byref(bid))
        if not p:
            raise OSError("open_block_write")
        n = len(data)
        if n > self.bufsz:
            raise ValueError("block too large")
        src = bytes(data)
        if L.ipcbuf_copy_in(self.data, p, src, n) != 0:  # hipMemcpy for a device ring
            raise OSError(f"copy into block: {device_error()}")
        L.ipcio_close_block_write(self.data, n)

    # reader ----------------------------------------------------------------------
    def read_header(self) -> bytes:
        L = dlib()
        if L.dada_hdu_open_read(self.h) != 0:
            raise OSError("open_read header")
        s = HduStruct.from_address(self.h)
        return C.string_at(s.header)

    def read_block(self):
        """bytes of the next block, or None at end of data (the 0-byte block
        PSRDADA's ipcio_close appends after a full one is taken and released
        here: it only carries the end of data)"""
        L = dlib()
        n, bid = C.c_uint64(), C.c_uint64()
        p = L.ipcio_open_block_read(self.data, C.byref(n), C.byref(bid))
        if not p:
            return None
        if not n.value:
            L.ipcio_close_block_read(self.data, 0)
            return None
        buf = C.create_string_buffer(n.value)
        if n.value and L.ipcbuf_copy_out(self.data, buf, p, n.value) != 0:
            raise OSError("copy out of block")
        L.ipcio_close_block_read(self.data, n.value)
        return buf.raw

    def view_block(self):
        """zero-copy uint8 view of the next block of a HOST ring, or None at
        end of data; valid until release_block(len(view))"""
        L = dlib()
        n, bid = C.c_uint64(), C.c_uint64()
        p = L.ipcio_open_block_read(self.data, C.byref(n), C.byref(bid))
        if not p:
            return None
        if not n.value:  # the end-of-data block
            L.ipcio_close_block_read(self.data, 0)
            return None
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(n.value,))

    def release_block(self, nbytes: int) -> None:
        if dlib().ipcio_close_block_read(self.data, nbytes) != 0:
            raise OSError("close_block_read")

    def set_read_depth(self, depth: int) -> None:
        """hold up to `depth` blocks at once (extension, include/b2p_dada.h)"""
        if dlib().ipcbuf_set_read_depth(self.data, depth) != 0:
            raise ValueError(f"read depth {depth}")
        self._held, self._eod_held = 0, False

    def open_block(self):
        """bytes of the next block, kept held, or None at end of data;
        release with close_block (oldest first).  A 0-byte end-of-data block
        is not returned: it goes back to the ring after the blocks before it"""
        L = dlib()
        n, bid = C.c_uint64(), C.c_uint64()
        p = L.ipcio_open_block_read(self.data, C.byref(n), C.byref(bid))
        if not p:
            return None
        if not n.value:
            if self._held:
                self._eod_held = True
            elif L.ipcio_close_block_read(self.data, 0) != 0:
                raise OSError("close_block_read")
            return None
        buf = C.create_string_buffer(n.value)
        if L.ipcbuf_copy_out(self.data, buf, p, n.value) != 0:
            raise OSError("copy out of block")
        self._held += 1
        return buf.raw

    def close_block(self) -> None:
        L = dlib()
        if L.ipcio_close_block_read(self.data, 0) != 0:
            raise OSError("close_block_read")
        self._held -= 1
        if self._eod_held and not self._held:
            self._eod_held = False
            if L.ipcio_close_block_read(self.data, 0) != 0:
                raise OSError("close_block_read")

    def eod(self) -> bool:
        return bool(dlib().ipcbuf_eod(self.data))

    def nfull(self, reader: int = -1) -> int:
        """blocks filled and not yet taken by reader `reader` (ipcbuf_get_nfull)"""
        return int(dlib().ipcbuf_get_nfull_iread(self.data, reader))

    def write(self, data: bytes) -> None:
        """stream bytes into the ring across blocks (ipcio_write)"""
        if dlib().ipcio_write(self.data, bytes(data), len(data)) != len(data):
            raise OSError("ipcio_write")

    def read(self, nbytes: int) -> bytes:
        """up to nbytes of the stream (fewer at end of data; ipcio_read)"""
        buf = C.create_string_buffer(nbytes)
        n = dlib().ipcio_read(self.data, buf, nbytes)
        if n < 0:
            raise OSError("ipcio_read")
        return buf.raw[:n]

    def close(self) -> None:
        if self.h:
            L = dlib()
            {"W": L.dada_hdu_unlock_write, "R": L.dada_hdu_unlock_read,
             "r": L.dada_hdu_close_view}[self.mode](self.h)
            L.dada_hdu_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_dada_file(path: str, header: bytes | str, payload) -> None:
    """A DADA file: 4096-B ASCII header then the payload (the files paf_diskdb
    reads, diskdb.cu:17,69)."""
    with open(path, "wb") as f:
        f.write(header_block(header))
        f.write(memoryview(payload))


def read_dada_file(path: str):
    import numpy as np
    with open(path, "rb") as f:
        hdr = f.read(HDR_SIZE)
        data = np.frombuffer(f.read(), dtype=np.uint8)
    return hdr.split(b"\0", 1)[0], data


# ---- BMF data-frame headers (include/b2p_df.h) ---------------------------------

class DfHdr(C.Structure):
    """b2p_df_hdr_t (= hdr_t, hdr.h:6-14)"""
    _fields_ = [("valid", C.c_int), ("idf", C.c_uint64), ("sec", C.c_uint64),
                ("epoch", C.c_int), ("beam", C.c_int), ("freq", C.c_double)]


def _df_lib():
    L = dlib()
    if not getattr(L, "_df_ready", False):
        L.b2p_df_decode.argtypes = [C.c_void_p, C.POINTER(DfHdr)]
        L.b2p_df_decode.restype = None
        L.b2p_df_encode.argtypes = [C.POINTER(DfHdr), C.c_void_p]
        L.b2p_df_encode.restype = None
        L.b2p_df_index.argtypes = [C.POINTER(DfHdr), C.POINTER(DfHdr)]
        L.b2p_df_index.restype = C.c_int64
        L.b2p_df_ref_advance.argtypes = [C.POINTER(DfHdr), C.c_uint64]
        L.b2p_df_ref_advance.restype = None
        L.b2p_df_chunk_from_ip.argtypes = [C.c_uint32]
        L.b2p_df_chunk_from_ip.restype = C.c_int
        L.b2p_df_epoch_days.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_double)]
        L.b2p_df_epoch_days.restype = C.c_int
        L.b2p_df_start_time.argtypes = [C.POINTER(DfHdr), C.c_double, C.c_char_p, C.c_size_t,
                                        C.POINTER(C.c_uint64)]
        L.b2p_df_start_time.restype = C.c_int
        L._df_ready = True
    return L


def df_decode(df: bytes) -> DfHdr:
    h = DfHdr()
    buf = C.create_string_buffer(bytes(df[:64]), 64)
    _df_lib().b2p_df_decode(buf, C.byref(h))
    return h


def df_encode(idf: int, sec: int, valid: int = 1, epoch: int = 0, beam: int = 0,
              freq: float = 0.0) -> bytes:
    h = DfHdr(valid, idf, sec, epoch, beam, freq)
    buf = C.create_string_buffer(64)
    _df_lib().b2p_df_encode(C.byref(h), buf)
    return buf.raw


def df_index(hdr: DfHdr, ref: DfHdr) -> int:
    return int(_df_lib().b2p_df_index(C.byref(hdr), C.byref(ref)))


def df_ref_advance(ref: DfHdr, ndf: int) -> DfHdr:
    r = DfHdr(ref.valid, ref.idf, ref.sec, ref.epoch, ref.beam, ref.freq)
    _df_lib().b2p_df_ref_advance(C.byref(r), ndf)
    return r


def df_chunk_from_ip(a: int, b: int, c: int, d: int) -> int:
    """chunk of the sender a.b.c.d (sin_addr.s_addr as stored, network order)"""
    s_addr = a | (b << 8) | (c << 16) | (d << 24)  # bytes in memory: a, b, c, d
    return int(_df_lib().b2p_df_chunk_from_ip(s_addr))


def df_epoch_days(epoch_file: str, epoch: int) -> float:
    """b2p_df_epoch_days: the day number the epoch file gives `epoch`
    (capture.c:808-815); OSError if the file is missing, KeyError if the
    epoch is not listed"""
    d = C.c_double()
    rc = _df_lib().b2p_df_epoch_days(epoch_file.encode(), epoch, C.byref(d))
    if rc == -1:
        raise OSError(f"cannot open epoch file {epoch_file}")
    if rc == -2:
        raise KeyError(f"epoch {epoch} not in {epoch_file}")
    return d.value


def df_start_time(idf: int, sec: int, days: float) -> tuple[str, int]:
    """(UTC_START, PICOSECONDS) of a capture starting at frame (idf, sec)
    (b2p_df_start_time, acquire_start_time capture.c:819-825)"""
    h = DfHdr(1, idf, sec, 0, 0, 0.0)
    buf = C.create_string_buffer(64)
    ps = C.c_uint64()
    if _df_lib().b2p_df_start_time(C.byref(h), days, buf, 64, C.byref(ps)) != 0:
        raise ValueError("start time does not convert")
    return buf.value.decode(), int(ps.value)
