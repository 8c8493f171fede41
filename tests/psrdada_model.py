"""A second, independent statement of PSRDADA's ring protocol, in Python --
test infrastructure only (like oracle/): it checks that libpafdada's rings
are PSRDADA rings on the wire.

It shares no code with csrc/dada: it talks to the SysV segments and
semaphores directly (libc through ctypes) and takes every field offset of
the shared ipcsync_t from tests/golden/psrdada_abi.json -- the layout
tools/psrdada_dwarf.py read out of the reference's statically linked
libpsrdada.  The steps follow that library's code as disassembled from the
reference's paf_diskdb (addresses cited per step, protocol summary in the
fixture's "protocol" entry):

  writer  lock_write @0x403b00, get_next_write @0x403f20, enable_sod
          @0x403cd0, mark_filled @0x404170, ipcio_close @0x405c10
  reader  lock_read @0x404360, get_next_read @0x404710, mark_cleared
          @0x404b80, unlock_read @0x4045f0

A process using this model plays the part of a libpsrdada process (dada_db /
dada_dbdisk / a PSRDADA writer) beside libpafdada's executables.
"""
from __future__ import annotations

import ctypes as C
import ctypes.util
import json
import os

from conftest import REPO

ABI = json.load(open(os.path.join(REPO, "tests", "golden", "psrdada_abi.json")))
SYNC = {m["name"]: m for m in ABI["structs"]["ipcsync_t"]["members"]}
SYNC_SIZE = ABI["structs"]["ipcsync_t"]["size"]
P = ABI["protocol"]
STEP = P["keys"]["semkey_connect"]
XFERS = 8
SODACK, EODACK, FULL, CLEAR, READER_CONN = (P["sem_data"][k] for k in
                                            ("SODACK", "EODACK", "FULL", "CLEAR", "READER_CONN"))
WRITE, READ = P["sem_connect"]["WRITE"], P["sem_connect"]["READ"]
IPC_NOWAIT, SEM_UNDO, IPC_RMID, IPC_STAT, GETVAL = 0o4000, 0x1000, 0, 2, 12

_libc = C.CDLL(ctypes.util.find_library("c"), use_errno=True)
_libc.shmget.argtypes = [C.c_int, C.c_size_t, C.c_int]
_libc.shmat.restype = C.c_void_p
_libc.shmat.argtypes = [C.c_int, C.c_void_p, C.c_int]
_libc.shmdt.argtypes = [C.c_void_p]
_libc.semget.argtypes = [C.c_int, C.c_int, C.c_int]
_libc.semctl.argtypes = [C.c_int, C.c_int, C.c_int]


class SemBuf(C.Structure):
    _fields_ = [("sem_num", C.c_ushort), ("sem_op", C.c_short), ("sem_flg", C.c_short)]


_libc.semop.argtypes = [C.c_int, C.POINTER(SemBuf), C.c_size_t]

_CTYPES = {"uint64_t": C.c_uint64, "int": C.c_int32, "key_t": C.c_int32,
           "unsigned int": C.c_uint32, "char": C.c_char}


def semop(semid: int, num: int, op: int, flags: int = 0) -> None:
    sb = SemBuf(num, op, flags)
    while _libc.semop(semid, C.byref(sb), 1) != 0:
        e = C.get_errno()
        if e != 4:  # EINTR
            raise OSError(e, os.strerror(e))


def semval(semid: int, num: int) -> int:
    return _libc.semctl(semid, num, GETVAL)


class Sync:
    """field access to an attached ipcsync_t by the DWARF offsets"""

    def __init__(self, addr: int):
        self.addr = addr

    def _ptr(self, name, i=0):
        m = SYNC[name]
        base = m["type"].split("[")[0]
        t = _CTYPES[base]
        return C.cast(self.addr + m["offset"] + i * C.sizeof(t), C.POINTER(t))

    def get(self, name, i=0):
        v = self._ptr(name, i)[0]
        return v[0] if isinstance(v, bytes) else v

    def set(self, name, value, i=0):
        p = self._ptr(name, i)
        p[0] = bytes([value]) if SYNC[name]["type"].startswith("char") else value


class Ring:
    """one PSRDADA ring (data or header) at `key`, attached the way
    ipcbuf_connect does (ipcsync_get @0x402fe0 + ipcbuf_get @0x403090)"""

    def __init__(self, key: int):
        self.key = key
        self.syncid = _libc.shmget(key, SYNC_SIZE, 0o666)
        if self.syncid < 0:
            raise OSError(C.get_errno(), f"no ring at {key:x}")
        a = _libc.shmat(self.syncid, None, 0)
        if a in (None, C.c_void_p(-1).value):
            raise OSError(C.get_errno(), "shmat")
        self.s = Sync(a)
        self.nbufs = self.s.get("nbufs")
        self.bufsz = self.s.get("bufsz")
        self.n_readers = self.s.get("n_readers")
        self.count_addr = a + P["ipcsync_segment"]["count_offset"]
        self.shmkey_addr = self.count_addr + self.nbufs
        self.semid_connect = _libc.semget(self.s.get("semkey_connect"), 2, 0o666)
        self.semid_data = [_libc.semget(self.s.get("semkey_data", r), 5, 0o666)
                           for r in range(self.n_readers)]
        self.blocks = []
        for i in range(self.nbufs):
            k = C.c_int32.from_address(self.shmkey_addr + 4 * i).value
            sid = _libc.shmget(k, self.bufsz, 0o666)
            if sid < 0:
                raise OSError(C.get_errno(), f"no block {i}")
            self.blocks.append(_libc.shmat(sid, None, 0))
        self.state, self.xfer, self.iread = "viewer", 0, -1

    def count(self, b: int) -> int:
        return C.c_uint8.from_address(self.count_addr + b).value

    def set_count(self, b: int, v: int) -> None:
        C.c_uint8.from_address(self.count_addr + b).value = v

    def close(self):
        for b in self.blocks:
            _libc.shmdt(b)
        _libc.shmdt(self.s.addr)
        self.blocks = []

    # ---- writer ------------------------------------------------------------------------
    def lock_write(self):  # @0x403b00
        semop(self.semid_connect, WRITE, -1, SEM_UNDO)
        self.state = "writing" if self.s.get("w_state") else "wchange"
        self.xfer = self.s.get("w_xfer") % XFERS

    def enable_sod(self, start_buf: int, start_byte: int):  # @0x403cd0
        s = self.s
        for r in range(self.n_readers):
            semop(self.semid_data[r], SODACK, -1)
        x = s.get("w_xfer") % XFERS
        self.xfer = x
        s.set("s_buf", start_buf, x)
        s.set("s_byte", start_byte, x)
        w = s.get("w_buf")
        if w == 0:
            s.set("eod", 0, x)
        for b in range(start_buf, w):
            self.set_count(b % self.nbufs, self.count(b % self.nbufs) + 1)
        self.state = "writing"
        s.set("w_state", 3)
        if w - start_buf:
            for r in range(self.n_readers):
                semop(self.semid_data[r], FULL, w - start_buf)

    def get_next_write(self) -> int:  # @0x403f20
        if self.state == "wchange":
            self.enable_sod(self.s.get("w_buf"), 0)
        b = self.s.get("w_buf") % self.nbufs
        while self.count(b):
            for r in range(self.n_readers):
                semop(self.semid_data[r], CLEAR, -1)
            self.set_count(b, self.count(b) - 1)
        return self.blocks[b]

    def mark_filled(self, nbytes: int):  # @0x404170
        s = self.s
        if self.state == "writer":  # start of data disabled: invisible to readers
            s.set("w_buf", s.get("w_buf") + 1)
            return
        if self.state == "wchange" or nbytes < self.bufsz:
            for r in range(self.n_readers):
                semop(self.semid_data[r], EODACK, -1)
            s.set("e_buf", s.get("w_buf"), self.xfer)
            s.set("e_byte", nbytes, self.xfer)
            s.set("eod", 1, self.xfer)
            s.set("w_xfer", s.get("w_xfer") + 1)
            self.xfer = s.get("w_xfer") % XFERS
            self.state = "writer"
            s.set("w_state", 0)
        w = s.get("w_buf")
        self.set_count(w % self.nbufs, self.count(w % self.nbufs) + 1)
        s.set("w_buf", w + 1)
        for r in range(self.n_readers):
            semop(self.semid_data[r], FULL, 1)

    def write_block(self, data: bytes):
        p = self.get_next_write()
        C.memmove(p, data, len(data))
        self.mark_filled(len(data))

    def disable_sod(self):  # @0x403c60 (ipcio_open 'w')
        assert self.state == "wchange"
        self.state = "writer"

    def write_invisible(self, data: bytes):
        """a block written while the start of data is disabled (WRITER):
        get_next_write's slot wait, then mark_filled only counts w_buf"""
        b = self.s.get("w_buf") % self.nbufs
        while self.count(b):
            for r in range(self.n_readers):
                semop(self.semid_data[r], CLEAR, -1)
            self.set_count(b, self.count(b) - 1)
        C.memmove(self.blocks[b], data, len(data))
        self.mark_filled(len(data))

    def end_transfer(self):
        """ipcio_close @0x405c10 after full blocks: enable_eod + a 0-byte
        end-of-data block, marked without taking its slot first (libpsrdada
        does not wait for it; libpafdada does)"""
        if self.state == "writing":
            self.state = "wchange"
            self.mark_filled(0)

    def unlock_write(self):  # @0x403b90
        semop(self.semid_connect, WRITE, 1, SEM_UNDO)
        self.state = "viewer"

    # ---- reader ------------------------------------------------------------------------
    def lock_read(self):  # @0x404360
        semop(self.semid_connect, READ, -1, SEM_UNDO)
        order = sorted(range(self.n_readers), key=lambda r: (self.s.get("r_bufs", r), r))
        for r in order:
            sb = SemBuf(READER_CONN, -1, IPC_NOWAIT | SEM_UNDO)
            if _libc.semop(self.semid_data[r], C.byref(sb), 1) == 0:
                self.iread = r
                break
        else:
            raise OSError("no free reader slot")
        self.state = "reading" if self.s.get("r_states", self.iread) else "reader"
        self.xfer = self.s.get("r_xfers", self.iread) % XFERS

    def get_next_read(self):  # @0x404710: (address, bytes) or None at end of data
        if self.state == "rstop":
            return None
        s, r = self.s, self.iread
        semop(self.semid_data[r], FULL, -1)
        start = 0
        if self.state == "reader":
            self.xfer = s.get("r_xfers", r) % XFERS
            self.state = "reading"
            s.set("r_states", 6, r)
            s.set("r_bufs", s.get("s_buf", self.xfer), r)
            start = s.get("s_byte", self.xfer)
            semop(self.semid_data[r], SODACK, 1)
        b = s.get("r_bufs", r)
        if s.get("eod", self.xfer) and s.get("e_buf", self.xfer) == b:
            n = s.get("e_byte", self.xfer) - start
        else:
            n = self.bufsz - start
        return self.blocks[b % self.nbufs] + start, n

    def mark_cleared(self):  # @0x404b80
        s, r = self.s, self.iread
        semop(self.semid_data[r], CLEAR, 1)
        if s.get("eod", self.xfer) and s.get("r_bufs", r) == s.get("e_buf", self.xfer):
            self.state = "rstop"
            s.set("r_states", 0, r)
            s.set("r_xfers", s.get("r_xfers", r) + 1, r)
            self.xfer = s.get("r_xfers", r) % XFERS
            semop(self.semid_data[r], EODACK, 1)
        else:
            s.set("r_bufs", s.get("r_bufs", r) + 1, r)

    def read_transfer(self):
        """every block of the next transfer: list of bytes (0-byte EOD block dropped)"""
        out = []
        while (got := self.get_next_read()) is not None:
            p, n = got
            if n:
                out.append(C.string_at(p, n))
            self.mark_cleared()
        return out

    def unlock_read(self):  # @0x4045f0
        semop(self.semid_data[self.iread], READER_CONN, 1, SEM_UNDO)
        semop(self.semid_connect, READ, 1, SEM_UNDO)
        self.iread, self.state = -1, "viewer"


def header_block(ring: Ring, text: bytes) -> bytes:
    return text + b"\0" * (ring.bufsz - len(text))
