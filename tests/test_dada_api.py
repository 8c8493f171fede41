"""The rest of the PSRDADA API libpafdada exports (CPU): every function the
reference's linked libpsrdada holds (tests/golden/psrdada_abi.json) beyond
the writer / reader calls its hosts make -- viewers (ipcio 'r',
dada_hdu_open_view), semaphore counts, tell / seek, the deferred start of
data (ipcio 'w' + ipcio_start / ipcio_stop), writer reset, hard reset,
zero_next_write, ascii_header_find / get_size, multilog_fprintf, ipcio_create
/ destroy, ipc_alloc / ipc_semop.  Where the protocol is involved the other
side is tests/psrdada_model.py, an independent statement of libpsrdada.
"""
import ctypes as C
import os
import re
import threading

import numpy as np
import pytest

import psrdada_model as pm
from paf_b2p import dada

L = dada.dlib()
P = C.c_void_p
_key_base = 0x7000 + (os.getpid() % 48) * 0x100
_n = [0]
SEEK_SET, SEEK_CUR = 0, 1
IPC_CREAT, IPC_RMID = 0o1000, 0
libc = C.CDLL(None, use_errno=True)
libc.shmat.restype = P
libc.shmat.argtypes = [C.c_int, P, C.c_int]
libc.shmdt.argtypes = [P]
libc.fopen.restype = P
libc.fclose.argtypes = [P]

for name, res, args in [
    ("ipcio_tell", C.c_uint64, [P]), ("ipcio_seek", C.c_int64, [P, C.c_int64, C.c_int]),
    ("ipcbuf_tell_write", C.c_int64, [P]), ("ipcbuf_tell_read", C.c_int64, [P]),
    ("ipcio_start", C.c_int, [P, C.c_uint64]), ("ipcio_stop", C.c_int, [P]),
    ("ipcio_close", C.c_int, [P]), ("ipcio_space_left", C.c_int64, [P]),
    ("ipcio_percent_full", C.c_float, [P]), ("ipcbuf_reset", C.c_int, [P]),
    ("ipcbuf_hard_reset", C.c_int, [P]), ("ipcbuf_zero_next_write", C.c_int, [P]),
    ("ipcio_zero_next_block", C.c_int, [P]), ("ipcbuf_get_write_count", C.c_uint64, [P]),
    ("ipcbuf_connect", C.c_int, [P, C.c_int]), ("ipcbuf_disconnect", C.c_int, [P]),
    ("ascii_header_find", C.c_void_p, [C.c_char_p, C.c_char_p]),
    ("ascii_header_get_size", C.c_size_t, [C.c_char_p]), ("ascii_header_get_size_fd", C.c_size_t, [C.c_int]),
    ("multilog_fprintf", C.c_int, [P, C.c_int, C.c_char_p, C.c_char_p]),
    ("dada_hdu_db_addresses", C.c_void_p, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("dada_hdu_lock_write_spec", C.c_int, [P, C.c_char]),
    ("ipcio_create", C.c_int, [P, C.c_int, C.c_uint64, C.c_uint64, C.c_uint]),
    ("ipcio_destroy", C.c_int, [P]), ("ipcio_connect", C.c_int, [P, C.c_int]),
    ("ipcio_disconnect", C.c_int, [P]), ("ipcbuf_get_nbufs", C.c_uint64, [P]),
    ("ipc_alloc", C.c_void_p, [C.c_int, C.c_size_t, C.c_int, C.POINTER(C.c_int)]),
    ("ipc_semop", C.c_int, [C.c_int, C.c_short, C.c_short, C.c_short]),
    ("ipcbuf_get_next_readable", C.c_void_p, [P, C.POINTER(C.c_uint64)]),
    ("ipcbuf_mark_cleared", C.c_int, [P]),
    ("ipcbuf_get_write_byte_xfer", C.c_uint64, [P]), ("ipcbuf_set_soclock_buf", C.c_uint64, [P]),
    ("ipcio_get_start_minimum", C.c_uint64, [P]),
    ("ipcbuf_set_read_depth", C.c_int, [P, C.c_int]),
    ("ipcbuf_lock_read", C.c_int, [P]), ("ipcbuf_unlock_read", C.c_int, [P]),
    ("ipcbuf_get_next_read", C.c_void_p, [P, C.POINTER(C.c_uint64)]),
]:
    f = getattr(L, name)
    f.restype, f.argtypes = res, args


def fresh_key():
    k = _key_base + 2 * (_n[0] % 120)
    _n[0] += 1
    dada.destroy_ring(k)
    return k


@pytest.fixture
def ring():
    made = []

    def make(nbufs, bufsz, nreaders=1):
        k = fresh_key()
        dada.create_ring(k, nbufs, bufsz, nreaders)
        made.append(k)
        return k

    yield make
    for k in made:
        dada.destroy_ring(k)


def blocks(n, bufsz, seed=0):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, bufsz, dtype=np.uint8).tobytes() for _ in range(n)]


def sync_of(k):
    """the ring's shared state, read with the model's DWARF offsets"""
    r = pm.Ring(k)
    st = {f: r.s.get(f) for f in ("w_buf", "w_xfer", "w_state")}
    st["r_bufs0"], st["r_xfers0"] = r.s.get("r_bufs", 0), r.s.get("r_xfers", 0)
    st["count"] = [r.count(b) for b in range(r.nbufs)]
    st["sodack"] = pm.semval(r.semid_data[0], pm.SODACK)
    st["eodack"] = pm.semval(r.semid_data[0], pm.EODACK)
    st["full"] = pm.semval(r.semid_data[0], pm.FULL)
    st["clear"] = pm.semval(r.semid_data[0], pm.CLEAR)
    r.close()
    return st


# ---- viewers ---------------------------------------------------------------------------

def test_viewer_follows_the_writer_and_stops_at_end_of_data(ring):
    """a viewer starts at the newest block written, then takes each block as
    it is written, takes nothing from the ring (the reader still gets every
    block), and stops once reader 0 is at the end-of-data block"""
    k = ring(4, 64)
    b = blocks(3, 64)
    with dada.Hdu(k, "W") as w:
        w.write_block(b[0])
        w.write_block(b[1])
        with dada.Hdu(k, "r") as v:
            assert v.read_block() == b[1]          # the newest, not the first
            w.write_block(b[2])
            assert v.read_block() == b[2]
            assert w.nfull(0) == 3                 # nothing taken by the viewer
            w.close()                              # 0-byte end-of-data block
            with dada.Hdu(k, "R") as r:
                assert [r.read_block() for _ in range(4)] == b + [None]
            got = [v.read_block() for _ in range(2)]
            assert got == [None, None] and v.eod()


def test_viewer_of_a_psrdada_writer_skips_ahead_when_lapped(ring):
    """the writer is the PSRDADA model: a viewer that falls a ring behind
    jumps to the oldest block still in the ring (w_buf - nbufs + 1)"""
    k = ring(2, 32)
    b = blocks(5, 32, seed=1)
    mw = pm.Ring(k)
    mw.lock_write()
    mw.write_block(b[0])
    with dada.Hdu(k, "r") as v, dada.Hdu(k, "R") as r:
        assert v.read_block() == b[0]
        assert r.read_block() == b[0]
        for x in b[1:]:                            # the reader keeps the writer going
            mw.write_block(x)
            assert r.read_block() == x
        assert v.read_block() == b[4]              # blocks 1..3 were lapped
    mw.end_transfer()
    mw.unlock_write()
    mw.close()


def test_viewer_streams_with_ipcio_read(ring):
    k = ring(4, 64)
    b = blocks(3, 64, seed=2)
    with dada.Hdu(k, "W") as w:
        w.write_block(b[0])
        with dada.Hdu(k, "r") as v:
            assert v.read(10) == b[0][:10]         # the view starts at its first read
            w.write_block(b[1])
            w.write_block(b[2])
            assert v.read(100) == (b[0] + b[1])[10:110]
            # ipcbuf_tell_read of a viewer counts up to viewbuf, the NEXT block
            # (libpsrdada @0x404ae0): a viewer's tell runs one block ahead
            assert L.ipcio_tell(v.data) == 110 + 64


# ---- semaphore counts ------------------------------------------------------------------

def test_semaphore_counts_follow_the_protocol(ring):
    k = ring(4, 64, nreaders=2)
    with dada.Hdu(k, "W") as w:
        d = w.data
        assert [L.ipcbuf_get_sodack_iread(d, r) for r in (0, 1)] == [8, 8]
        assert [L.ipcbuf_get_eodack_iread(d, r) for r in (0, 1)] == [8, 8]
        assert [L.ipcbuf_get_reader_conn_iread(d, r) for r in (0, 1)] == [1, 1]
        assert L.ipcbuf_get_read_semaphore_count(d) == 2
        b = blocks(2, 64, seed=3)
        w.write_block(b[0])
        w.write_block(b[1])
        assert [L.ipcbuf_get_nfull_iread(d, r) for r in (0, 1)] == [2, 2]
        assert L.ipcbuf_get_nfull(d) == 2           # not a reader: reader 0's
        assert L.ipcbuf_get_sodack_iread(d, 0) == 7  # the start of data took one
        assert L.ipcio_space_left(d) == (4 - 2) * 64
        assert L.ipcio_percent_full(d) == pytest.approx(0.5)
        with dada.Hdu(k, "R") as r:
            slot = C.c_int.from_address(r.data + 96).value  # ipcbuf_t.iread
            assert L.ipcbuf_get_reader_conn_iread(d, slot) == 0
            assert L.ipcbuf_get_read_semaphore_count(d) == 1
            assert r.read_block() == b[0]
            assert L.ipcbuf_get_nfull_iread(d, slot) == 1
            assert L.ipcbuf_get_nclear_iread(d, slot) == 1
            assert L.ipcbuf_get_sodack_iread(d, slot) == 8  # acknowledged
        assert L.ipcio_close(d) == 0               # end of data: EODACK taken
        assert [L.ipcbuf_get_eodack_iread(d, r) for r in (0, 1)] == [7, 7]


# ---- tell / seek -----------------------------------------------------------------------

def test_tell_and_seek_in_a_transfer(ring):
    k = ring(4, 64)
    stream = bytes(np.random.default_rng(4).integers(0, 256, 160, dtype=np.uint8))
    with dada.Hdu(k, "W") as w:
        w.write(stream[:100])
        assert L.ipcio_tell(w.data) == 100
        assert L.ipcbuf_tell_write(w.data) == 64   # one block marked so far
        w.write(stream[100:])
    with dada.Hdu(k, "R") as r:
        assert r.read(10) == stream[:10]
        assert L.ipcio_tell(r.data) == 10
        assert L.ipcio_seek(r.data, 70, SEEK_SET) == 70   # forward: read and dropped
        assert L.ipcbuf_tell_read(r.data) == 64
        assert r.read(5) == stream[70:75]
        assert L.ipcio_seek(r.data, -8, SEEK_CUR) == 67   # back within the block
        assert r.read(3) == stream[67:70]
        assert L.ipcio_seek(r.data, 10, SEEK_SET) == -1   # not back past the block
        assert r.read(1000) == stream[70:]
        assert r.eod()


# ---- deferred start of data ------------------------------------------------------------

def test_deferred_start_and_stop_read_by_psrdada(ring):
    """ipcio 'w': blocks are written invisibly until ipcio_start names the
    stream byte the transfer starts at; ipcio_stop ends it and keeps the
    lock; a second start, then ipcio_close.  The PSRDADA model reader sees
    exactly stream[start1:stop1] and stream[start2:end]"""
    k = ring(8, 64)
    stream = bytes(np.random.default_rng(5).integers(0, 256, 7 * 64, dtype=np.uint8))
    h = L.dada_hdu_create(None)
    L.dada_hdu_set_key(h, k)
    assert L.dada_hdu_connect(h) == 0
    assert L.dada_hdu_lock_write_spec(h, b"w") == 0
    d = dada.HduStruct.from_address(h).data_block
    assert L.ipcio_write(d, stream[:192], 192) == 192
    assert L.ipcio_start(d, 96) == 0                      # block 1, byte 32
    assert L.ipcio_write(d, stream[192:320], 128) == 128
    assert L.ipcio_stop(d) == 0                           # end of data after block 4
    m = pm.Ring(k)
    m.lock_read()
    assert b"".join(m.read_transfer()) == stream[96:320]
    assert L.ipcio_write(d, stream[320:384], 64) == 64
    assert L.ipcio_start(d, 352) == 0                     # block 5 not marked yet: pending
    assert L.ipcio_write(d, stream[384:448], 64) == 64
    assert L.ipcio_close(d) == 0
    m.state = "reader"                                    # ipcbuf_reset of the model reader
    assert b"".join(m.read_transfer()) == stream[352:448]
    m.unlock_read()
    m.close()
    assert L.dada_hdu_unlock_write(h) != 0 or True        # already closed by ipcio_close
    L.dada_hdu_destroy(h)


def test_deferred_start_read_by_libpafdada(ring):
    """the same deferred start, libpafdada on both sides: the reader's first
    block starts at the transfer's start byte (s_byte)"""
    k = ring(8, 64)
    stream = bytes(np.random.default_rng(9).integers(0, 256, 5 * 64, dtype=np.uint8))
    h = L.dada_hdu_create(None)
    L.dada_hdu_set_key(h, k)
    assert L.dada_hdu_connect(h) == 0 and L.dada_hdu_lock_write_spec(h, b"w") == 0
    d = dada.HduStruct.from_address(h).data_block
    assert L.ipcio_write(d, stream[:200], 200) == 200
    assert L.ipcio_start(d, 70) == 0                      # block 1, byte 6
    assert L.ipcio_write(d, stream[200:], len(stream) - 200) == len(stream) - 200
    assert L.ipcio_close(d) == 0
    with dada.Hdu(k, "R") as r:
        assert r.read(1000) == stream[70:]
        assert r.eod()
    L.dada_hdu_unlock_write(h)
    L.dada_hdu_destroy(h)


def test_psrdada_deferred_writer_read_by_libpafdada(ring):
    """the PSRDADA model writes blocks with the start of data disabled, then
    enables it at block 2 byte 10 (enable_sod, as ipcio_start does) and ends
    the transfer; paf's reader gets exactly the stream from there"""
    k = ring(8, 64)
    blocks = [bytes(np.random.default_rng(10 + i).integers(0, 256, 64, dtype=np.uint8)) for i in range(5)]
    m = pm.Ring(k)
    m.lock_write()
    m.disable_sod()
    for b in blocks[:3]:
        m.write_invisible(b)
    m.enable_sod(2, 10)                                   # w_buf 3 > 2: blocks 2.. become visible
    for b in blocks[3:]:
        m.write_block(b)
    m.end_transfer()
    m.unlock_write()
    m.close()
    with dada.Hdu(k, "R") as r:
        assert r.read(1000) == b"".join(blocks)[2 * 64 + 10:]
        assert r.eod()


def test_start_refused_unless_deferred(ring):
    k = ring(2, 64)
    with dada.Hdu(k, "W") as w:
        assert L.ipcio_start(w.data, 0) == -1
    with dada.Hdu(k, "R") as r:
        assert L.ipcio_stop(r.data) == -1


# ---- resets and zeroing ----------------------------------------------------------------

def test_writer_reset_returns_the_ring_to_its_created_state(ring):
    k = ring(3, 64)
    b = blocks(4, 64, seed=6)
    with dada.Hdu(k, "W") as w:
        for x in b[:2]:
            w.write_block(x)
    with dada.Hdu(k, "R") as r:
        assert [r.read_block() for _ in range(3)] == b[:2] + [None]
    with dada.Hdu(k, "W") as w:
        assert L.ipcbuf_reset(w.data) == 0
        st = sync_of(k)
        assert (st["w_buf"], st["w_xfer"], st["r_bufs0"], st["r_xfers0"]) == (0, 0, 0, 0)
        assert st["count"] == [0, 0, 0] and (st["sodack"], st["eodack"]) == (8, 8)
        for x in b[2:]:
            w.write_block(x)
    with dada.Hdu(k, "R") as r:
        assert [r.read_block() for _ in range(3)] == b[2:] + [None]


def test_transfer_after_reset_is_not_cut_at_an_old_end_block(ring):
    """a writer reset returns every transfer slot to its created state: the
    second transfer after it runs past the block where the second transfer
    before it ended (e_buf[1] = 3), instead of ending there with that
    transfer's byte count (libpsrdada's reset rewrites only eod[])"""
    k = ring(4, 64)
    b = blocks(8, 64, seed=11)
    for x in ([b[0]], [b[1]]):         # transfers 0 and 1: a block, then the 0-byte end block
        with dada.Hdu(k, "W") as w:
            w.write_block(x[0])
        with dada.Hdu(k, "R") as r:
            assert [r.read_block() for _ in range(2)] == x + [None]
    m = pm.Ring(k)
    assert [m.s.get("e_buf", x) for x in (0, 1)] == [1, 3]
    m.close()
    with dada.Hdu(k, "W") as w:
        assert L.ipcbuf_reset(w.data) == 0
        m = pm.Ring(k)
        assert [m.s.get("e_buf", x) for x in range(8)] == [0] * 8
        assert [m.s.get("e_byte", x) for x in range(8)] == [0] * 8
        m.close()
        w.write_block(b[2])            # transfer 0 after the reset: blocks 0, 1
    with dada.Hdu(k, "R") as r:
        assert [r.read_block() for _ in range(2)] == [b[2], None]
    got = []

    def reader():
        with dada.Hdu(k, "R") as r:
            while (x := r.read_block()) is not None:
                got.append(x)

    t = threading.Thread(target=reader)
    t.start()
    with dada.Hdu(k, "W") as w:        # transfer 1 after the reset: blocks 2..6 (old end: 3)
        for x in b[3:8]:
            w.write_block(x)
    t.join(timeout=30)
    assert not t.is_alive() and got == b[3:8]


def test_read_depth_set_before_the_read_lock_is_kept(ring):
    """ipcbuf_set_read_depth may come before ipcbuf_lock_read: the lock (and
    an unlock / relock) keeps it, so the reader can hold two blocks"""
    k = ring(4, 64)
    b = blocks(3, 64, seed=12)
    with dada.Hdu(k, "W") as w:
        for x in b:
            w.write_block(x)
    ib = C.create_string_buffer(104)
    assert L.ipcbuf_connect(ib, k) == 0
    assert L.ipcbuf_set_read_depth(ib, 2) == 0
    assert L.ipcbuf_lock_read(ib) == 0
    n = C.c_uint64()
    p0 = L.ipcbuf_get_next_read(ib, C.byref(n))
    p1 = L.ipcbuf_get_next_read(ib, C.byref(n))    # a second block held at once
    assert p0 and p1 and C.string_at(p0, 64) == b[0] and C.string_at(p1, 64) == b[1]
    assert L.ipcbuf_mark_cleared(ib) == 0 and L.ipcbuf_mark_cleared(ib) == 0
    assert L.ipcbuf_unlock_read(ib) == 0 and L.ipcbuf_lock_read(ib) == 0
    q0 = L.ipcbuf_get_next_read(ib, C.byref(n))
    q1 = L.ipcbuf_get_next_read(ib, C.byref(n))    # still depth 2 after the relock
    assert q0 and C.string_at(q0, 64) == b[2] and q1 and n.value == 0   # the 0-byte end block
    assert L.ipcbuf_mark_cleared(ib) == 0 and L.ipcbuf_mark_cleared(ib) == 0
    assert L.ipcbuf_unlock_read(ib) == 0
    L.ipcbuf_disconnect(ib)


def test_hard_reset_without_anyone_reading(ring):
    k = ring(3, 64)
    b = blocks(5, 64, seed=7)
    with dada.Hdu(k, "W") as w:
        for x in b[:2]:
            w.write_block(x)                      # nobody reads these
    ib = C.create_string_buffer(104)
    assert L.ipcbuf_connect(ib, k) == 0
    assert L.ipcbuf_hard_reset(ib) == 0
    st = sync_of(k)
    assert (st["w_buf"], st["full"], st["clear"], st["count"]) == (0, 0, 0, [0, 0, 0])
    L.ipcbuf_disconnect(ib)
    with dada.Hdu(k, "W") as w:
        for x in b[2:4]:
            w.write_block(x)                      # no wait on the discarded fills
    with dada.Hdu(k, "R") as r:
        assert [r.read_block() for _ in range(3)] == b[2:4] + [None]


def test_zero_next_write(ring):
    k = ring(2, 64)
    with dada.Hdu(k, "W") as w:
        assert L.ipcbuf_zero_next_write(w.data) == 0      # fresh ring: free at once
        w.write_block(b"\7" * 64)
        w.write_block(b"\7" * 64)
        with dada.Hdu(k, "R") as r:
            assert r.read_block() == b"\7" * 64
            assert r.read_block() == b"\7" * 64
            assert L.ipcio_zero_next_block(w.data) == 0   # block 1: cleared, so free
        nb, bs = C.c_uint64(), C.c_uint64()
        h = dada.HduStruct.from_address(w.h)
        addrs = C.cast(L.dada_hdu_db_addresses(w.h, C.byref(nb), C.byref(bs)), C.POINTER(C.c_void_p))
        assert (nb.value, bs.value) == (2, 64) and h.data_block
        assert C.string_at(addrs[1], 64) == b"\0" * 64
        assert C.string_at(addrs[0], 64) == b"\7" * 64


def test_next_readable_waits_like_next_read(ring):
    k = ring(2, 64)
    with dada.Hdu(k, "W") as w, dada.Hdu(k, "R") as r:
        w.write_block(b"\5" * 64)
        n = C.c_uint64()
        p = L.ipcbuf_get_next_readable(r.data, C.byref(n))
        assert p and n.value == 64 and C.string_at(p, 64) == b"\5" * 64
        assert L.ipcbuf_mark_cleared(r.data) == 0


# ---- ipcio_create / destroy, ipc helpers -------------------------------------------------

def test_ipcio_create_and_destroy():
    k = fresh_key()
    io = C.create_string_buffer(152)
    assert L.ipcio_create(io, k, 3, 128, 1) == 0
    other = C.create_string_buffer(152)
    assert L.ipcio_connect(other, k) == 0
    assert L.ipcbuf_get_nbufs(other) == 3
    L.ipcio_disconnect(other)
    assert L.ipcio_destroy(io) == 0
    assert L.ipcio_connect(other, k) == -1


def test_ipc_alloc_and_semop():
    k = fresh_key() + 0x900000
    sid = C.c_int(-1)
    p = L.ipc_alloc(k, 4096, IPC_CREAT | 0o600, C.byref(sid))
    assert p and sid.value >= 0
    C.memmove(p, b"abc", 3)
    assert C.string_at(p, 3) == b"abc"
    libc.shmdt(p)
    libc.shmctl(sid.value, IPC_RMID, None)
    sem = libc.semget(k, 1, IPC_CREAT | 0o600)
    assert sem >= 0
    assert L.ipc_semop(sem, 0, 2, 0) == 0
    assert L.ipc_semop(sem, 0, -3, 0o4000) == -1          # IPC_NOWAIT: would block
    assert L.ipc_semop(sem, 0, -2, 0) == 0
    libc.semctl(sem, 0, IPC_RMID)


# ---- ascii header, multilog ------------------------------------------------------------

def test_ascii_header_find():
    hdr = b"HDR_SIZE 4096\nNCHAN    256\nOBS_NCHAN 336\n"
    base = C.cast(C.c_char_p(hdr), P).value
    buf = C.create_string_buffer(hdr)
    at = L.ascii_header_find(buf, b"NCHAN")
    assert at - C.addressof(buf) == hdr.index(b"NCHAN    256")
    assert L.ascii_header_find(buf, b"HDR_SIZE") == C.addressof(buf)
    assert L.ascii_header_find(buf, b"CHAN") is None        # only inside other keys
    assert L.ascii_header_find(buf, b"NBIT") is None
    del base


def test_ascii_header_get_size(tmp_path):
    f = tmp_path / "a.dada"
    dada.write_dada_file(str(f), "HDR_SIZE 8192\nNCHAN 4\n", np.zeros(16384, np.uint8))
    assert L.ascii_header_get_size(str(f).encode()) == 8192
    fd = os.open(str(f), os.O_RDONLY)
    os.lseek(fd, 100, 0)
    assert L.ascii_header_get_size_fd(fd) == 8192
    assert os.lseek(fd, 0, 1) == 0                          # offset put back to 0
    os.close(fd)
    assert L.ascii_header_get_size(str(tmp_path / "none").encode()) == 2 ** 64 - 1


def test_multilog_fprintf_line(tmp_path):
    path = tmp_path / "log.txt"
    fp = libc.fopen(str(path).encode(), b"w")
    assert L.multilog_fprintf(fp, 3, b"%s", b"boom") == 0   # LOG_ERR
    assert L.multilog_fprintf(fp, 4, b"%s", b"careful\n") == 0  # LOG_WARNING
    assert L.multilog_fprintf(fp, 6, b"%s", b"fine") == 0   # LOG_INFO
    libc.fclose(fp)
    lines = path.read_text().splitlines()
    ts = r"^\[\d{4}-\d\d-\d\d-\d\d:\d\d:\d\d\] "
    assert re.match(ts + r"ERR: boom$", lines[0])
    assert re.match(ts + r"WARN: careful$", lines[1])
    assert re.match(ts + r"fine$", lines[2])


def test_writer_thread_and_viewer_thread(ring):
    """a viewer in another thread waiting (0.1 s polls) for the writer's next
    block gets it as soon as it is marked filled"""
    k = ring(4, 64)
    b = blocks(2, 64, seed=8)
    got = []
    with dada.Hdu(k, "W") as w:
        w.write_block(b[0])
        with dada.Hdu(k, "r") as v:
            assert v.read_block() == b[0]
            t = threading.Thread(target=lambda: got.append(v.read_block()))
            t.start()
            w.write_block(b[1])
            t.join(timeout=10)
            assert not t.is_alive() and got == [b[1]]
