"""DADA layer (CPU): ASCII headers, SysV rings, the diskdb / dbdisk / dada_db
executables, and the configs[0] plumbing (diskdb file -> ring -> CPU path).

The ring contract follows PSRDADA as the reference uses it (SURVEY.md 3.1,
3.2, Appendix A): header ring at key+1, one writer, N readers each seeing
every block, a short block ends the transfer.
"""
import os
import subprocess
import threading
import time

import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
from conftest import REPO
from paf_b2p import dada

BIN = dada.BIN_DIR
TEMPLATE = """HEADER       DADA                # Distributed aquisition and data analysis
HDR_VERSION  1.0                 # Version of this ASCII header
HDR_SIZE     4096                # Size of the header in bytes
UTC_START    2018-11-05-00:00:00 # yyyy-mm-dd-hh:mm:ss
OBS_OFFSET   0                   # bytes offset from the start MJD/UTC
TELESCOPE    Effelsberg       # telescope name
TSAMP        88473.6               # sampling interval in microseconds
NBIT         32                      # number of bits per sample, here record float
NDIM         1                   # dimension of samples (2=complex, 1=real)
NPOL         1                   # number of polarizations observed
NCHAN        336                    # number of channels here
"""

_key_lock = threading.Lock()
_key_base = 0x1000 + (os.getpid() % 48) * 0x100  # one window of 128 keys per test process
_next_key = [0]


def fresh_key() -> int:
    """a ring key of this process's own window (xdist workers never share
    one: destroying "leftovers" must not remove another worker's live ring)"""
    with _key_lock:
        k = _key_base + 2 * (_next_key[0] % 128)
        _next_key[0] += 1
    dada.destroy_ring(k)  # leftovers of an aborted run
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


# ---- ASCII header (capture.c:758-778 usage) ---------------------------------------

def test_header_get_values():
    assert dada.header_get(TEMPLATE, "NCHAN", "%d") == 336
    assert dada.header_get(TEMPLATE, "TSAMP", "%lf") == 88473.6
    assert dada.header_get(TEMPLATE, "TELESCOPE") == "Effelsberg"
    assert dada.header_get(TEMPLATE, "NOPE") is None
    # whole-word, line-start match only
    assert dada.header_get("XNCHAN 5\nNCHAN 7\n", "NCHAN", "%d") == 7
    assert dada.header_get("NCHANX 5\n", "NCHAN", "%d") is None


def test_header_set_replaces_keeps_comment_and_appends():
    h = dada.header_set(TEMPLATE, "NCHAN", 1024)
    assert dada.header_get(h, "NCHAN", "%d") == 1024
    line = [ln for ln in h.decode().splitlines() if ln.startswith("NCHAN")][0]
    assert "# number of channels here" in line
    h2 = dada.header_set(h, "FREQ", "1340.5")
    assert dada.header_get(h2, "FREQ", "%lf") == 1340.5
    assert h2.decode().count("\n") == h.decode().count("\n") + 1
    h3 = dada.header_del(h2, "FREQ")
    assert dada.header_get(h3, "FREQ") is None
    # every other key untouched
    for k in ("HEADER", "TSAMP", "UTC_START", "NBIT"):
        assert dada.header_get(h3, k) == dada.header_get(TEMPLATE, k)


def test_reference_template_parses():
    path = os.path.join(REPO, "paf-baseband2power_amd", "conf", "header_baseband2power.txt")
    text = open(path).read()
    assert dada.header_get(text, "NCHAN", "%d") == 336
    assert dada.header_get(text, "NBIT", "%d") == 32
    assert dada.header_get(text, "HDR_SIZE", "%d") == 4096


# ---- rings -----------------------------------------------------------------------------

def test_ring_roundtrip_and_short_block_eod(ring):
    k = ring(3, 4096)
    rng = np.random.default_rng(1)
    blocks = [rng.integers(0, 256, 4096, dtype=np.uint8).tobytes() for _ in range(7)] + [b"x" * 100]
    got = []

    def reader():
        with dada.Hdu(k, "R") as r:
            got.append(r.read_header())
            while True:
                b = r.read_block()
                if b is None:
                    break
                got.append(b)

    t = threading.Thread(target=reader)
    t.start()
    with dada.Hdu(k, "W") as w:
        w.write_header(TEMPLATE)
        for b in blocks:  # 8 blocks through a 3-block ring: flow control
            w.write_block(b)
    t.join(30)
    assert not t.is_alive()
    assert got[0].decode() == TEMPLATE
    assert got[1:] == blocks


def test_ring_zero_copy_view(ring):
    """view_block / release_block: the reader sees each block in place"""
    k = ring(2, 4096)
    blocks = [bytes([i]) * 4096 for i in range(5)] + [b"y" * 10]
    got = []

    def reader():
        with dada.Hdu(k, "R") as r:
            r.read_header()
            while (v := r.view_block()) is not None:
                got.append(v.tobytes())
                r.release_block(len(v))

    t = threading.Thread(target=reader)
    t.start()
    with dada.Hdu(k, "W") as w:
        w.write_header(TEMPLATE)
        for b in blocks:
            w.write_block(b)
    t.join(30)
    assert not t.is_alive()
    assert got == blocks


def test_ring_full_last_block_then_empty_eod(ring):
    k = ring(2, 1024)
    out = []

    def reader():
        with dada.Hdu(k, "R") as r:
            r.read_header()
            while (b := r.read_block()) is not None:
                out.append(len(b))
            out.append("eod" if r.eod() else "no-eod")

    t = threading.Thread(target=reader)
    t.start()
    with dada.Hdu(k, "W") as w:
        w.write_header("HDR 1\n")
        for _ in range(3):
            w.write_block(b"\1" * 1024)
    # unlock_write (close) ends the transfer with an empty block
    t.join(30)
    assert out == [1024, 1024, 1024, "eod"]


def test_ring_carries_several_transfers(ring):
    """End of data is kept per transfer (e_buf / e_byte / eod of transfer
    x % 8, PSRDADA): a second transfer on the same ring is read in
    full after the first one's EOD, and a reader that is behind stops at the
    first transfer's (empty or short) EOD block instead of reading it as data
    (PSRDADA rings carry one transfer after another)"""
    k = ring(12, 1024)                   # 9 blocks in all: no reader runs meanwhile
    with dada.Hdu(k, "W") as w:          # transfer 1 ends with a short block
        w.write_header("XFER 1\n")
        for i in range(3):
            w.write_block(bytes([i]) * 1024)
        w.write_block(b"a" * 10)
    with dada.Hdu(k, "W") as w:          # transfer 2: unlock_write ends it (empty block)
        w.write_header("XFER 2\n")
        for i in range(2):
            w.write_block(bytes([10 + i]) * 1024)
    with dada.Hdu(k, "W") as w:          # transfer 3: full blocks then a 0-byte EOD
        w.write_header("XFER 3\n")
        w.write_block(b"z" * 1024)
    got = []
    for _ in range(3):                   # the reader was behind all three
        with dada.Hdu(k, "R") as r:
            h = r.read_header().split(b"\n")[0]
            blocks = []
            while (b := r.read_block()) is not None:
                blocks.append(b)
            got.append((h, [len(b) for b in blocks], [b[0] for b in blocks], r.eod()))
    assert got == [(b"XFER 1", [1024, 1024, 1024, 10], [0, 1, 2, 97], True),
                   (b"XFER 2", [1024, 1024], [10, 11], True),
                   (b"XFER 3", [1024], [122], True)]


def test_two_readers_each_see_every_block(ring):
    k = ring(2, 512, nreaders=2)
    res = {0: [], 1: []}

    def reader(i):
        with dada.Hdu(k, "R") as r:
            r.read_header()
            while (b := r.read_block()) is not None:
                res[i].append(b[0])

    ts = [threading.Thread(target=reader, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    with dada.Hdu(k, "W") as w:
        w.write_header("HDR 1\n")
        for i in range(9):
            w.write_block(bytes([i]) * 512)
    for t in ts:
        t.join(30)
    assert res[0] == list(range(9)) and res[1] == list(range(9))


def test_single_writer_lock(ring):
    """one writer at a time: a second lock_write waits for the first writer's
    unlock (PSRDADA's WRITE semaphore, ipcbuf_lock_write @0x403b00)"""
    k = ring(2, 512)
    events = []
    w1 = dada.Hdu(k, "W")

    def second():
        with dada.Hdu(k, "W"):
            events.append("second locked")

    t = threading.Thread(target=second)
    t.start()
    t.join(0.5)
    assert t.is_alive() and not events  # waiting on the lock
    events.append("first unlocks")
    w1.close()
    t.join(30)
    assert not t.is_alive()
    assert events == ["first unlocks", "second locked"]


def test_connect_missing_ring_fails():
    k = fresh_key()
    with pytest.raises(OSError):
        dada.Hdu(k, "R")


def test_dada_db_tool_create_destroy():
    k = fresh_key()
    r = subprocess.run([f"{BIN}/dada_db", "-k", f"{k:x}", "-b", "8192", "-n", "4", "-r", "1",
                        "-l", "-p"], capture_output=True, text=True)
    if r.returncode != 0:  # -l needs CAP_IPC_LOCK or RLIMIT_MEMLOCK room: refused cleanly
        assert "cannot lock the ring in RAM" in r.stderr
        with pytest.raises(OSError):
            dada.Hdu(k, "W")
        r = subprocess.run([f"{BIN}/dada_db", "-k", f"{k:x}", "-b", "8192", "-n", "4", "-r", "1", "-p"],
                           capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    with dada.Hdu(k, "W") as w:
        assert w.bufsz == 8192
    assert subprocess.run([f"{BIN}/dada_db", "-k", f"{k:x}", "-d"]).returncode == 0
    assert subprocess.run([f"{BIN}/dada_db", "-k", f"{k:x}", "-d"],
                          capture_output=True).returncode != 0


# ---- executables: diskdb -> ring -> dbdisk (byte-exact) -------------------------------

def run_diskdb(key, path, hdr_path, sod=1, threads=None):
    return subprocess.Popen([f"{BIN}/paf_diskdb", "-a", f"{key:x}", "-b", os.path.dirname(path),
                             "-c", os.path.basename(path), "-d", hdr_path, "-e", str(sod)]
                            + ([] if threads is None else ["-T", str(threads)]),
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE)


@pytest.mark.parametrize("payload_blocks", [3.0, 2.5])
def test_diskdb_to_dbdisk_bytes(tmp_path, ring, payload_blocks):
    bufsz = 64 * 1024
    k = ring(4, bufsz)
    payload = np.random.default_rng(3).integers(0, 256, int(bufsz * payload_blocks),
                                                dtype=np.uint8)
    src = tmp_path / "obs.dada"
    dada.write_dada_file(str(src), "FILE_HEADER_IS_SKIPPED 1\n", payload)
    hdr = tmp_path / "header.txt"
    hdr.write_text(TEMPLATE)
    out = tmp_path / "out.dada"
    sink = subprocess.Popen([f"{BIN}/paf_dbdisk", "-k", f"{k:x}", "-o", str(out), "-W"],
                            stderr=subprocess.PIPE)
    src_p = run_diskdb(k, str(src), str(hdr))
    assert src_p.wait(60) == 0, src_p.stderr.read()
    assert sink.wait(60) == 0, sink.stderr.read()
    h, data = dada.read_dada_file(str(out))
    assert h.decode() == TEMPLATE                # diskdb.cu:79-93: the template header
    assert np.array_equal(data, payload)         # diskdb.cu:69,103-121: payload only


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("payload_blocks", [2.0, 2.37, 0.4, 0.0])
def test_diskdb_parallel_readers_same_bytes(tmp_path, ring, threads, payload_blocks):
    """-T N: each block is read as N contiguous slices in parallel (2 MiB
    pieces); the ring sees the same blocks as one fread per block gives --
    whole blocks, then the short (or empty) one that ends the transfer"""
    bufsz = (5 << 20) + 4096  # not a whole number of 2 MiB pieces
    k = ring(3, bufsz)
    payload = np.random.default_rng(int(payload_blocks * 100) + threads).integers(
        0, 256, int(bufsz * payload_blocks), dtype=np.uint8)
    src = tmp_path / "obs.dada"
    dada.write_dada_file(str(src), "FILE_HEADER_IS_SKIPPED 1\n", payload)
    hdr = tmp_path / "header.txt"
    hdr.write_text(TEMPLATE)
    seen = []

    def consumer():
        with dada.Hdu(k, "R") as r:
            r.read_header()
            while (b := r.read_block()) is not None:
                seen.append(bytes(b))

    t = threading.Thread(target=consumer)
    t.start()
    p = run_diskdb(k, str(src), str(hdr), threads=threads)
    assert p.wait(60) == 0, p.stderr.read()
    t.join(60)
    nfull = len(payload) // bufsz
    assert [len(b) for b in seen[:nfull]] == [bufsz] * nfull
    assert b"".join(seen) == payload.tobytes()
    assert f"{threads} reader" in p.stderr.read().decode()


def test_diskdb_reads_a_fifo_and_a_growing_file_to_their_end(tmp_path, ring):
    """the payload is read until end of file, not up to a size taken when the
    file was opened (advisor, round 4): a FIFO (no size, no pread) is read
    in order, and a file that grows after paf_diskdb opened it is read to
    its final end -- as the reference's fread loop did (diskdb.cu:103-121)"""
    bufsz = 1 << 16
    hdr = tmp_path / "header.txt"
    hdr.write_text(TEMPLATE)
    payload = np.random.default_rng(7).integers(0, 256, 5 * bufsz + 1234, dtype=np.uint8)
    whole = tmp_path / "whole.dada"
    dada.write_dada_file(str(whole), "FILE_HEADER_IS_SKIPPED 1\n", payload)
    blob = whole.read_bytes()

    def consume(k, seen):
        with dada.Hdu(k, "R") as r:
            r.read_header()
            while (b := r.read_block()) is not None:
                seen.append(bytes(b))

    # 1. a FIFO, written in odd pieces by another thread
    k = ring(3, bufsz)
    fifo = tmp_path / "obs.fifo"
    os.mkfifo(fifo)
    seen = []
    t = threading.Thread(target=consume, args=(k, seen))
    t.start()

    def feed():
        with open(fifo, "wb") as f:
            for i in range(0, len(blob), 9999):
                f.write(blob[i:i + 9999])
    w = threading.Thread(target=feed)
    w.start()
    p = run_diskdb(k, str(fifo), str(hdr), threads=4)
    assert p.wait(60) == 0, p.stderr.read()
    w.join(60)
    t.join(60)
    assert b"".join(seen) == payload.tobytes()
    assert [len(b) for b in seen[:5]] == [bufsz] * 5
    # 2. a file that grows after it was opened: paf_diskdb waits on a full
    #    ring (no reader yet) while the rest of the payload is appended
    k2 = ring(2, bufsz)
    grow = tmp_path / "grow.dada"
    grow.write_bytes(blob[: 4096 + 2 * bufsz + 100])  # header + two blocks (fill the ring) + a bit
    p = run_diskdb(k2, str(grow), str(hdr), threads=2)
    time.sleep(0.5)                                    # both blocks written, waiting for a third
    with open(grow, "ab") as f:
        f.write(blob[4096 + 2 * bufsz + 100:])
    seen2 = []
    consume(k2, seen2)
    assert p.wait(60) == 0, p.stderr.read()
    assert b"".join(seen2) == payload.tobytes()


def test_diskdb_stops_cleanly_on_sigterm(tmp_path, ring):
    """SIGTERM while paf_diskdb waits on its input (a FIFO that has delivered
    a block and a half): the whole block goes out, the half block is dropped
    -- the end of data takes its place -- the transfer ends and paf_diskdb
    exits 0, so the reader downstream finishes normally"""
    import signal
    bufsz = 1 << 16
    hdr = tmp_path / "header.txt"
    hdr.write_text(TEMPLATE)
    payload = np.random.default_rng(11).integers(0, 256, 3 * bufsz, dtype=np.uint8)
    whole = tmp_path / "whole.dada"
    dada.write_dada_file(str(whole), "FILE_HEADER_IS_SKIPPED 1\n", payload)
    blob = whole.read_bytes()
    k = ring(4, bufsz)
    fifo = tmp_path / "obs.fifo"
    os.mkfifo(fifo)
    out = tmp_path / "out.dada"
    sink = subprocess.Popen([f"{BIN}/paf_dbdisk", "-k", f"{k:x}", "-o", str(out)], stderr=subprocess.PIPE)
    p = run_diskdb(k, str(fifo), str(hdr), threads=2)
    f = open(fifo, "wb")
    try:
        f.write(blob[: 4096 + bufsz + bufsz // 2])
        f.flush()
        t_end = time.time() + 30
        while (not out.exists() or out.stat().st_size < 4096 + bufsz) and time.time() < t_end:
            time.sleep(0.02)
        time.sleep(0.2)  # the half block read, paf_diskdb waiting for the rest
        assert p.poll() is None
        p.send_signal(signal.SIGTERM)
        assert p.wait(30) == 0, p.stderr.read()
        assert sink.wait(30) == 0, sink.stderr.read()
    finally:
        f.close()
        for q in (p, sink):
            if q.poll() is None:
                q.kill()
                q.wait()
    assert b"stopped by a signal after 1 blocks" in p.stderr.read()
    _, data = dada.read_dada_file(str(out))
    assert data.tobytes() == payload[:bufsz].tobytes()


def test_dbdisk_stops_cleanly_on_sigterm(tmp_path, ring):
    """SIGTERM while paf_dbdisk waits for the next block (the writer idle,
    its transfer open): the wait gives up, the file keeps every block so
    far, paf_dbdisk exits 0"""
    import signal
    k = ring(4, 1344)
    out = tmp_path / "power.dada"
    sink = subprocess.Popen([f"{BIN}/paf_dbdisk", "-k", f"{k:x}", "-o", str(out)], stderr=subprocess.PIPE)
    try:
        with dada.Hdu(k, "W") as w:
            w.write_header(TEMPLATE)
            for n in (1, 2):
                w.write_block(bytes([n]) * 1344)
            t_end = time.time() + 10
            while (not out.exists() or out.stat().st_size < 4096 + 2 * 1344) and time.time() < t_end:
                time.sleep(0.01)
            sink.send_signal(signal.SIGTERM)
            assert sink.wait(10) == 0, sink.stderr.read()
    finally:
        if sink.poll() is None:
            sink.kill()
            sink.wait()
    assert b"stopped by a signal after 2 blocks" in sink.stderr.read()
    assert dada.read_dada_file(str(out))[1].tobytes() == b"\1" * 1344 + b"\2" * 1344


def test_diskdb_rejects_bad_thread_count(tmp_path):
    r = subprocess.run([f"{BIN}/paf_diskdb", "-a", "dada", "-c", "x", "-d", "y", "-T", "0"],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "-T takes 1..64" in r.stderr


def test_dbdisk_default_file_name(tmp_path, ring):
    k = ring(2, 1024)
    sink = subprocess.Popen([f"{BIN}/paf_dbdisk", "-k", f"{k:x}", "-D", str(tmp_path)])
    with dada.Hdu(k, "W") as w:
        w.write_header(TEMPLATE)
        w.write_block(b"\7" * 1024)
    assert sink.wait(30) == 0
    assert os.listdir(tmp_path) == ["2018-11-05-00:00:00_0000000000000000.000000.dada"]


def test_dbdisk_writes_each_block_as_it_leaves_the_ring(tmp_path, ring):
    """a spectrum is in the file once paf_dbdisk has taken it from the ring,
    while the transfer is still open (as dada_dbdisk writes: no stdio buffer
    holding small blocks back until it fills or the transfer ends)"""
    k = ring(4, 1344)  # one 336-channel fp32 spectrum per block (header_baseband2power.txt:42)
    out = tmp_path / "power.dada"
    sink = subprocess.Popen([f"{BIN}/paf_dbdisk", "-k", f"{k:x}", "-o", str(out)], stderr=subprocess.PIPE)
    try:
        with dada.Hdu(k, "W") as w:
            w.write_header(TEMPLATE)
            for n in (1, 2):
                w.write_block(bytes([n]) * 1344)
                t_end = time.time() + 10
                while (not out.exists() or out.stat().st_size < 4096 + n * 1344) and time.time() < t_end:
                    time.sleep(0.01)
                assert out.stat().st_size == 4096 + n * 1344
        assert sink.wait(30) == 0, sink.stderr.read()
    finally:
        if sink.poll() is None:
            sink.kill()
            sink.wait()
    _, data = dada.read_dada_file(str(out))
    assert data.tobytes() == b"\1" * 1344 + b"\2" * 1344


# ---- configs[0]: 256 ch x 2 pol, 1024x1024 integrate from a diskdb file, CPU path ---

def test_config1_diskdb_plumbing_cpu(tmp_path, ring):
    """paf_diskdb feeds one full 1 GiB integration through a ring; a CPU
    consumer (the oracle, as the reference has no CPU path) integrates every
    block it receives; the spectrum equals the oracle run on the file."""
    g = npo.Geom(nbit=8, nchan_chunk=256)  # configs[0]: 256 x 2 pol, 1<<20 samples
    nblk = 4
    bufsz = g.block_bytes // nblk
    k = ring(3, bufsz)
    payload = co.fill_synthetic(g, g.block_bytes, 20181105, 0, 0)
    src = tmp_path / "c1.dada"
    dada.write_dada_file(str(src), "NBIT 8\nNCHAN 256\n", payload)
    hdr = tmp_path / "hdr.txt"
    hdr.write_text(TEMPLATE)
    acc = np.zeros(g.nout, dtype=np.uint64)
    seen = []

    def consumer():
        with dada.Hdu(k, "R") as r:
            r.read_header()
            while (b := r.read_block()) is not None:
                seen.append(len(b))
                co.integrate(g, np.frombuffer(b, dtype=np.uint8), nthreads=4, acc=acc)

    t = threading.Thread(target=consumer)
    t.start()
    p = run_diskdb(k, str(src), str(hdr))
    assert p.wait(300) == 0
    t.join(300)
    assert seen == [bufsz] * nblk
    direct = co.power(g, payload, nthreads=8)
    assert np.array_equal(co.finalize(g, acc).view(np.uint32), direct.view(np.uint32))
    del payload


def test_paf_baseband2power_cli_help_and_no_gpu(tmp_path, have_gpu):
    exe = f"{BIN}/paf_baseband2power"
    r = subprocess.run([exe, "-h"], capture_output=True, text=True)
    assert r.returncode == 1 and "-a  Hexacdecimal shared memory key" in r.stdout
    r = subprocess.run([exe, "-a", "zz", "-b", "adad"], capture_output=True, text=True)
    assert r.returncode == 1 and "Could not parse key" in r.stderr
    if have_gpu:
        return
    r = subprocess.run([exe, "-a", "dada", "-b", "adad", "-c", str(tmp_path), "-d", "0"],
                       capture_output=True, text=True)
    assert r.returncode == 1
    log = (tmp_path / "paf_baseband2power.log").read_text()
    assert "START PAF_PROCESS" in log and "no HIP device" in log


def test_device_ring_without_gpu_fails_cleanly(tmp_path, have_gpu):
    # dada_db -g: the holder cannot get a device here, so creation fails,
    # says why, and leaves no segment behind
    if have_gpu:
        pytest.skip("a GPU is present")
    key = fresh_key()
    r = subprocess.run([os.path.join(BIN, "dada_db"), "-k", f"{key:x}", "-b", "4096", "-n", "2",
                        "-g", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "holder failed" in r.stderr
    with pytest.raises(OSError):
        dada.Hdu(key, "R")
    assert not dada.destroy_ring(key)


def test_host_ring_reports_no_device(ring):
    key = ring(2, 4096)
    with dada.Hdu(key, "W") as w:
        assert w.device == -1


def test_dfdb_refuses_host_ring_for_assembly(tmp_path, ring):
    # frame assembly writes device memory: paf_dfdb needs a dada_db -g ring
    key = ring(2, 48 * 7168)
    (tmp_path / "s.df").write_bytes(b"")
    (tmp_path / "s.chunks").write_bytes(b"")
    hdr = tmp_path / "h.txt"
    hdr.write_text("HDR_SIZE 4096\n")
    r = subprocess.run([os.path.join(BIN, "paf_dfdb"), "-a", f"{key:x}", "-b", str(hdr), "-c",
                        str(tmp_path / "s.df"), "-k", str(tmp_path / "s.chunks")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "not GPU-resident" in r.stderr


@pytest.mark.parametrize("short_last", [True, False])
def test_reader_read_depth_two(ring, short_last):
    # extension: a reader holds two blocks; releases go oldest first, the ring
    # keeps every block until it is released, and EOD (short block, or the
    # empty block of unlock_write) still ends the transfer
    key = ring(3, 4096)
    blocks = [bytes([i]) * 4096 for i in range(6)] + ([b"\x07" * 100] if short_last else [])
    got, held_max = [], [0]

    def reader():
        with dada.Hdu(key, "R") as r:
            r.read_header()
            r.set_read_depth(2)
            held = []
            while (b := r.open_block()) is not None:
                held.append(b)
                held_max[0] = max(held_max[0], len(held))
                if len(held) == 2:
                    got.append(held.pop(0))
                    r.close_block()
            while held:
                got.append(held.pop(0))
                r.close_block()

    t = threading.Thread(target=reader)
    t.start()
    with dada.Hdu(key, "W") as w:
        w.write_header("HDR_SIZE 4096\n")
        for b in blocks:
            w.write_block(b)
    t.join(60)
    assert not t.is_alive()
    assert got == blocks and held_max[0] == 2


def test_ring_transfers_property(ring):
    """Random transfers through a small ring with a concurrent reader: each
    transfer's blocks arrive in order and unchanged, its end is a short,
    empty or (at unlock_write) appended empty block, and the next transfer
    follows after unlock_read + lock_read (end of data per transfer: e_buf / e_byte)"""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    transfer = st.tuples(st.integers(0, 5), st.sampled_from(["full", "short", "empty"]),
                         st.integers(1, 511))

    @settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
    @given(xfers=st.lists(transfer, min_size=1, max_size=3), nbufs=st.integers(2, 4),
           seed=st.integers(0, 1 << 30))
    def check(xfers, nbufs, seed):
        bufsz = 512
        k = ring(nbufs, bufsz)
        rng = np.random.default_rng(seed)
        want = []
        for nfull, end, short in xfers:
            blocks = [rng.integers(0, 256, bufsz, dtype=np.uint8).tobytes() for _ in range(nfull)]
            if end == "short":
                blocks.append(rng.integers(0, 256, short, dtype=np.uint8).tobytes())
            want.append(blocks)
        got = []

        def reader():
            for t in range(len(xfers)):
                with dada.Hdu(k, "R") as r:
                    h = r.read_header()
                    blocks = []
                    while (b := r.read_block()) is not None:
                        blocks.append(b)
                    got.append((int(h.split()[1]), blocks, r.eod()))

        th = threading.Thread(target=reader)
        th.start()
        for t, (blocks, (nfull, end, short)) in enumerate(zip(want, xfers)):
            with dada.Hdu(k, "W") as w:
                w.write_header(f"XFER {t}\n")
                for b in blocks:
                    w.write_block(b)
                if end == "empty":
                    w.write_block(b"")          # an explicit 0-byte EOD block
        th.join(60)
        assert not th.is_alive()
        assert [g[0] for g in got] == list(range(len(xfers)))
        for (_, blocks, eod), exp in zip(got, want):
            assert blocks == exp and eod
        dada.destroy_ring(k)

    check()


def test_dbdisk_overwrites_only_with_W(tmp_path, ring):
    """as dada_dbdisk: an existing output file is an error unless -W is given"""
    out = tmp_path / "o.dada"
    out.write_bytes(b"old")
    for flags, want_rc in (([], 1), (["-W", "-b", "0"], 0)):
        k = ring(2, 1024)
        sink = subprocess.Popen([f"{BIN}/paf_dbdisk", "-k", f"{k:x}", "-o", str(out)] + flags,
                                stderr=subprocess.PIPE, text=True)
        if want_rc == 0:
            with dada.Hdu(k, "W") as w:
                w.write_header(TEMPLATE)
                w.write_block(b"\5" * 1024)
        rc = sink.wait(30)
        err = sink.stderr.read()
        assert rc == want_rc, err
        if want_rc:
            assert "-W overwrites" in err and out.read_bytes() == b"old"
    h, data = dada.read_dada_file(str(out))
    assert h.decode() == TEMPLATE and data.tobytes() == b"\5" * 1024


def test_ascii_header_matches_a_dict_model():
    """ascii_header_set / _get / _del against a dict: random sequences of
    sets (new keys appended, existing keys replaced in place), deletes and
    lookups of keys that share prefixes and suffixes with each other"""
    from hypothesis import given, settings, strategies as st
    keys = st.sampled_from(["NCHAN", "NCHAN_CHUNK", "XNCHAN", "NCH", "FREQ", "UTC_START", "A", "AB", "B_A"])
    vals = st.one_of(st.integers(-10 ** 6, 10 ** 9).map(str),
                     st.text(alphabet="abcdefXYZ0123456789.-:_", min_size=1, max_size=24))
    ops = st.lists(st.tuples(st.sampled_from(["set", "del", "get"]), keys, vals), max_size=40)

    @settings(max_examples=200, deadline=None, derandomize=True)
    @given(ops)
    def run(seq):
        model = {}
        h = b"HDR_SIZE 4096\n"
        for op, k, v in seq:
            if op == "set":
                h = dada.header_set(h, k, v)
                model[k] = v
            elif op == "del":
                h = dada.header_del(h, k)
                model.pop(k, None)
            assert dada.header_get(h, k) == model.get(k), (op, k, h)
        for k in ("NCHAN", "NCHAN_CHUNK", "XNCHAN", "NCH", "FREQ", "UTC_START", "A", "AB", "B_A"):
            assert dada.header_get(h, k) == model.get(k), (k, h)
        assert dada.header_get(h, "HDR_SIZE", "%d") == 4096
    run()


def test_device_error_is_empty_until_a_device_ring_call_fails():
    # dada_device_error: per thread, "" until a device-ring call fails (host
    # rings never set it); the Python OSErrors carry it (paf_b2p.dada)
    import threading
    assert isinstance(dada.device_error(), str)
    got = []
    t = threading.Thread(target=lambda: got.append(dada.device_error()))
    t.start()
    t.join()
    assert got == [""]
