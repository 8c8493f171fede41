"""libpafdada against the reference's own libpsrdada (CPU).

tests/golden/psrdada_abi.json holds what tools/psrdada_dwarf.py read out of
the libpsrdada the reference links statically into its executables: struct
layouts and prototypes (DWARF) and the ring protocol (disassembly).  These
tests pin to it

  * include/b2p_dada.h (struct layouts and prototypes of every PSRDADA
    function libpafdada exports), and the PSRDADA stand-in headers the hosts'
    -DB2P_PSRDADA build is compile-checked against (tests/c/psrdada_api);
  * the shared state of a libpafdada ring: sync segment fields, key
    schedule, semaphore sets and their values, block segments;
  * the protocol, by running libpafdada's executables against
    tests/psrdada_model.py -- an independent Python statement of the same
    libpsrdada code -- in both directions (model writer -> paf_dbdisk,
    paf_diskdb -> model reader), byte for byte and state for state.
"""
import json
import os
import re
import subprocess
import threading

import numpy as np
import pytest

import psrdada_model as pm
from conftest import REPO
from paf_b2p import dada

ABI = json.load(open(os.path.join(REPO, "tests", "golden", "psrdada_abi.json")))
INCLUDE = os.path.join(REPO, "include")
STANDINS = os.path.join(REPO, "tests", "c", "psrdada_api")
BIN = dada.BIN_DIR
_key_base = 0x4000 + (os.getpid() % 48) * 0x100
_n = [0]


def fresh_key():
    k = _key_base + 2 * (_n[0] % 128)
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


def test_fixture_is_current():
    """the committed fixture is what tools/psrdada_dwarf.py reads from the
    reference today (only where /root/reference exists; never on the GPU box)"""
    if not os.path.isdir("/root/reference"):
        pytest.skip("no /root/reference here")
    r = subprocess.run(["python3", os.path.join(REPO, "tools", "psrdada_dwarf.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


# ---- struct layouts ------------------------------------------------------------------

def _layout_probe(tmp_path, includes, prelude, structs):
    lines = [prelude, "#include <stdio.h>", "#include <stddef.h>", "int main(void) {"]
    for cname, key in structs:
        lines.append(f'printf("{key} size %zu\\n", sizeof({cname}));')
        for m in ABI["structs"][key]["members"]:
            lines.append(f'printf("{key} {m["name"]} %zu %zu\\n", offsetof({cname}, {m["name"]}), '
                         f'sizeof((({cname} *)0)->{m["name"]}));')
    lines += ["return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    cmd = ["gcc", "-std=gnu11", "-D_GNU_SOURCE", str(src), "-o", str(exe)]
    for i in includes:
        cmd += ["-I", i]
    subprocess.run(cmd, check=True)
    got = {}
    for ln in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        p = ln.split()
        got[(p[0], p[1])] = tuple(int(x) for x in p[2:])
    return got


def _expected(structs):
    want = {}
    for _, key in structs:
        want[(key, "size")] = (ABI["structs"][key]["size"],)
        for m in ABI["structs"][key]["members"]:
            want[(key, m["name"])] = (m["offset"], m["size"])
    return want


def test_libpafdada_struct_layouts_match_dwarf(tmp_path):
    """ipcbuf_t, ipcio_t, dada_hdu_t of include/b2p_dada.h and the shared
    ipcsync_t are libpsrdada's, member for member"""
    structs = [("ipcbuf_t", "ipcbuf_t"), ("ipcio_t", "ipcio_t"), ("dada_hdu_t", "dada_hdu_t"),
               ("struct ipcsync", "ipcsync_t")]
    got = _layout_probe(tmp_path, [INCLUDE, os.path.join(REPO, "paf-baseband2power_amd", "csrc", "dada")],
                        '#include "dada_internal.h"', structs)
    assert got == _expected(structs)


def test_standin_struct_layouts_match_dwarf(tmp_path):
    structs = [("ipcbuf_t", "ipcbuf_t"), ("ipcio_t", "ipcio_t"), ("dada_hdu_t", "dada_hdu_t")]
    got = _layout_probe(tmp_path, [STANDINS], '#include "dada_hdu.h"', structs)
    assert got == _expected(structs)


# ---- prototypes ----------------------------------------------------------------------

_NORM = [(r"\bunsigned\b(?!\s+(int|char|long|short))", "unsigned int"), (r"\blong\b(?!\s+int)", "long int"),
         (r"\s*\*", " *"), (r"\s+", " ")]


def _norm(t: str) -> str:
    t = t.strip()
    for a, b in _NORM:
        t = re.sub(a, b, t)
    return t.replace("struct dada_hdu", "dada_hdu_t").replace("* *", "**").strip()


def _param_type(p: str) -> str:
    p = p.strip()
    if p == "...":
        return "..."
    m = re.match(r"^(.*?)(\w+)$", p)  # drop the parameter name
    t = m.group(1) if m and m.group(1).strip() else p
    return _norm(t)


def declarations(path: str):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"^\s*#.*$", " ", text, flags=re.M)  # preprocessor lines
    text = re.sub(r"__attribute__\s*\(\((?:[^()]|\([^()]*\))*\)\)", " ", text)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(\w+)\s*\(([^;{}()]*)\)\s*;", text):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        if name not in ABI["functions"]:
            continue
        ps = [] if params.strip() in ("", "void") else [_param_type(p) for p in params.split(",")]
        out[name] = (_norm(ret.replace("typedef", "")), ps)
    return out


def _dwarf_proto(name):
    f = ABI["functions"][name]
    return _norm(f["return"]), [_norm(p["type"]) if p["type"] != "..." else "..." for p in f["params"]]


def test_libpafdada_prototypes_match_dwarf():
    """every PSRDADA function include/b2p_dada.h declares has libpsrdada's
    return and parameter types (so hosts built against either library's
    headers call the other correctly)"""
    decl = declarations(os.path.join(INCLUDE, "b2p_dada.h"))
    assert len(decl) >= 45
    bad = {n: (d, _dwarf_proto(n)) for n, d in decl.items() if d != _dwarf_proto(n)}
    assert not bad, bad


def test_standin_prototypes_match_dwarf():
    decl = {}
    for f in os.listdir(STANDINS):
        if f.endswith(".h"):
            decl.update(declarations(os.path.join(STANDINS, f)))
    assert len(decl) >= 25
    bad = {n: (d, _dwarf_proto(n)) for n, d in decl.items() if d != _dwarf_proto(n)}
    assert not bad, bad


def test_libpafdada_exports_the_whole_psrdada_api():
    """every function of the libpsrdada the reference links (all 113 its
    debug info holds) is declared in include/b2p_dada.h and exported by
    libpafdada -- not only the subset the reference's hosts call"""
    lib = os.path.join(REPO, "paf-baseband2power_amd", "lib", "libpafdada.so")
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    have = {ln.split()[-1] for ln in out.splitlines()}
    assert len(ABI["functions"]) == 113
    assert set(ABI["functions"]) <= have, sorted(set(ABI["functions"]) - have)
    assert set(ABI["functions"]) <= decl_names(), sorted(set(ABI["functions"]) - decl_names())


def decl_names():
    return set(declarations(os.path.join(INCLUDE, "b2p_dada.h")))


# ---- shared state of a libpafdada ring ----------------------------------------------

def test_ring_wire_layout(ring):
    """sync segment, key schedule, semaphore sets and block segments of a ring
    made by libpafdada's dada_db are the ones libpsrdada makes
    (ipcbuf_create_work @0x4033b0)"""
    nbufs, bufsz, nread = 5, 8192, 2
    k = ring(nbufs, bufsz, nread)
    r = pm.Ring(k)
    try:
        s = r.s
        assert (r.nbufs, r.bufsz, r.n_readers) == (nbufs, bufsz, nread)
        assert s.get("semkey_connect") == k + 0x10000
        assert [s.get("semkey_data", i) for i in range(8)] == [k + 0x10000 * (2 + i) for i in range(8)]
        keys = [pm.C.c_int32.from_address(r.shmkey_addr + 4 * i).value for i in range(nbufs)]
        assert keys == [k + 0x10000 * (10 + i) for i in range(nbufs)]
        assert [s.get("eod", x) for x in range(8)] == [1] * 8
        assert all(s.get(f, x) == 0 for f in ("s_buf", "s_byte", "e_buf", "e_byte") for x in range(8))
        assert (s.get("w_buf"), s.get("w_xfer"), s.get("w_state"), s.get("on_device_id")) == (0, 0, 0, -1)
        assert [r.count(b) for b in range(nbufs)] == [0] * nbufs
        assert [pm.semval(r.semid_connect, i) for i in range(2)] == [1, nread]
        for d in r.semid_data:
            assert [pm.semval(d, i) for i in range(5)] == [8, 8, 0, 0, 1]  # SODACK EODACK FULL CLEAR CONN
        # the sync segment is 520 + 5*nbufs bytes; every block segment bufsz
        assert _segsz(k) == 520 + 5 * nbufs
        assert all(_segsz(kb) == bufsz for kb in keys)
        h = pm.Ring(k + 1)  # the header ring, same schedule from key + 1
        assert h.s.get("semkey_connect") == k + 1 + 0x10000 and h.bufsz == 4096
        h.close()
    finally:
        r.close()


class ShmidDs(pm.C.Structure):  # struct shmid_ds (x86-64 glibc): the size field only
    _fields_ = [("perm", pm.C.c_byte * 48), ("shm_segsz", pm.C.c_size_t), ("rest", pm.C.c_byte * 64)]


def _segsz(key):
    sid = pm._libc.shmget(key, 0, 0)
    assert sid >= 0
    ds = ShmidDs()
    pm._libc.shmctl.argtypes = [pm.C.c_int, pm.C.c_int, pm.C.c_void_p]
    assert pm._libc.shmctl(sid, pm.IPC_STAT, pm.C.byref(ds)) == 0
    return ds.shm_segsz


# ---- protocol: libpafdada executables against the model -----------------------------

TEMPLATE = "HEADER DADA\nHDR_SIZE 4096\nUTC_START 2018-11-05-00:00:00\nOBS_OFFSET 0\n"


@pytest.mark.parametrize("tail", ["short", "full"])
def test_model_writer_to_paf_dbdisk(tmp_path, ring, tail):
    """a PSRDADA writer (the model) -> paf_dbdisk (libpafdada): the file holds
    the header and every byte; a short last block, or the 0-byte block
    ipcio_close appends after a full one, ends the transfer"""
    bufsz = 4096
    k = ring(4, bufsz)
    rng = np.random.default_rng(7)
    nbytes = 6 * bufsz + (1234 if tail == "short" else 0)
    payload = rng.integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    out = tmp_path / "out.dada"
    sink = subprocess.Popen([f"{BIN}/paf_dbdisk", "-k", f"{k:x}", "-o", str(out)], stderr=subprocess.PIPE)
    hdr, data = pm.Ring(k + 1), pm.Ring(k)
    try:
        hdr.lock_write()
        data.lock_write()
        hdr.write_block(pm.header_block(hdr, TEMPLATE.encode()))
        for off in range(0, nbytes, bufsz):
            data.write_block(payload[off:off + bufsz])
        data.end_transfer()  # a no-op after a short block (the transfer already ended)
        data.unlock_write()
        hdr.unlock_write()
        assert sink.wait(60) == 0, sink.stderr.read()
    finally:
        hdr.close()
        data.close()
    h, body = dada.read_dada_file(str(out))
    assert h.decode() == TEMPLATE and body.tobytes() == payload


def test_paf_diskdb_to_model_reader(tmp_path, ring):
    """paf_diskdb (libpafdada, diskdb.cu's writer calls) -> a PSRDADA reader
    (the model): header, then every byte, then end of data; the shared
    state afterwards is what libpsrdada's code leaves"""
    bufsz = 8192
    k = ring(8, bufsz)
    payload = np.random.default_rng(8).integers(0, 256, bufsz * 5 // 2, dtype=np.uint8)
    src = tmp_path / "obs.dada"
    dada.write_dada_file(str(src), "SKIPPED 1\n", payload)
    hfile = tmp_path / "hdr.txt"
    hfile.write_text(TEMPLATE)
    p = subprocess.run([f"{BIN}/paf_diskdb", "-a", f"{k:x}", "-b", str(tmp_path), "-c", "obs.dada",
                        "-d", str(hfile), "-e", "1"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    hdr, data = pm.Ring(k + 1), pm.Ring(k)
    try:
        hdr.lock_read()
        data.lock_read()
        hp, hn = hdr.get_next_read()
        assert pm.C.string_at(hp, hn).split(b"\0")[0].decode() == TEMPLATE
        hdr.mark_cleared()
        blocks = data.read_transfer()
        assert data.state == "rstop"
        assert b"".join(blocks) == payload.tobytes() and [len(b) for b in blocks] == [bufsz, bufsz, bufsz // 2]
        s = data.s
        assert (s.get("w_buf"), s.get("w_xfer"), s.get("w_state")) == (3, 1, 0)
        assert (s.get("s_buf", 0), s.get("e_buf", 0), s.get("e_byte", 0), s.get("eod", 0)) == (0, 2, bufsz // 2, 1)
        assert (s.get("r_bufs", 0), s.get("r_xfers", 0), s.get("r_states", 0)) == (2, 1, 0)
        # every semaphore back where it started, the fills accounted in count[]
        assert [pm.semval(data.semid_data[0], i) for i in range(5)] == [8, 8, 0, 3, 0]
        assert [data.count(b) for b in range(3)] == [1, 1, 1]
        data.unlock_read()
        hdr.unlock_read()
    finally:
        hdr.close()
        data.close()


def test_transfers_alternate_between_libraries(ring):
    """transfer 1 written by libpafdada, transfer 2 by the model, transfer 3
    by libpafdada again, through a 3-block ring; one libpafdada reader takes
    all three (header + blocks each): the two writers share the ring's
    count[] / semaphores without a block lost or overwritten"""
    k = ring(3, 1024)
    rng = np.random.default_rng(9)
    want = [[rng.integers(0, 256, 1024, dtype=np.uint8).tobytes() for _ in range(n)] + [b"e" * m]
            for n, m in ((2, 100), (4, 10), (1, 1000))]
    got = []

    def reader():
        for _ in range(3):
            with dada.Hdu(k, "R") as r:
                h = r.read_header()
                blocks = []
                while (b := r.read_block()) is not None:
                    blocks.append(b)
                got.append((h.split(b"\n")[0], blocks))

    t = threading.Thread(target=reader)
    t.start()
    for i, blocks in enumerate(want):
        if i == 1:
            hdr, data = pm.Ring(k + 1), pm.Ring(k)
            hdr.lock_write()
            data.lock_write()
            hdr.write_block(pm.header_block(hdr, b"XFER 1\n"))
            for b in blocks:
                data.write_block(b)
            data.unlock_write()
            hdr.unlock_write()
            hdr.close()
            data.close()
        else:
            with dada.Hdu(k, "W") as w:
                w.write_header(f"XFER {i}\n")
                for b in blocks:
                    w.write_block(b)
    t.join(60)
    assert not t.is_alive()
    assert got == [(f"XFER {i}".encode(), want[i]) for i in range(3)]


def test_foreign_device_ring_is_refused(ring):
    """a PSRDADA device ring made by libpsrdada (64-B CUDA handle segments,
    no libpafdada holder) is refused cleanly, not read past its segments"""
    k = ring(2, 64)                      # block segments of a CUDA-handle's size
    r = pm.Ring(k)
    r.s.set("on_device_id", 0)           # as libpsrdada's dada_db -g would leave it
    r.close()
    with pytest.raises(OSError):
        dada.Hdu(k, "R")
    assert dada.destroy_ring(k)           # removed without touching an absent holder


def test_two_readers_one_from_each_library(ring):
    """a 2-reader ring: one libpafdada reader and one PSRDADA reader (the
    model) each take every block of the transfer libpafdada writes; the
    writer waits for both (CLEAR of every reader, get_next_write @0x403f20)"""
    k = ring(2, 2048, nreaders=2)
    rng = np.random.default_rng(10)
    want = [rng.integers(0, 256, 2048, dtype=np.uint8).tobytes() for _ in range(7)] + [b"t" * 5]
    got = {}

    def ours():
        with dada.Hdu(k, "R") as r:
            r.read_header()
            blocks = []
            while (b := r.read_block()) is not None:
                blocks.append(b)
            got["libpafdada"] = blocks

    def model():
        hdr, data = pm.Ring(k + 1), pm.Ring(k)
        try:
            hdr.lock_read()
            data.lock_read()
            hdr.get_next_read()
            hdr.mark_cleared()
            got["psrdada"] = data.read_transfer()
            got["slot"] = data.iread
            data.unlock_read()
            hdr.unlock_read()
        finally:
            hdr.close()
            data.close()

    ts = [threading.Thread(target=ours), threading.Thread(target=model)]
    for t in ts:
        t.start()
    with dada.Hdu(k, "W") as w:
        w.write_header("HDR_SIZE 4096\n")
        for b in want:
            w.write_block(b)
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts)
    assert got["libpafdada"] == want and got["psrdada"] == want
    assert got["slot"] in (0, 1)


def test_destroy_cleans_a_half_built_ring(ring):
    """a ring whose creator died after the semaphores and blocks but before
    the sync segment was complete (here: the sync segment removed) leaves
    no object behind dada_db -d, so its key can be used again"""
    k = ring(3, 4096)
    sid = pm._libc.shmget(k, 0, 0)
    pm._libc.shmctl(sid, pm.IPC_RMID, None)   # only the sync segment goes
    assert not dada.destroy_ring(k)           # nothing complete to destroy ...
    assert pm._libc.semget(k + 0x10000, 0, 0) < 0
    assert all(pm._libc.shmget(k + 0x10000 * (10 + i), 0, 0) < 0 for i in range(3))
    dada.create_ring(k, 3, 4096)              # ... and the key is free again


def test_mixed_library_transfers_property(ring):
    """Random transfers (more than the 8 in-flight transfer slots, so xfer
    indices wrap), each written by libpafdada or by the PSRDADA model and
    then read by libpafdada or by the model: every transfer arrives whole
    and in order, and the shared counters agree with the protocol"""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    xfer = st.tuples(st.sampled_from(["paf", "model"]), st.sampled_from(["paf", "model"]),
                     st.integers(0, 3), st.sampled_from(["short", "full"]), st.integers(1, 255))

    @settings(max_examples=20, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
    @given(xfers=st.lists(xfer, min_size=1, max_size=12), nbufs=st.integers(4, 6),
           seed=st.integers(0, 1 << 30))
    def check(xfers, nbufs, seed):
        bufsz = 256
        k = ring(nbufs, bufsz)
        rng = np.random.default_rng(seed)
        nblocks = 0
        for t, (wlib, rlib, nfull, end, short) in enumerate(xfers):
            blocks = [rng.integers(0, 256, bufsz, dtype=np.uint8).tobytes() for _ in range(nfull)]
            if end == "short":
                blocks.append(rng.integers(0, 256, short, dtype=np.uint8).tobytes())
            head = f"XFER {t}\n".encode()
            if wlib == "paf":
                with dada.Hdu(k, "W") as w:
                    w.write_header(head)
                    for b in blocks:
                        w.write_block(b)
            else:
                hdr, data = pm.Ring(k + 1), pm.Ring(k)
                hdr.lock_write()
                data.lock_write()
                hdr.write_block(pm.header_block(hdr, head))
                for b in blocks:
                    data.write_block(b)
                if end == "full":
                    if blocks:
                        data.end_transfer()
                    else:  # libpsrdada writes nothing for an empty transfer: end it explicitly
                        data.get_next_write()
                        data.mark_filled(0)
                data.unlock_write()
                hdr.unlock_write()
                hdr.close()
                data.close()
            nblocks += len(blocks) + (end == "full")
            if rlib == "paf":
                with dada.Hdu(k, "R") as r:
                    h = r.read_header()
                    got = []
                    while (b := r.read_block()) is not None:
                        got.append(b)
                    assert r.eod()
            else:
                hdr, data = pm.Ring(k + 1), pm.Ring(k)
                hdr.lock_read()
                data.lock_read()
                p, n = hdr.get_next_read()
                h = pm.C.string_at(p, n)
                hdr.mark_cleared()
                got = data.read_transfer()
                data.unlock_read()
                hdr.unlock_read()
                hdr.close()
                data.close()
            assert h.split(b"\0")[0] == head and got == blocks, (t, wlib, rlib)
        r = pm.Ring(k)
        try:
            assert (r.s.get("w_buf"), r.s.get("w_xfer"), r.s.get("r_xfers", 0)) == \
                (nblocks, len(xfers), len(xfers))
            assert [pm.semval(r.semid_data[0], i) for i in (0, 1, 2)] == [8, 8, 0]  # SODACK EODACK FULL
        finally:
            r.close()
        dada.destroy_ring(k)

    check()
