"""The hosts build against PSRDADA's own API (CPU, compile-only).

INTEGRATION.md tells a maintainer who keeps PSRDADA's dada_db / dada_dbdisk
to build paf_baseband2power and paf_diskdb against the real libpsrdada
(-DB2P_PSRDADA, PSRDADA's include directory, -lpsrdada).  libpsrdada is not
in this image, so this test compiles both hosts with -DB2P_PSRDADA against
declarations-only stand-ins for PSRDADA's headers (tests/c/psrdada_api,
restated from SURVEY.md Appendix A) and checks the objects' undefined DADA
symbols: every one must be in the PSRDADA subset the reference's hosts call
(Appendix A "writer subset" + "reader subset"); none of libpafdada's
extensions (device rings, read depth, dada_hdu_open_read, ascii_header_del,
ipcbuf_get_nbufs / ipcbuf_get_buffer) may remain.
"""
import os
import re
import subprocess

import pytest

from conftest import REPO

HOSTS = os.path.join(REPO, "paf-baseband2power_amd", "csrc", "host")
API = os.path.join(REPO, "tests", "c", "psrdada_api")

# the calls the reference makes (writer) and the reader
# half its baseband2power stage needs
PSRDADA_SUBSET = {
    "dada_hdu_create", "dada_hdu_set_key", "dada_hdu_connect", "dada_hdu_lock_write",
    "dada_hdu_unlock_write", "dada_hdu_disconnect", "dada_hdu_destroy", "ipcbuf_get_bufsz",
    "ipcbuf_enable_sod", "ipcbuf_disable_sod", "ipcbuf_get_next_write", "ipcbuf_mark_filled",
    "ipcio_open_block_write", "ipcio_close_block_write", "fileread", "ascii_header_set",
    "multilog_open", "multilog_add", "multilog_close", "multilog",
    "dada_hdu_lock_read", "dada_hdu_unlock_read", "ipcbuf_get_next_read", "ipcbuf_mark_cleared",
    "ipcio_open_block_read", "ipcio_close_block_read", "ipcbuf_eod", "ascii_header_get",
    # paf_diskdb -T pre-maps the ring's blocks: the block count, from the
    # libpsrdada linked into the reference's own paf_diskdb (0x4053b0,
    # tests/golden/psrdada_abi.json)
    "ipcbuf_get_nbufs",
}
DADA_PREFIX = re.compile(r"^(dada_|ipcbuf_|ipcio_|ascii_header_|multilog|fileread)")


def undefined(obj):
    out = subprocess.run(["nm", "-u", str(obj)], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


# The stand-ins' return types are the DWARF's (tests/test_psrdada_abi.py); the
# alternative header set swaps each return type the hosts consume between int
# and a wider signed type, so the hosts depend on none of them beyond "< 0".
ALTERNATIVES = {
    "ipcio.h": [("ssize_t ipcio_close_block_read(", "int ipcio_close_block_read("),
                ("ssize_t ipcio_close_block_write(", "int ipcio_close_block_write(")],
    "futils.h": [("long fileread(", "int fileread(")],
    "ipcbuf.h": [("int ipcbuf_mark_filled(", "ssize_t ipcbuf_mark_filled("),
                 ("int ipcbuf_mark_cleared(", "ssize_t ipcbuf_mark_cleared("),
                 ("int ipcbuf_eod(", "long ipcbuf_eod(")],
    "dada_hdu.h": [("int dada_hdu_lock_read(", "long dada_hdu_lock_read("),
                   ("int dada_hdu_unlock_write(", "long dada_hdu_unlock_write(")],
}


def api_dir(variant, tmp_path):
    if variant == "published":
        return API
    d = tmp_path / "alt_api"
    d.mkdir()
    for name in os.listdir(API):
        src = open(os.path.join(API, name)).read()
        for a, b in ALTERNATIVES.get(name, []):
            assert a in src, (name, a)
            src = src.replace(a, b)
        (d / name).write_text(src)
    return str(d)


@pytest.mark.parametrize("variant", ["published", "alternative"])
@pytest.mark.parametrize("host", ["paf_baseband2power", "paf_diskdb"])
def test_host_compiles_against_psrdada_subset(host, variant, tmp_path):
    """-Wconversion -Werror against the stand-ins and against the same API
    with every uncertain return type swapped: the hosts depend on no
    return type beyond "negative means failure"."""
    obj = tmp_path / f"{host}.o"
    r = subprocess.run(["gcc", "-c", "-O2", "-std=gnu11", "-D_GNU_SOURCE", "-Wall", "-Wextra",
                        "-Wconversion", "-Werror", "-DB2P_PSRDADA", "-I", api_dir(variant, tmp_path),
                        "-I", os.path.join(REPO, "include"),
                        os.path.join(HOSTS, f"{host}.c"), "-o", str(obj)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    dada = {s for s in undefined(obj) if DADA_PREFIX.match(s)}
    assert dada, "no DADA calls found"
    assert dada <= PSRDADA_SUBSET, sorted(dada - PSRDADA_SUBSET)


def test_default_build_still_uses_libpafdada_extensions(tmp_path):
    # the default build keeps the GPU-resident ring path (ipcbuf_get_device,
    # read depth 2), which the PSRDADA build drops
    obj = tmp_path / "b2p.o"
    subprocess.run(["gcc", "-c", "-O2", "-std=gnu11", "-D_GNU_SOURCE", "-I", os.path.join(REPO, "include"),
                    os.path.join(HOSTS, "paf_baseband2power.c"), "-o", str(obj)], check=True)
    u = undefined(obj)
    assert {"ipcbuf_get_device", "ipcbuf_set_read_depth"} <= u


def test_psrdada_mode_diskdb_runs(tmp_path):
    """The PSRDADA-mode paf_diskdb (bin/psrdada_api: compiled against the
    Appendix A declarations, linked against libpafdada, whose calls it
    shares) writes a file into a ring byte for byte, header ring included,
    with the short last block ending the transfer (diskdb.cu:69-121)"""
    import numpy as np

    from paf_b2p import dada
    exe = os.path.join(dada.BIN_DIR, "psrdada_api", "paf_diskdb")
    assert os.path.exists(exe), "make -C paf-baseband2power_amd all builds it"
    key = 0x6e00 + (os.getpid() % 64) * 4
    dada.destroy_ring(key)
    bufsz = 32 * 1024
    dada.create_ring(key, 4, bufsz, 1)
    try:
        payload = np.random.default_rng(5).integers(0, 256, bufsz * 5 // 2, dtype=np.uint8)
        src = tmp_path / "obs.dada"
        dada.write_dada_file(str(src), "SKIPPED 1\n", payload)
        hdr = tmp_path / "header.txt"
        hdr.write_text("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\n")
        out = tmp_path / "out.dada"
        sink = subprocess.Popen([os.path.join(dada.BIN_DIR, "paf_dbdisk"), "-k", f"{key:x}", "-o",
                                 str(out)], stderr=subprocess.PIPE)
        src_p = subprocess.run([exe, "-a", f"{key:x}", "-b", str(tmp_path), "-c", "obs.dada", "-d",
                                str(hdr), "-e", "1"], capture_output=True, text=True, timeout=60)
        assert src_p.returncode == 0, src_p.stderr
        assert sink.wait(60) == 0, sink.stderr.read()
        h, data = dada.read_dada_file(str(out))
        assert h.decode() == hdr.read_text()
        assert np.array_equal(data, payload)
    finally:
        dada.destroy_ring(key)
