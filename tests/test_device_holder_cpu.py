"""The device-ring holder's lifecycle on the CPU (SURVEY.md 8f rank 3;
DESIGN.md 7b): `dada_db -g` with libpafdada reaching a host-memory test
double of the HIP runtime (tests/c/fake_hip.c, built here as
libamdhip64.so.7 and put first on LD_LIBRARY_PATH of the processes these
tests start -- never loaded by anything else).

* the holder's export record in block 0's segment (dada_device_ring_info):
  no retry on a clean ring; a refused primer is counted and harmless; a
  ring block refused once is exported after a retry and counted, so the GPU
  suite's zero-retry assertion (tests/conftest.py) has something to see;
* the ordering rule survives a destroyer killed while it waits: the holder
  keeps the blocks while an importer stays attached and frees them the
  moment it detaches (the advisor's round-5 finding: a waiter counter left
  +1 by a killed `dada_db -d` let the holder free mapped blocks);
* `dada_db -d` with an importer attached reports the importer (EBUSY), not
  "nothing to destroy"."""
import os
import signal
import subprocess
import sys
import time

import numpy as np
import pytest

from conftest import REPO
from paf_b2p import dada

BIN = dada.BIN_DIR
_KEY = [0x4c00 + (os.getpid() % 64) * 0x40]


def _key():
    _KEY[0] += 4
    dada.destroy_ring(_KEY[0])
    return _KEY[0]


@pytest.fixture(scope="module")
def fake_env(tmp_path_factory):
    d = tmp_path_factory.mktemp("fake_hip")
    subprocess.run(["gcc", "-O1", "-g", "-fPIC", "-shared", "-Wall", "-Werror", "-o", str(d / "libamdhip64.so.7"),
                    os.path.join(REPO, "tests", "c", "fake_hip.c")], check=True)
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = str(d) + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
    env.pop("FAKE_HIP_REFUSE", None)
    env["FAKE_HIP_LOG"] = str(d / "hip.log")
    return env


def _create(env, key, refuse=""):
    e = dict(env, FAKE_HIP_REFUSE=refuse)
    return subprocess.run([os.path.join(BIN, "dada_db"), "-k", f"{key:x}", "-b", "8192", "-n", "3", "-g", "0"],
                          capture_output=True, text=True, timeout=60, env=e)


def _destroy(env, key):
    return subprocess.run([os.path.join(BIN, "dada_db"), "-k", f"{key:x}", "-d"], capture_output=True, text=True,
                          timeout=60, env=env)


@pytest.mark.parametrize("refuse,retries,primer", [("", 0, 0), ("0", 0, 1), ("1", 1, 0), ("1,2", 1, 0),
                                                   ("0,3", 1, 1)])
def test_holder_export_record(fake_env, refuse, retries, primer):
    """call 0 is the primer's export; call 1 block 0's; a refused block
    export is tried once more on the same pointer (call 2), then on a fresh
    allocation -- each block that needed either counts one retry"""
    key = _key()
    r = _create(fake_env, key, refuse)
    try:
        assert r.returncode == 0, r.stderr
        info = dada.device_ring_info(key)
        assert info["holder_state"] == 1 and info["holder_pid"] > 0 and info["device"] == 0, info
        assert info["export_retries"] == retries, (info, r.stderr)
        assert info["primer_refused"] == primer, (info, r.stderr)
        assert ("IPC export retr" in r.stderr) == (retries > 0), r.stderr
        assert ("primer allocation was not exportable" in r.stderr) == bool(primer), r.stderr
    finally:
        d = _destroy(fake_env, key)
    assert d.returncode == 0, d.stderr
    with pytest.raises(OSError):
        dada.device_ring_info(key)


def test_holder_gives_up_after_refused_tries(fake_env):
    """every try of block 0 refused (4 allocations, each tried twice): the
    ring is not made and the caller is told which call failed"""
    key = _key()
    r = _create(fake_env, key, ",".join(str(i) for i in range(1, 9)))
    assert r.returncode != 0
    assert "hipIpcGetMemHandle" in r.stderr and "holder failed" in r.stderr, r.stderr
    with pytest.raises(OSError):
        dada.device_ring_info(key)
    dada.destroy_ring(key)


def _importer(env, key):
    """a process that connects to the ring (every block's handle imported)
    and stays attached: libpafdada through ctypes alone, since paf_b2p
    imports torch, whose own HIP runtime would be found before the double"""
    code = ("import ctypes as C, time; L = C.CDLL(%r); L.dada_hdu_create.restype = C.c_void_p; "
            "L.dada_hdu_create.argtypes = [C.c_void_p]; L.dada_hdu_set_key.argtypes = [C.c_void_p, C.c_int]; "
            "L.dada_hdu_connect.argtypes = [C.c_void_p]; h = L.dada_hdu_create(None); "
            "L.dada_hdu_set_key(h, %d); assert L.dada_hdu_connect(h) == 0; print('attached', flush=True); "
            "time.sleep(120)") % (dada.DADA_LIB, key)
    p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         env=env)
    assert p.stdout.readline().strip() == "attached", p.stderr.read()
    return p


def _state(key):
    return dada.device_ring_info(key)["holder_state"]


def test_killed_destroyer_does_not_free_blocks_under_an_importer(fake_env):
    key = _key()
    assert _create(fake_env, key).returncode == 0
    imp = _importer(fake_env, key)
    try:
        t_end = time.time() + 5
        while dada.device_ring_info(key)["importers"] < 1 and time.time() < t_end:
            time.sleep(0.05)
        assert dada.device_ring_info(key)["importers"] == 1
        d = subprocess.Popen([os.path.join(BIN, "dada_db"), "-k", f"{key:x}", "-d"], stderr=subprocess.PIPE,
                             env=fake_env)
        time.sleep(1.0)  # the destroyer has told the holder to stop and is waiting for it
        assert d.poll() is None
        d.send_signal(signal.SIGKILL)
        d.wait()
        # the holder is stopping, but an importer is attached: the blocks stay
        t_end = time.time() + 2.5
        while time.time() < t_end:
            assert _state(key) == 1, "holder freed the blocks while an importer had them open"
            time.sleep(0.05)
        imp.kill()
        imp.wait()
        t_end = time.time() + 5
        while _state(key) != 2 and time.time() < t_end:
            time.sleep(0.02)
        assert _state(key) == 2, "holder did not free the blocks once the importer was gone"
    finally:
        if imp.poll() is None:
            imp.kill()
            imp.wait()
        _destroy(fake_env, key)
    log = open(fake_env["FAKE_HIP_LOG"]).read()
    assert "free " in log


def test_destroy_with_importer_reports_it(fake_env):
    """dada_db -d while a process has the blocks open: exits 1 naming the
    importer (EBUSY kept through the ring's removal), and the holder frees
    the blocks once that process detaches"""
    key = _key()
    assert _create(fake_env, key).returncode == 0
    imp = _importer(fake_env, key)
    pid = dada.device_ring_info(key)["holder_pid"]
    try:
        d = _destroy(fake_env, key)
        assert d.returncode == 1
        assert "still have the blocks open" in d.stderr, d.stderr
        assert "nothing (complete) to destroy" not in d.stderr, d.stderr
    finally:
        imp.kill()
        imp.wait()
    t_end = time.time() + 5
    while os.path.exists(f"/proc/{pid}") and time.time() < t_end:
        try:
            if open(f"/proc/{pid}/stat").read().split(") ")[1].startswith("Z"):
                break
        except OSError:
            break
        time.sleep(0.05)
    st = open(f"/proc/{pid}/stat").read().split(") ")[1][0] if os.path.exists(f"/proc/{pid}") else "gone"
    assert st in ("Z", "gone"), st


def test_holder_without_primer_diagnostic(fake_env):
    """DADA_HOLDER_NO_PRIMER=1 (tools/devring_probe.py noprimer): block 0 is
    the holder's first allocation again, so a refused first export lands on
    a ring block and is counted as its retry"""
    key = _key()
    r = _create(dict(fake_env, DADA_HOLDER_NO_PRIMER="1"), key, "0")
    try:
        assert r.returncode == 0, r.stderr
        info = dada.device_ring_info(key)
        assert info["export_retries"] == 1 and info["primer_refused"] == 0, (info, r.stderr)
        assert "on block 0" in r.stderr, r.stderr
    finally:
        assert _destroy(fake_env, key).returncode == 0


@pytest.mark.parametrize("fail_at", [1, 2])
def test_diskdb_failed_copy_ends_the_transfer(fake_env, tmp_path, fail_at):
    """paf_diskdb into a GPU-resident ring whose copy into block `fail_at`
    fails (a HIP error): it exits 1 with an ERR line naming the copy, and
    ends the transfer with the 0-byte end-of-data block where that block
    was -- the reader gets the blocks copied before and a clean end, never a
    half-copied block"""
    key = _key()
    kf = tmp_path / "in.dada"
    dada.write_dada_file(str(kf), "x 1\n", np.arange(3 * 8192, dtype=np.uint32).view(np.uint8)[:3 * 8192])
    hdr = tmp_path / "hdr.txt"
    hdr.write_text("HDR_SIZE 4096\nNBIT 8\n")
    assert _create(fake_env, key).returncode == 0
    out = tmp_path / "out.dada"
    try:
        sink = subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{key:x}", "-o", str(out)],
                                stderr=subprocess.PIPE, text=True, env=fake_env)
        src = subprocess.run([os.path.join(BIN, "paf_diskdb"), "-a", f"{key:x}", "-b", str(tmp_path), "-c",
                              "in.dada", "-d", str(hdr), "-e", "1"], capture_output=True, text=True, timeout=60,
                             env=dict(fake_env, FAKE_HIP_MEMCPY_FAIL=str(fail_at)))
        _, serr = sink.communicate(timeout=60)
        assert src.returncode == 1 and "ERR: copy into device block failed" in src.stderr, src.stderr
        assert sink.returncode == 0, serr
        assert f"in {fail_at - 1} blocks" in serr, serr  # the blocks before the failed copy, then the end
        assert os.path.getsize(out) == 4096 + (fail_at - 1) * 8192
    finally:
        if sink.poll() is None:
            sink.kill()
            sink.wait()
        assert _destroy(fake_env, key).returncode == 0
