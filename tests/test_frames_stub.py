"""CPU tests of the frame-assembly hosts on their GPU path (no GPU):
`paf_dfdb` (a recorded frame stream into a ring) and `paf_capture` (UDP
frames into a ring: receive threads, the sorting thread, block switching),
built with ThreadSanitizer against the CPU test double of libpafb2p
(tests/c/b2p_cpu_stub.c: b2p_memset and b2p_assemble on the context's queue,
work completing up to B2P_STUB_DELAY_US late) and libpafdada's sources, with
-DB2P_TEST_HOST_RING_AS_DEVICE so a host ring takes the GPU-resident path.
Downstream, the stage built the same way integrates the ring's blocks (the
double sums BMF's big-endian words as the library does) and `paf_dbdisk`
writes the spectra; every spectrum must equal the C oracle's of the block
the oracle assembles from the same frames (capture.c:540, 562-568).

The failure sweep fails each b2p_* call these hosts make, at its first and
second call (B2P_STUB_FAIL): the host exits 1 with an ERR line on stderr,
the ring's transfer ends (the block being assembled becomes the 0-byte
end-of-data block, never a half-assembled block), and the stage downstream
exits 0 with correct spectra of the blocks delivered before -- or the call
was never reached and every spectrum comes out.  tests/test_gpu_device_ring.py
and tests/test_gpu_capture.py run the same hosts on the HIP library."""
import os
import re
import subprocess
import time

import numpy as np
import pytest
from hypothesis import HealthCheck, assume, given, seed, settings
from hypothesis import strategies as st

import b2p_oracle as npo
import oracle_c as co
from conftest import REPO
from paf_b2p import dada

BIN = dada.BIN_DIR
PKG = os.path.join(REPO, "paf-baseband2power_amd")
HOST = os.path.join(PKG, "csrc", "host")
STUB = os.path.join(REPO, "tests", "c", "b2p_cpu_stub.c")
DADA_SRC = [os.path.join(PKG, "csrc", "dada", f)
            for f in ("dada_ring.c", "dada_query.c", "dada_device.c", "ascii_header.c", "df_header.c")]
_KEY = [0x8000 + (os.getpid() % 64) * 0x40]  # a key window of its own (holder tests use 0x4c00..)
NCHUNK, BLOCK_NDF, NBLK = 4, 32, 3
REF_IDF, REF_SEC = 249990, 54  # the stream crosses a 27-s period
TSAN_ENV = {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1",
            "ASAN_OPTIONS": "detect_leaks=0:exitcode=86", "UBSAN_OPTIONS": "print_stacktrace=1:exitcode=87"}


def _key():
    _KEY[0] += 4
    return _KEY[0]


@pytest.fixture(scope="module")
def exes(tmp_path_factory):
    d = tmp_path_factory.mktemp("frames_stub")
    out = {}
    sans = {"": ["-fsanitize=thread"],  # the threads
            "_asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]}  # memory a failure frees
    for name in ("paf_dfdb", "paf_capture", "paf_baseband2power"):
        for tag, san in sans.items():
            exe = d / (name + tag)
            subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror",
                            *san, "-fno-omit-frame-pointer", "-I", os.path.join(REPO, "include"),
                            "-DB2P_TEST_HOST_RING_AS_DEVICE", os.path.join(HOST, name + ".c"), STUB, *DADA_SRC,
                            "-o", str(exe), "-pthread", "-ldl", "-lm"], check=True)
            out[name + tag] = str(exe)
    return out


def _stream(tmp_path, lost=0, seed=3, nblk=NBLK):
    """a BMF frame stream of nblk blocks (paf_dfgen: frames shuffled within a
    window, `lost` frames left out), its frames and chunk indices, and the
    blocks the oracle assembles from it"""
    g = npo.Geom(nbit=16, big_endian=1, nchunk=NCHUNK, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=BLOCK_NDF * 128)
    payload = co.fill_synthetic(g, g.block_bytes * nblk, 20181105, 4, seed)
    src = tmp_path / "in.dada"
    dada.write_dada_file(str(src), "NBIT 16\n", payload)
    df, ck = tmp_path / "s.df", tmp_path / "s.chunks"
    subprocess.run([os.path.join(BIN, "paf_dfgen"), "-i", str(src), "-o", str(df), "-n", str(NCHUNK),
                    "-c", str(ck), "-x", str(REF_IDF), "-s", str(REF_SEC), "-f", "1300", "-r", str(seed),
                    "-w", str(BLOCK_NDF * NCHUNK * 3 // 2), "-l", str(lost)], check=True, capture_output=True)
    dfs = np.fromfile(df, np.uint8).reshape(-1, npo.DF_BYTES)
    chunk = np.fromfile(ck, np.uint8)
    blocks, idf, sec = [], REF_IDF, REF_SEC
    for b in range(nblk):
        want = np.zeros(g.block_bytes, np.uint8)  # lost frames read as zeros
        co.assemble(dfs, chunk, idf, sec, want, BLOCK_NDF, NCHUNK)
        if not lost:
            assert np.array_equal(want, payload[b * g.block_bytes:(b + 1) * g.block_bytes])
        blocks.append(want)
        gi = idf + BLOCK_NDF
        idf, sec = gi % 250000, sec + (gi // 250000) * 27
    return g, df, ck, blocks


def _header(tmp_path, g):
    h = tmp_path / "hdr.txt"
    h.write_text(f"HDR_SIZE 4096\nNBIT 16\nNDIM 2\nNPOL 2\nNCHAN {NCHUNK * 7}\nNCHUNK {NCHUNK}\n"
                 "NCHAN_CHUNK 7\nNSAMP_DF 128\nBYTE_ORDER BE\nTSAMP 0.84375\n")
    return str(h)


def _chain(tmp_path, exes, g, producer, env, start_producer=None, stage_env=None, timeout=120):
    """producer -> host ring (as a device ring) -> the stage -> paf_dbdisk;
    returns (spectra, exit codes and stderr of [dbdisk, stage, producer]).
    start_producer(producer process): called once the three are running.
    stage_env: the stage's own environment (default: the producer's)"""
    kin, kout = _key(), _key()
    for k in (kin, kout):
        dada.destroy_ring(k)
    dada.create_ring(kin, 3, g.block_bytes)
    dada.create_ring(kout, 8, g.nout * 4)
    out = tmp_path / "power.dada"
    procs = []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out), "-W"],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([exes["paf_baseband2power"], "-a", f"{kin:x}", "-b", f"{kout:x}", "-c",
                                   str(tmp_path), "-d", "0", "-f", "header"],
                                  stderr=subprocess.PIPE, text=True, env=stage_env or env),
                 subprocess.Popen([a.replace("KEY", f"{kin:x}") for a in producer],
                                  stderr=subprocess.PIPE, text=True, env=env)]
        if start_producer:
            start_producer(procs[2])
        errs = [None] * 3
        for i in (2, 1, 0):
            errs[i] = procs[i].communicate(timeout=timeout)[1]
        rcs = [p.returncode for p in procs]
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in (kin, kout):
            dada.destroy_ring(k)
    for e in errs[1:]:
        assert "Sanitizer" not in e and "runtime error" not in e, e[-3000:]
    return data.view(np.uint32).reshape(-1, g.nout), rcs, errs


def _check(g, sp, blocks):
    for b in range(sp.shape[0]):
        assert np.array_equal(sp[b], co.power(g, blocks[b]).view(np.uint32)), b


@pytest.mark.parametrize("lost,delay", [(0, 0), (40, 500)])
def test_dfdb_gpu_path_on_the_cpu_double(exes, tmp_path, lost, delay):
    g, df, ck, blocks = _stream(tmp_path, lost)
    env = dict(os.environ, B2P_STUB_DELAY_US=str(delay), **TSAN_ENV)
    sp, rcs, errs = _chain(tmp_path, exes, g,
                           [exes["paf_dfdb"], "-a", "KEY", "-b", _header(tmp_path, g), "-c", str(df), "-k", str(ck),
                            "-n", str(NCHUNK), "-x", str(REF_IDF), "-s", str(REF_SEC)], env)
    assert rcs == [0, 0, 0], errs
    assert sp.shape[0] == NBLK, errs[2]
    _check(g, sp, blocks)
    placed = [int(x) for x in re.findall(r"block \d+: (\d+) of", errs[2])]
    nframes = os.path.getsize(df) // npo.DF_BYTES  # the frames paf_dfgen kept (-l drops some)
    assert sum(placed) == nframes and (nframes < NBLK * BLOCK_NDF * NCHUNK) == bool(lost), errs[2]


def _capture_cmd(exes, hdr, port, san=""):
    return [exes["paf_capture" + san], "-a", "KEY", "-f", hdr, "-c", str(BLOCK_NDF), "-n", str(NBLK), "-P", str(port),
            "-N", "3", "-m", "freq:1300", "-x", str(REF_IDF), "-s", str(REF_SEC), "-t", "1", "-b", "1", "-d", "0"]


def _sender(df, ck, port, delay_s=1.5):
    def go(producer=None):
        time.sleep(delay_s)  # the capture binds its ports and opens its context first
        snd = subprocess.run([os.path.join(BIN, "paf_dfsend"), "-i", str(df), "-k", str(ck), "-P", str(port),
                              "-N", "3", "-r", "50"], capture_output=True, text=True)
        assert snd.returncode == 0, snd.stderr
    return go


@pytest.mark.parametrize("delay", [0, 500])
def test_capture_gpu_path_on_the_cpu_double(exes, tmp_path, delay):
    """three receive threads, the sorting thread and the assembly on the
    double's queue, under ThreadSanitizer; frames over loopback UDP"""
    g, df, ck, blocks = _stream(tmp_path, seed=11)
    env = dict(os.environ, B2P_STUB_DELAY_US=str(delay), **TSAN_ENV)
    port = 26000 + (os.getpid() % 400) * 16 + delay // 100
    sp, rcs, errs = _chain(tmp_path, exes, g, _capture_cmd(exes, _header(tmp_path, g), port), env,
                           start_producer=_sender(df, ck, port))
    assert rcs == [0, 0, 0], errs
    assert sp.shape[0] == NBLK, errs[2]
    _check(g, sp, blocks)
    assert "0.000% lost" in errs[2] and "3 receive thread(s) over 3 port(s)" in errs[2], errs[2]


# the b2p_* calls each host makes on its GPU path (b2p_open is refused before
# any ring block: covered by its ERR line too)
CALLS = {"paf_dfdb": ["b2p_open", "b2p_memcpy", "b2p_memset", "b2p_assemble", "b2p_sync"],
         "paf_capture": ["b2p_open", "b2p_memcpy", "b2p_memset", "b2p_assemble", "b2p_sync"]}


@pytest.mark.parametrize("san", ["", "_asan"])
@pytest.mark.parametrize("host", ["paf_dfdb", "paf_capture"])
def test_frame_hosts_never_fail_silently(exes, tmp_path, host, san):
    """_asan: the host built with AddressSanitizer and UBSan (ThreadSanitizer
    otherwise): before the fix that closes the context before the ring is
    detached, a failed clear of paf_dfdb's block left the other clear queued
    into a ring block the failure path had unmapped (a SEGV here, a GPU
    fault on the HIP library)"""
    g, df, ck, blocks = _stream(tmp_path, seed=5)
    hdr = _header(tmp_path, g)
    failed_runs = 0
    for i, call in enumerate(CALLS[host]):
        for nth in (1, 2):
            run_dir = tmp_path / f"{call}_{nth}"
            run_dir.mkdir()
            env = dict(os.environ, B2P_STUB_FAIL=f"{call}:{nth}", B2P_STUB_DELAY_US="200", **TSAN_ENV)
            if host == "paf_dfdb":
                cmd = [exes["paf_dfdb" + san], "-a", "KEY", "-b", hdr, "-c", str(df), "-k", str(ck), "-n", str(NCHUNK),
                       "-x", str(REF_IDF), "-s", str(REF_SEC)]
                start = None
            else:
                port = 27000 + (os.getpid() % 400) * 32 + (16 if san else 0) + i * 2 + nth
                cmd, start = _capture_cmd(exes, hdr, port, san), _sender(df, ck, port)
            # the stage downstream runs without injected failures
            stage_env = dict(env)
            stage_env.pop("B2P_STUB_FAIL")
            sp, rcs, errs = _chain(run_dir, exes, g, cmd, env, start, stage_env)
            injected = "injected failure of" in errs[2]
            if rcs[2] == 0:
                assert not injected, (call, nth, errs[2])
                assert sp.shape[0] == NBLK, (call, nth)
            else:
                failed_runs += 1
                assert rcs[2] == 1 and injected, (call, nth, rcs, errs[2])
                assert "] ERR: " in errs[2], (call, nth, errs[2])
            assert rcs[:2] == [0, 0], (call, nth, rcs, errs[1][-800:])  # the stage and sink end cleanly
            _check(g, sp, blocks)  # every block delivered is whole and correct
    assert failed_runs >= len(CALLS[host]), failed_runs



_SCALE = int(os.environ.get("B2P_HYPOTHESIS_SCALE", "1"))
_SEED = os.environ.get("B2P_HYPOTHESIS_SEED")


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=4 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(st.sampled_from(["paf_dfdb", "paf_capture"]), st.integers(1, 12), st.integers(1, 48), st.integers(1, 5),
       st.floats(0.0, 0.3), st.floats(0.05, 1.5), st.sampled_from([1000, 249_990]), st.integers(0, 2 ** 31),
       st.sampled_from([0, 300, 1500]))
def test_frame_hosts_random_streams(exes, tmp_path_factory, host, nchunk, block_ndf, nblk, loss, shuffle, ref_idf,
                                    s, delay):
    """the random streams tests/test_gpu_stage_random.py sends through the
    HIP library (chunk counts, block lengths, 0-30 % of frames lost at the
    source, arrival shuffled within up to one block for paf_dfdb and 1.5
    for the capture), here through either
    host's GPU path on the double under ThreadSanitizer, its queue completing
    work up to `delay` us late: every spectrum equals the oracle's of its
    block as the oracle places the stream.  A capture run whose loopback
    dropped a frame says nothing about the capture and is discarded."""
    tmp = tmp_path_factory.mktemp("rand")
    g = npo.Geom(nbit=16, big_endian=1, nchunk=nchunk, nsamp_df=128, nchan_chunk=7, nsamp_int=block_ndf * 128)
    per_block = block_ndf * nchunk
    # paf_dfdb drops a frame that arrives more than one block behind the
    # newest (as the capture drops late frames, capture.c:464-531): its
    # streams are shuffled within one block (as tests/test_gpu_stage_random.py's
    # are); the capture's spill holds 256 frame times, so up to 1.5 blocks
    window = max(1, min(int((min(shuffle, 1.0) if host == "paf_dfdb" else shuffle) * per_block), 200 * nchunk))
    payload = co.fill_synthetic(g, g.block_bytes * nblk, s, 4, 2)
    src = tmp / "in.dada"
    dada.write_dada_file(str(src), "NBIT 16\n", payload)
    df, ck = tmp / "s.df", tmp / "s.chunks"
    ref_sec = 27 * 54
    subprocess.run([os.path.join(BIN, "paf_dfgen"), "-i", str(src), "-o", str(df), "-n", str(nchunk),
                    "-c", str(ck), "-x", str(ref_idf), "-s", str(ref_sec), "-f", "1300", "-r", str(s % 997),
                    "-w", str(window), "-l", str(int(loss * 1000))], check=True, capture_output=True)
    dfs = np.fromfile(df, dtype=np.uint8).reshape(-1, npo.DF_BYTES)
    chunk = np.fromfile(ck, dtype=np.uint8)
    assume(len(dfs) > 0)  # every frame lost at the source: nothing to place
    h = npo.df_decode(dfs)
    rel = np.trunc(h["idf"].astype(np.float64) + (h["sec"].astype(np.float64) - ref_sec) / 1.08e-4 - ref_idf)
    last = int(rel.max()) // block_ndf + 1  # blocks up to the last frame's
    hdr = tmp / "hdr.txt"
    hdr.write_text(f"HDR_SIZE 4096\nNBIT 16\nNDIM 2\nNPOL 2\nNCHAN {nchunk * 7}\nNCHUNK {nchunk}\n"
                   "NCHAN_CHUNK 7\nNSAMP_DF 128\nBYTE_ORDER BE\nTSAMP 0.84375\n")
    env = dict(os.environ, B2P_STUB_DELAY_US=str(delay), **TSAN_ENV)
    if host == "paf_dfdb":
        cmd, start, n_out = ([exes["paf_dfdb"], "-a", "KEY", "-b", str(hdr), "-c", str(df), "-k", str(ck), "-n",
                              str(nchunk), "-x", str(ref_idf), "-s", str(ref_sec)], None, last)
    else:
        port = 28000 + (os.getpid() % 400) * 16 + s % 13
        cmd = [exes["paf_capture"], "-a", "KEY", "-f", str(hdr), "-c", str(block_ndf), "-n", str(nblk), "-P",
               str(port), "-N", "3", "-m", "freq:1300", "-x", str(ref_idf), "-s", str(ref_sec), "-t", "1", "-d", "0"]
        start, n_out = _sender(df, ck, port), min(nblk, last)  # the capture ends with the stream
    sp, rcs, errs = _chain(tmp, exes, g, cmd, env, start)
    assert rcs == [0, 0, 0], [e[-800:] for e in errs]
    if host == "paf_capture":
        m = re.search(r"capture: (\d+) frames received", errs[2])
        assert m, errs[2][-800:]
        assume(int(m.group(1)) == len(dfs))  # the loopback delivered every frame sent
    assert sp.shape[0] == n_out, errs[2][-800:]
    idf, sec = ref_idf, ref_sec
    for b in range(n_out):
        want = np.zeros(g.block_bytes, np.uint8)
        co.assemble(dfs, chunk, idf, sec, want, block_ndf, nchunk)
        assert np.array_equal(sp[b], co.power(g, want).view(np.uint32)), (host, b, errs[2][-600:])
        gi = idf + block_ndf
        idf, sec = gi % 250000, sec + (gi // 250000) * 27


def test_capture_sigterm_delivers_the_block_being_filled(exes, tmp_path):
    """SIGTERM while frames of block 1 are still arriving (the stream has
    not gone idle): the capture delivers the block being filled -- block 0,
    whole -- ends the ring's transfer and exits 0; the stage writes its
    spectrum and ends cleanly (the reference stopped on a quit flag,
    capture.c:32-39)"""
    import signal
    g, df, ck, blocks = _stream(tmp_path, seed=13)
    dfs = np.fromfile(df, np.uint8).reshape(-1, npo.DF_BYTES)
    chunk = np.fromfile(ck, np.uint8)
    h = npo.df_decode(dfs)
    rel = np.trunc(h["idf"].astype(np.float64) + (h["sec"].astype(np.float64) - REF_SEC) / 1.08e-4 - REF_IDF)
    keep = rel < BLOCK_NDF * 1.5  # block 0 and half of block 1
    part_df, part_ck = tmp_path / "part.df", tmp_path / "part.chunks"
    dfs[keep].tofile(part_df)
    chunk[keep].tofile(part_ck)
    hdr = _header(tmp_path, g)
    port = 29000 + (os.getpid() % 400) * 8
    env = dict(os.environ, B2P_STUB_DELAY_US="300", **TSAN_ENV)
    cmd = [exes["paf_capture"], "-a", "KEY", "-f", hdr, "-c", str(BLOCK_NDF), "-P", str(port), "-N", "3",
           "-m", "freq:1300", "-x", str(REF_IDF), "-s", str(REF_SEC), "-t", "60", "-d", "0"]
    def start(capture):
        _sender(part_df, part_ck, port)()
        time.sleep(1.0)  # every frame sorted; the stream not idle for 60 s
        capture.send_signal(signal.SIGTERM)

    sp, rcs, errs = _chain(tmp_path, exes, g, cmd, env, start)
    assert rcs == [0, 0, 0], [e[-800:] for e in errs]
    assert "stopped by a signal" in errs[2], errs[2][-800:]
    assert sp.shape[0] == 1, errs[2][-800:]
    _check(g, sp, blocks)


def test_dfdb_sigterm_delivers_the_block_in_hand(exes, tmp_path):
    """SIGTERM while paf_dfdb waits for a free ring block (the ring full, no
    reader yet): once a block frees, the one it was waiting to fill is
    assembled and delivered, then the transfer ends and paf_dfdb exits 0;
    the stage downstream integrates exactly those blocks, each equal to the
    oracle's"""
    import signal
    g, df, ck, blocks = _stream(tmp_path, seed=17, nblk=6)  # stopped after 3 of the 6
    kin, kout = _key(), _key()
    for k in (kin, kout):
        dada.destroy_ring(k)
    dada.create_ring(kin, 2, g.block_bytes)
    dada.create_ring(kout, 8, g.nout * 4)
    out = tmp_path / "power.dada"
    env = dict(os.environ, B2P_STUB_DELAY_US="300", **TSAN_ENV)
    procs = []
    try:
        dfdb = subprocess.Popen([exes["paf_dfdb"], "-a", f"{kin:x}", "-b", _header(tmp_path, g), "-c", str(df),
                                 "-k", str(ck), "-n", str(NCHUNK), "-x", str(REF_IDF), "-s", str(REF_SEC)],
                                stderr=subprocess.PIPE, text=True, env=env)
        procs.append(dfdb)
        time.sleep(1.5)  # blocks 0 and 1 fill the ring; block 2 waits for a free slot
        assert dfdb.poll() is None
        dfdb.send_signal(signal.SIGTERM)
        time.sleep(0.3)
        procs += [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                   stderr=subprocess.PIPE, text=True),
                  subprocess.Popen([exes["paf_baseband2power"], "-a", f"{kin:x}", "-b", f"{kout:x}", "-c",
                                    str(tmp_path), "-d", "0", "-f", "header"], stderr=subprocess.PIPE, text=True,
                                   env=env)]
        errs = [p.communicate(timeout=60)[1] for p in procs]
        rcs = [p.returncode for p in procs]
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in (kin, kout):
            dada.destroy_ring(k)
    assert rcs == [0, 0, 0], [e[-800:] for e in errs]
    m = re.search(r"stopped by a signal after (\d+) blocks", errs[0])
    assert m and 1 <= int(m.group(1)) < 6, errs[0][-800:]  # (3 when the ring filled before the signal)
    sp = data.view(np.uint32).reshape(-1, g.nout)
    assert sp.shape[0] == int(m.group(1))
    _check(g, sp, blocks)
