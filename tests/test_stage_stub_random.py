"""CPU property test of the stage's orchestration (no GPU): the real
`paf_baseband2power` host code, linked against the CPU test double of
libpafb2p (tests/c/b2p_cpu_stub.c: exact sums; every call finished on
return, or a stream model whose work completes up to 2 ms late, drawn per
example) and libpafdada's sources, between PSRDADA writers in this process
and `paf_dbdisk`.  Random layouts (int8, int16 LE and BMF's int16 BE),
ring depths, block counts, short last blocks, output pols, sum or mean, and
every threading mode of the stage:

  single       one host ring (worker)
  single_dev   one ring on the GPU-resident path (run_device_pipelined, with
               -DB2P_TEST_HOST_RING_AS_DEVICE)
  gathered     -n 2 / 3 host rings (worker, barriers per round)
  gathered_dev -n 2 / 3 on the GPU-resident path (worker_gather_dev: rounds
               of queued blocks, asynchronous gathers)
  split        -t 2 / 3 (worker_split: shares of one block, partials reduced)

Every output spectrum must equal the C oracle's of its block(s).
B2P_STAGE_TSAN=1 builds the stage with ThreadSanitizer.  This runs
in the CPU suite every round; tests/test_gpu_stage_random.py runs the same
kinds of cases through the HIP library on a GPU."""
import os
import subprocess
import threading
import time

import numpy as np
import pytest
from hypothesis import HealthCheck, given, seed, settings
from hypothesis import strategies as st

import b2p_oracle as npo
import oracle_c as co
from conftest import REPO
from paf_b2p import dada

BIN = dada.BIN_DIR
PKG = os.path.join(REPO, "paf-baseband2power_amd")
STAGE = os.path.join(PKG, "csrc", "host", "paf_baseband2power.c")
STUB = os.path.join(REPO, "tests", "c", "b2p_cpu_stub.c")
DADA_SRC = [os.path.join(PKG, "csrc", "dada", f) for f in ("dada_ring.c", "dada_query.c", "dada_device.c",
                                                            "ascii_header.c", "df_header.c")]
_SCALE = int(os.environ.get("B2P_HYPOTHESIS_SCALE", "1"))
_SEED = os.environ.get("B2P_HYPOTHESIS_SEED")
_KEY = [0x5a00 + (os.getpid() % 64) * 0x80]
# B2P_STAGE_TSAN=1: the stage built with ThreadSanitizer (halt on the first
# report), so the random cases also hunt data races in its threads
_TSAN = ["-fsanitize=thread", "-fno-omit-frame-pointer"] if os.environ.get("B2P_STAGE_TSAN") else []
_ASAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"]
ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:exitcode=86", "UBSAN_OPTIONS": "print_stacktrace=1:exitcode=87"}


@pytest.fixture(scope="module")
def stages(tmp_path_factory):
    d = tmp_path_factory.mktemp("stub_stage")
    out = {}
    # "_asan": AddressSanitizer + UBSan builds, for the failure sweep: a
    # failure path that frees or detaches memory the double's queue (standing
    # for a HIP stream) still writes into is a heap-use-after-free there
    for name, defs, san in (("host", [], _TSAN), ("dev", ["-DB2P_TEST_HOST_RING_AS_DEVICE"], _TSAN),
                            ("host_asan", [], _ASAN), ("dev_asan", ["-DB2P_TEST_HOST_RING_AS_DEVICE"], _ASAN)):
        exe = d / f"stage_{name}"
        subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror",
                        *san, "-I", os.path.join(REPO, "include"), *defs, STAGE, STUB, *DADA_SRC, "-o",
                        str(exe), "-pthread", "-ldl", "-lm"], check=True)
        out[name] = str(exe)
    return out


def _key():
    _KEY[0] += 0x10 * 4
    return _KEY[0]


@st.composite
def cases(draw):
    nbit = draw(st.sampled_from([8, 16]))
    word = 4 * nbit // 8
    nchunk = draw(st.integers(1, 8))
    ncc = draw(st.integers(1, 32))
    base = 1
    while (base * ncc * word) % 16:
        base *= 2
    nsamp_df = base * draw(st.integers(1, 2))
    mode = draw(st.sampled_from(["single", "single_dev", "gathered", "gathered_dev", "split"]))
    nmem = draw(st.integers(2, 3)) if mode != "single" and mode != "single_dev" else 1
    nframes = draw(st.integers(1, 48))
    if mode == "split":
        nframes = max(nmem, nframes - nframes % nmem)
    g = npo.Geom(nbit=nbit, big_endian=int(nbit == 16 and draw(st.booleans())), nchunk=nchunk,
                 nsamp_df=nsamp_df, nchan_chunk=ncc,
                 npol_out=draw(st.sampled_from([1, 2])), nsamp_int=nframes * nsamp_df,
                 mean=int(draw(st.booleans())))
    nblk = draw(st.integers(1, 10))
    shorter = [draw(st.integers(0, 2)) for _ in range(nmem)] if mode.startswith("gathered") else [0]
    return dict(g=g, mode=mode, nmem=nmem, nbufs=draw(st.integers(2, 6)), nblk=nblk,
                nblks=[max(1, nblk - d) for d in shorter],
                short=mode in ("single", "single_dev", "split") and nframes > 1 and draw(st.booleans()),
                sync=mode in ("single", "gathered") and draw(st.booleans()),
                seed=draw(st.integers(0, 2 ** 32 - 1)),
                # the double's stream model: synchronous, or work completing
                # up to this many us after it is enqueued (b2p_cpu_stub.c)
                delay_us=draw(st.sampled_from([0, 300, 2000])))


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=40 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(cases())
def test_stage_orchestration_random(stages, tmp_path_factory, case):
    g, mode, nmem = case["g"], case["mode"], case["nmem"]
    tmp = tmp_path_factory.mktemp("run")
    rings = 1 if mode == "split" else nmem
    base, kout = _key(), _key()
    keys = [base + 0x10 * r for r in range(rings)]
    nblks = case["nblks"] if mode.startswith("gathered") else [case["nblk"]]
    blocks = [[co.fill_synthetic(g, g.block_bytes, case["seed"], r, b) for b in range(nblks[r])]
              for r in range(rings)]
    # a longer transfer's writer must not wait on a stage that has left
    nbufs = case["nbufs"] if len(set(nblks)) == 1 else max(case["nbufs"], max(nblks) + 1)
    hdr = (f"HDR_SIZE 4096\nNBIT {g.nbit}\nNDIM 2\nNPOL 2\nNCHAN {g.nchunk * g.nchan_chunk}\n"
           f"NCHUNK {g.nchunk}\nNCHAN_CHUNK {g.nchan_chunk}\nNSAMP_DF {g.nsamp_df}\n"
           f"BYTE_ORDER {'BE' if g.big_endian else 'LE'}\n"
           "TSAMP 0.84375\n")
    for k in keys + [kout]:
        dada.destroy_ring(k)
    for k in keys:
        dada.create_ring(k, nbufs, g.block_bytes)
    onsub = nmem if mode.startswith("gathered") else 1
    dada.create_ring(kout, 4, onsub * g.nout * 4)
    args = ["-f", "header", "-p", str(g.npol_out)] + (["-m"] if g.mean else []) + (["-S"] if case["sync"] else [])
    if mode.startswith("gathered"):
        args += ["-n", str(nmem), "-G", "copy"]
    if mode == "split":
        args += ["-t", str(nmem), "-G", "copy"]
    # B2P_STAGE_ASAN=1: the AddressSanitizer + UBSan builds (a hunt for
    # memory the double's late queues touch after the stage let it go)
    exe = stages[("dev" if mode.endswith("_dev") else "host") + ("_asan" if os.environ.get("B2P_STAGE_ASAN") else "")]
    out = tmp / "power.dada"
    procs, errs = [], []
    try:
        env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
                   B2P_STUB_DELAY_US=os.environ.get("B2P_STUB_DELAY_US", str(case["delay_us"])), **ASAN_ENV)
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([exe, "-a", f"{base:x}", "-b", f"{kout:x}", "-c", str(tmp), "-d", "0"] + args,
                                  stderr=subprocess.PIPE, env=env)]

        def writer(k, bl):
            try:
                with dada.Hdu(k, "W") as w:
                    w.write_header(hdr)
                    for b in bl:
                        w.write_block(b.tobytes())
                    if case["short"]:
                        w.write_block(bl[0][: g.frame_bytes].tobytes())
            except Exception as e:  # noqa: BLE001 -- reported below
                errs.append(e)
        ths = [threading.Thread(target=writer, args=(k, bl)) for k, bl in zip(keys, blocks)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(60)
        assert not errs, errs
        for p in procs[::-1]:
            _, e = p.communicate(timeout=60)
            assert p.returncode == 0, (case, e.decode(errors="replace")[-800:])
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in keys + [kout]:
            dada.destroy_ring(k)
    sp = data.view(np.uint32).reshape(-1, onsub, g.nout)
    n = min(nblks)
    assert sp.shape[0] == n, case
    for b in range(n):
        for r in range(onsub):
            want = co.power(g, blocks[r][b], nthreads=2).view(np.uint32)
            assert np.array_equal(sp[b, r], want), (case, b, r)
    log = open(str(tmp / "paf_baseband2power.log")).read()
    assert f"FINISH PAF_PROCESS: {n} integrations" in log, (case, log[-600:])
    if len(set(nblks)) == 1:
        assert ("partial integration skipped" in log) == case["short"], (case, log[-600:])
    else:  # the shorter transfer's end costs one integration, whatever the writers' timing
        assert f"FINISH PAF_PROCESS: {n} integrations, 1 skipped, ok" in log, (case, log[-600:])


def test_failed_stage_names_its_errors_on_stderr(stages, tmp_path):
    """a run that fails (here: no input ring at the key) exits 1 and repeats
    this run's ERR log lines on stderr, as the reference reports errors
    there (paf_baseband2power.cu:51-52); earlier runs' lines in the same
    log file are not repeated"""
    (tmp_path / "paf_baseband2power.log").write_text("[earlier] ERR: an earlier run's error\n")
    k = _key()
    dada.destroy_ring(k)
    r = subprocess.run([stages["host"], "-a", f"{k:x}", "-b", f"{k + 2:x}", "-c", str(tmp_path), "-d", "0",
                        "-f", "int8:256"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert f"ERR: cannot attach/lock input ring {k:x}" in r.stderr, r.stderr
    assert "FAILED, log" in r.stderr and "earlier run" not in r.stderr, r.stderr


@pytest.mark.parametrize("mode", ["gathered", "gathered_dev"])
@pytest.mark.parametrize("ndev,gather,want", [(8, None, "RCCL ncclGather"), (1, None, "peer copies"),
                                              (4, "rccl", "refused")])
def test_stage_n8_group_transport(stages, tmp_path, mode, ndev, gather, want):
    """`paf_baseband2power -n 8 -d 0` (configs[4]'s eight
    sub-bands) with B2P_STUB_NDEV devices visible: on 8 distinct GPUs every
    member r drives GPU r and the stage picks RCCL (group_mode), not peer
    copies; on one GPU it picks peer copies; `-G rccl` with members sharing
    GPUs is refused at set-up as RCCL refuses it, and the stage exits 1
    naming the call on stderr.  Spectra equal the oracle's where it runs."""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=16, npol_out=1, nsamp_int=64)
    nmem, nblk = 8, 3
    base, kout = _key(), _key()
    base += 0x1000  # room for 8 rings at key + 0x10 r
    keys = [base + 0x10 * r for r in range(nmem)]
    blocks = [[co.fill_synthetic(g, g.block_bytes, 88, r, b) for b in range(nblk)] for r in range(nmem)]
    hdr = (f"HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN {g.nchan_chunk}\nNCHUNK 1\nNCHAN_CHUNK {g.nchan_chunk}\n"
           "NSAMP_DF 1\nBYTE_ORDER LE\nTSAMP 0.84375\n")
    for k in keys + [kout]:
        dada.destroy_ring(k)
    for k in keys:
        dada.create_ring(k, 4, g.block_bytes)
    dada.create_ring(kout, 4, nmem * g.nout * 4)
    out = tmp_path / "power.dada"
    env = dict(os.environ, B2P_STUB_NDEV=str(ndev))
    args = ["-n", str(nmem), "-f", "header"] + (["-G", gather] if gather else [])
    procs = []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([stages["dev" if mode.endswith("_dev") else "host"], "-a", f"{base:x}", "-b",
                                   f"{kout:x}", "-c", str(tmp_path), "-d", "0"] + args,
                                  stderr=subprocess.PIPE, text=True, env=env)]
        for k, bl in zip(keys, blocks):  # 3 blocks and the end of data fit the 4-block rings
            with dada.Hdu(k, "W") as w:
                w.write_header(hdr)
                for b in bl:
                    w.write_block(b.tobytes())
        if want == "refused":  # the stage reads every ring's header, then sets the group up
            _, err = procs[1].communicate(timeout=60)
            assert procs[1].returncode == 1, err
            assert "b2p_group_open" in err and "Duplicate GPU" in err, err
            return
        for p in procs[::-1]:
            _, e = p.communicate(timeout=60)
            assert p.returncode == 0, e[-800:] if isinstance(e, str) else e.decode(errors="replace")[-800:]
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in keys + [kout]:
            dada.destroy_ring(k)
    log = open(str(tmp_path / "paf_baseband2power.log")).read()
    assert f"gather of {nmem} sub-bands to GPU 0 via {want}" in log, log[-1500:]
    for r in range(nmem):
        assert f"member {r}: GPU {r if ndev == 8 else 0} " in log, log[-1500:]
    sp = data.view(np.uint32).reshape(-1, nmem, g.nout)
    assert sp.shape[0] == nblk
    for b in range(nblk):
        for r in range(nmem):
            assert np.array_equal(sp[b, r], co.power(g, blocks[r][b], nthreads=1).view(np.uint32)), (b, r)


def test_stage_recorded_gather_case_async(stages, tmp_path):
    """round 5's failing GPU example (profiles/r05_gpu_suite_gather_flake.txt),
    through the stage's real host code on the asynchronous CPU double (work
    completes 0-3 ms after it is enqueued): -n 2 on the GPU-resident path,
    rings of 6 blocks written by paf_diskdb processes, transfers of 1 and 2
    blocks, int8 11 x 53 ch, 67 frames of 8 samples, npol_out 2, mean.  Each
    of 12 runs must exit 0 with the one common integration of both
    sub-bands equal to the oracle's, the unmatched block of the longer
    transfer logged as skipped."""
    g = npo.Geom(nbit=8, big_endian=0, nchunk=11, nsamp_df=8, nchan_chunk=53, npol_out=2, nsamp_int=536, mean=1)
    nblks = [1, 2]
    blocks = [[co.fill_synthetic(g, g.block_bytes, 1440, r, b) for b in range(nblks[r])] for r in range(2)]
    want = [co.power(g, blocks[r][0], nthreads=2).view(np.uint32) for r in range(2)]
    hdr = (f"HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN {g.nchunk * g.nchan_chunk}\nNCHUNK {g.nchunk}\n"
           f"NCHAN_CHUNK {g.nchan_chunk}\nNSAMP_DF {g.nsamp_df}\nBYTE_ORDER LE\nTSAMP 0.84375\n")
    for r in range(2):
        dada.write_dada_file(str(tmp_path / f"in{r}.dada"), "FILE_HEADER_IS_SKIPPED 1\n",
                             np.concatenate([b.reshape(-1).view(np.uint8) for b in blocks[r]]))
        (tmp_path / f"hdr{r}.txt").write_text(hdr)
    env = dict(os.environ, B2P_STUB_DELAY_US="3000")
    for run in range(12):
        base, kout = _key(), _key()
        keys = [base, base + 0x10]
        for k in keys + [kout]:
            dada.destroy_ring(k)
        for k in keys:
            dada.create_ring(k, 6, g.block_bytes)
        dada.create_ring(kout, 4, 2 * g.nout * 4)
        d = tmp_path / f"run{run}"
        d.mkdir()
        procs = []
        try:
            procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(d / "p.dada")],
                                      stderr=subprocess.PIPE),
                     subprocess.Popen([stages["dev"], "-a", f"{base:x}", "-b", f"{kout:x}", "-c", str(d), "-d", "0",
                                       "-f", "header", "-n", "2", "-p", "2", "-m"], stderr=subprocess.PIPE, env=env)]
            procs += [subprocess.Popen([os.path.join(BIN, "paf_diskdb"), "-a", f"{keys[r]:x}", "-b", str(tmp_path),
                                        "-c", f"in{r}.dada", "-d", str(tmp_path / f"hdr{r}.txt"), "-e", "1"],
                                       stderr=subprocess.PIPE) for r in (run % 2, 1 - run % 2)]
            for p in procs[::-1]:
                _, e = p.communicate(timeout=60)
                assert p.returncode == 0, (run, p.args[0], e.decode(errors="replace")[-800:])
            _, data = dada.read_dada_file(str(d / "p.dada"))
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
            for k in keys + [kout]:
                dada.destroy_ring(k)
        sp = data.view(np.uint32).reshape(-1, 2, g.nout)
        assert sp.shape[0] == 1, run
        assert np.array_equal(sp[0, 0], want[0]) and np.array_equal(sp[0, 1], want[1]), run
        log = (d / "paf_baseband2power.log").read_text()
        assert "FINISH PAF_PROCESS: 1 integrations, 1 skipped, ok" in log, log[-800:]


@pytest.mark.parametrize("mode,fail", [
    ("single", "b2p_push:3"),
    ("single_dev", "b2p_integrate:1,b2p_integrate_n:1"),
    ("single_dev", "b2p_sync:1"),
    ("gathered", "b2p_push:4"),
    ("gathered", "b2p_group_gather:2"),
    ("gathered_dev", "b2p_integrate:2,b2p_integrate_n:2"),
    ("gathered_dev", "b2p_group_gather_async:1"),
    ("gathered_dev", "b2p_group_wait:1"),
    ("split", "b2p_push:3"),
    ("split", "b2p_group_reduce:2"),
])
def test_stage_failure_paths(stages, tmp_path, mode, fail):
    """a HIP error in the middle of a run, injected into the CPU double
    (B2P_STUB_FAIL) in each threading mode: the stage stops every member,
    ends the output transfer (paf_dbdisk exits 0), exits 1 within seconds,
    repeats its ERR line on stderr, and every spectrum it did write equals
    the oracle's -- no hang, no garbage after a failure"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=32, npol_out=1, nsamp_int=256)
    nmem = 1 if mode.startswith("single") else 2
    nblk = 6
    rings = 1 if mode in ("single", "single_dev", "split") else nmem
    base, kout = _key(), _key()
    keys = [base + 0x10 * r for r in range(rings)]
    blocks = [[co.fill_synthetic(g, g.block_bytes, 31, r, b) for b in range(nblk)] for r in range(rings)]
    hdr = (f"HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 32\nNCHUNK 1\nNCHAN_CHUNK 32\nNSAMP_DF 1\n"
           "BYTE_ORDER LE\nTSAMP 0.84375\n")
    for k in keys + [kout]:
        dada.destroy_ring(k)
    for k in keys:
        dada.create_ring(k, nblk + 2, g.block_bytes)  # every block and the end of data fit: writers never wait
    onsub = nmem if mode.startswith("gathered") else 1
    dada.create_ring(kout, 8, onsub * g.nout * 4)
    args = ["-f", "header"]
    if mode.startswith("gathered"):
        args += ["-n", str(nmem), "-G", "copy"]
    if mode == "split":
        args += ["-t", "2", "-G", "copy"]
    out = tmp_path / "power.dada"
    env = dict(os.environ, B2P_STUB_FAIL=fail, B2P_STUB_DELAY_US="300")
    procs = []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([stages["dev" if mode.endswith("_dev") else "host"], "-a", f"{base:x}", "-b",
                                   f"{kout:x}", "-c", str(tmp_path), "-d", "0"] + args,
                                  stderr=subprocess.PIPE, text=True, env=env)]
        for k, bl in zip(keys, blocks):
            with dada.Hdu(k, "W") as w:
                w.write_header(hdr)
                for b in bl:
                    w.write_block(b.tobytes())
        _, err = procs[1].communicate(timeout=60)
        assert procs[1].returncode == 1, err
        _, derr = procs[0].communicate(timeout=60)
        assert procs[0].returncode == 0, derr
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in keys + [kout]:
            dada.destroy_ring(k)
    assert "b2p_cpu_stub: injected failure of" in err, err
    assert "] ERR: " in err and "FAILED, log" in err, err
    log = open(str(tmp_path / "paf_baseband2power.log")).read()
    assert "FAILED" in log.splitlines()[-1], log[-800:]
    sp = data.view(np.uint32).reshape(-1, onsub, g.nout)
    assert sp.shape[0] < nblk
    for b in range(sp.shape[0]):
        for r in range(onsub):
            assert np.array_equal(sp[b, r], co.power(g, blocks[r][b], nthreads=1).view(np.uint32)), (b, r)


_CALLS = ["b2p_push", "b2p_integrate", "b2p_integrate_n", "b2p_finish_async", "b2p_finish_partial_async",
          "b2p_finalize_sums", "b2p_fence", "b2p_fence_wait", "b2p_fence_done", "b2p_flush", "b2p_sync",
          "b2p_memcpy", "b2p_group_gather", "b2p_group_gather_async", "b2p_group_wait", "b2p_group_done",
          "b2p_group_reduce", "b2p_group_sync"]


@pytest.mark.parametrize("san", ["", "_asan"])
@pytest.mark.parametrize("mode", ["single", "single_dev", "gathered", "gathered_dev", "split"])
def test_stage_never_fails_silently(stages, tmp_path, mode, san):
    """every entry point the stage calls, failed at its 1st and its 2nd call
    (B2P_STUB_FAIL), in every threading mode: the stage either never made
    that call (exit 0, every spectrum) or exits 1 within seconds with an ERR
    line on stderr naming what failed, the output transfer ended, and only
    correct spectra written -- no silent exit, no hang.  _asan: the stage
    built with AddressSanitizer and UBSan, so memory a failure path releases
    while queued work still uses it is reported (exit 1 without the ERR
    line the assertion wants, and the report in the message)"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=16, npol_out=1, nsamp_int=128)
    nmem = 1 if mode.startswith("single") else 2
    nblk = 4
    rings = 1 if mode in ("single", "single_dev", "split") else nmem
    onsub = nmem if mode.startswith("gathered") else 1
    blocks = [[co.fill_synthetic(g, g.block_bytes, 47, r, b) for b in range(nblk)] for r in range(rings)]
    want = [[co.power(g, blocks[r][b], nthreads=1).view(np.uint32) for b in range(nblk)] for r in range(rings)]
    hdr = (f"HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 16\nNCHUNK 1\nNCHAN_CHUNK 16\nNSAMP_DF 1\n"
           "BYTE_ORDER LE\nTSAMP 0.84375\n")
    args = ["-f", "header"] + (["-n", str(nmem), "-G", "copy"] if mode.startswith("gathered") else []) \
        + (["-t", "2", "-G", "copy"] if mode == "split" else [])
    failed_runs = 0
    for call in _CALLS:
        for nth in (1, 2):
            base, kout = _key(), _key()
            keys = [base + 0x10 * r for r in range(rings)]
            for k in keys + [kout]:
                dada.destroy_ring(k)
            for k in keys:
                dada.create_ring(k, nblk + 2, g.block_bytes)
            dada.create_ring(kout, nblk + 2, onsub * g.nout * 4)
            d = tmp_path / f"{call}_{nth}"
            d.mkdir()
            env = dict(os.environ, B2P_STUB_FAIL=f"{call}:{nth}", B2P_STUB_DELAY_US="200", **ASAN_ENV)
            procs = []
            try:
                procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o",
                                           str(d / "p.dada")], stderr=subprocess.PIPE),
                         subprocess.Popen([stages[("dev" if mode.endswith("_dev") else "host") + san], "-a",
                                           f"{base:x}",
                                           "-b", f"{kout:x}", "-c", str(d), "-d", "0"] + args,
                                          stderr=subprocess.PIPE, text=True, env=env)]
                for k, bl in zip(keys, blocks):
                    with dada.Hdu(k, "W") as w:
                        w.write_header(hdr)
                        for b in bl:
                            w.write_block(b.tobytes())
                _, err = procs[1].communicate(timeout=60)
                _, derr = procs[0].communicate(timeout=60)
                rc = procs[1].returncode
                assert procs[0].returncode == 0, (call, nth, derr)
                _, data = dada.read_dada_file(str(d / "p.dada"))
            finally:
                for p in procs:
                    if p.poll() is None:
                        p.kill()
                        p.wait()
                for k in keys + [kout]:
                    dada.destroy_ring(k)
            assert "Sanitizer" not in err and "runtime error" not in err, (call, nth, err[-4000:])
            injected = "injected failure of" in err
            sp = data.view(np.uint32).reshape(-1, onsub, g.nout)
            if rc == 0:
                assert not injected, (call, nth, err)  # a failure the stage swallowed
                assert sp.shape[0] == nblk, (call, nth)
            else:
                failed_runs += 1
                assert rc == 1 and injected, (call, nth, rc, err)
                assert "] ERR: " in err and "FAILED, log" in err, (call, nth, err)
                assert sp.shape[0] <= nblk, (call, nth)  # (a failure after the last output still fails the run)
            for b in range(sp.shape[0]):
                for r in range(onsub):
                    assert np.array_equal(sp[b, r], want[r][b]), (call, nth, b, r)
    assert failed_runs >= 4, failed_runs  # the mode's own calls were reached


@pytest.mark.parametrize("mode", ["single", "single_dev", "gathered", "gathered_dev", "split"])
def test_stage_input_ring_removed_under_it(stages, tmp_path, mode):
    """an input ring destroyed while the stage waits on it for its next block
    (its semaphores removed: the wait fails with EIDRM) is not an end of
    data: the stage names the ring and the error in an ERR line on stderr,
    wakes every other member waiting on its own ring, ends the output
    transfer and exits 1 -- within seconds, after writing the spectra of the
    blocks it had, each equal to the oracle's"""
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=16, npol_out=1, nsamp_int=128)
    nmem = 1 if mode.startswith("single") else 2
    rings = 1 if mode in ("single", "single_dev", "split") else nmem
    onsub = nmem if mode.startswith("gathered") else 1
    nblk = 2
    blocks = [[co.fill_synthetic(g, g.block_bytes, 53, r, b) for b in range(nblk)] for r in range(rings)]
    hdr = (f"HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 16\nNCHUNK 1\nNCHAN_CHUNK 16\nNSAMP_DF 1\n"
           "BYTE_ORDER LE\nTSAMP 0.84375\n")
    base, kout = _key(), _key()
    keys = [base + 0x10 * r for r in range(rings)]
    for k in keys + [kout]:
        dada.destroy_ring(k)
    for k in keys:
        dada.create_ring(k, 4, g.block_bytes)
    dada.create_ring(kout, 8, onsub * g.nout * 4)
    args = ["-f", "header"] + (["-n", str(nmem), "-G", "copy"] if mode.startswith("gathered") else []) \
        + (["-t", "2", "-G", "copy"] if mode == "split" else [])
    out = tmp_path / "power.dada"
    procs, writers = [], []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([stages["dev" if mode.endswith("_dev") else "host"], "-a", f"{base:x}", "-b",
                                   f"{kout:x}", "-c", str(tmp_path), "-d", "0"] + args,
                                  stderr=subprocess.PIPE, text=True)]
        for k, bl in zip(keys, blocks):  # the transfers stay open: the stage waits for a third block
            w = dada.Hdu(k, "W")
            writers.append(w)
            w.write_header(hdr)
            for b in bl:
                w.write_block(b.tobytes())
        log = tmp_path / "paf_baseband2power.log"
        t_end = time.time() + 20
        while time.time() < t_end and (not log.exists() or "integration" not in log.read_text()
                                       and "round" not in log.read_text() and "launch" not in log.read_text()):
            time.sleep(0.05)
        time.sleep(0.5)
        assert procs[1].poll() is None  # waiting for the next block
        dada.destroy_ring(keys[0])
        _, err = procs[1].communicate(timeout=30)
        _, derr = procs[0].communicate(timeout=30)
        assert procs[1].returncode == 1, err
        assert procs[0].returncode == 0, derr
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for w in writers:
            try:
                w.close()
            except OSError:
                pass
        for k in keys + [kout]:
            dada.destroy_ring(k)
    assert f"reading input ring {keys[0]:x} failed" in err and "] ERR: " in err, err
    sp = data.view(np.uint32).reshape(-1, onsub, g.nout)
    assert sp.shape[0] == nblk, sp.shape
    for b in range(nblk):
        for r in range(onsub):
            assert np.array_equal(sp[b, r], co.power(g, blocks[r][b], nthreads=1).view(np.uint32)), (b, r)


@pytest.mark.parametrize("gather", [False, True])
def test_pipeline_pins_the_stages_like_the_reference(stages, tmp_path, gather):
    """python -m paf_b2p.pipeline --pin: the stages bound to CPUs as the
    reference's launcher binds them (taskset -c 0 paf_diskdb, taskset -c 1
    paf_baseband2power, dada_dbdisk -b 2; paf-baseband2power.py:68,80,83,
    86-95), chain r shifted by 3r; the stage (here the CPU double's build,
    behind a wrapper that records its CPU list) runs on its CPU and every
    spectrum equals the oracle's"""
    from paf_b2p import pipeline
    from test_gpu_pipeline import write_conf
    nsub = 2
    assert pipeline.pin_cpus(None, 0) == (None, None, None)
    assert [pipeline.pin_cpus(0, r) for r in range(2)] == [(0, 1, 2), (3, 4, 5)]
    assert [pipeline.pin_cpus(1, r, True) for r in range(3)] == [(1, 2, 3), (4, 2, 3), (5, 2, 3)]
    with pytest.raises(ValueError, match="not available"):
        pipeline.run("unused.conf", str(tmp_path), 0, "x.dada", pin=max(os.sched_getaffinity(0)) + 1)
    if not set(range(3 * nsub)) <= os.sched_getaffinity(0):
        pytest.skip("CPUs 0-5 are not all available to this process")
    g = npo.Geom(nbit=8, nchan_chunk=64, nsamp_int=1 << 10)
    nblk = 2
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 64\nTSAMP 0.84375\n")
    files, payloads = [], []
    for r in range(nsub):
        p = co.fill_synthetic(g, g.block_bytes * nblk, 20181105, r, 0)
        f = tmp_path / f"sb{r}.dada"
        dada.write_dada_file(str(f), "x 1\n", p)
        files.append(str(f))
        payloads.append(p)
    kin = _key()
    _key()  # kin + 0x10: the second sub-band's ring
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 10, 1, 256, 64, kin, _key(), str(hfile))
    wrap = tmp_path / "stage.sh"
    wrap.write_text("#!/bin/bash\ngrep Cpus_allowed_list /proc/self/status > \"$B2P_AFF_DIR/$$\"\n"
                    f"exec {stages['host']} \"$@\"\n")
    wrap.chmod(0o755)
    aff = tmp_path / "aff"
    aff.mkdir()
    env_keep = dict(os.environ)
    os.environ["B2P_AFF_DIR"] = str(aff)
    try:
        outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, files, nsub=nsub,
                            gather=gather, timeout=120, stage_exe=str(wrap), pin=0)
    finally:
        os.environ.clear()
        os.environ.update(env_keep)
    seen = sorted(p.read_text().split()[-1] for p in aff.iterdir())
    assert seen == (["1"] if gather else ["1", "4"]), seen
    for r in range(nsub):
        data = dada.read_dada_file(outs[0 if gather else r])[1]
        sp = data.view(np.uint32).reshape(-1, nsub if gather else 1, g.nout)
        assert sp.shape[0] == nblk
        for i in range(nblk):
            blk = payloads[r][i * g.block_bytes:(i + 1) * g.block_bytes]
            assert np.array_equal(sp[i, r if gather else 0], co.power(g, blk).view(np.uint32)), (r, i)


def test_pipeline_memcheck_runs_the_stage_on_the_debug_library(stages, tmp_path):
    """-e 1 (the reference runs the stage under cuda-memcheck,
    paf-baseband2power.py:89-90): the stage's loader finds the bounds-checked
    debug build of libpafb2p (lib/debug) ahead of the release one; the other
    stages keep the default environment"""
    from paf_b2p import pipeline
    from test_gpu_pipeline import write_conf
    assert pipeline.stage_env(0) is None
    dbg = os.path.join(PKG, "lib", "debug")
    assert pipeline.stage_env(1)["LD_LIBRARY_PATH"].split(":")[0] == dbg
    g = npo.Geom(nbit=8, nchan_chunk=64, nsamp_int=1 << 10)
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 64\nTSAMP 0.84375\n")
    p = co.fill_synthetic(g, g.block_bytes, 20181105, 0, 0)
    f = tmp_path / "sb0.dada"
    dada.write_dada_file(str(f), "x 1\n", p)
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 10, 1, 256, 64, _key(), _key(), str(hfile))
    wrap = tmp_path / "stage.sh"
    wrap.write_text(f"#!/bin/bash\necho \"$LD_LIBRARY_PATH\" > {tmp_path}/ldpath\nexec {stages['host']} \"$@\"\n")
    wrap.chmod(0o755)
    outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, str(f), timeout=120, stage_exe=str(wrap), memcheck=1)
    assert (tmp_path / "ldpath").read_text().split(":")[0].strip() == dbg
    sp = dada.read_dada_file(outs[0])[1].view(np.uint32).reshape(-1, g.nout)
    assert sp.shape[0] == 1 and np.array_equal(sp[0], co.power(g, p).view(np.uint32))


def test_pipeline_ctrl_c_lets_the_stages_finish(stages, tmp_path):
    """Ctrl-C on `python -m paf_b2p.pipeline` (SIGINT to its process group,
    as a terminal sends it): the launcher waits for the stages, which got the
    same signal -- paf_diskdb ends its transfer, the stage ends its output
    transfer -- then removes the rings; the spectra written so far are in
    the file, whole, and no process of the run is left"""
    import signal
    import sys
    import textwrap
    g = npo.Geom(nbit=8, nchan_chunk=64, nsamp_int=1 << 10)
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 64\nTSAMP 0.84375\n")
    block = co.fill_synthetic(g, g.block_bytes, 20181105, 0, 0)
    fifo = tmp_path / "obs.fifo"
    os.mkfifo(fifo)
    kin, kout = _key(), _key()
    from test_gpu_pipeline import write_conf
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 10, 1, 256, 64, kin, kout, str(hfile))
    script = tmp_path / "run.py"
    script.write_text(textwrap.dedent(f"""\
        import sys
        sys.path.insert(0, {os.path.join(REPO, "paf-baseband2power_amd")!r})
        from paf_b2p import pipeline
        pipeline.run({str(conf)!r}, {str(tmp_path / "out")!r}, 0, {str(fifo)!r}, timeout=120,
                     stage_exe={stages["host"]!r})
        """))
    run = subprocess.Popen([sys.executable, str(script)], stderr=subprocess.PIPE, text=True,
                           start_new_session=True)
    out = tmp_path / "out" / "power.dada"
    t_end = time.time() + 30
    while True:  # the write end opens once paf_diskdb has the read end open
        try:
            fd = os.open(fifo, os.O_WRONLY | os.O_NONBLOCK)
            break
        except OSError:
            assert run.poll() is None and time.time() < t_end, run.communicate()[1][-2000:]
            time.sleep(0.05)
    os.set_blocking(fd, True)
    f = os.fdopen(fd, "wb")
    try:
        f.write(b"H" * 4096 + block.tobytes() + block.tobytes()[: g.block_bytes // 2])
        f.flush()
        t_end = time.time() + 30
        while (not out.exists() or out.stat().st_size < 4096 + g.nout * 4) and time.time() < t_end:
            time.sleep(0.05)
        time.sleep(0.3)
        assert run.poll() is None
        os.killpg(run.pid, signal.SIGINT)
        _, err = run.communicate(timeout=60)
    finally:
        f.close()
        if run.poll() is None:
            os.killpg(run.pid, signal.SIGKILL)
            run.wait()
    assert "KeyboardInterrupt" in err, err[-2000:]
    with pytest.raises(ProcessLookupError):  # every process of the run has ended
        os.killpg(run.pid, 0)
    log = (tmp_path / "out" / "paf_baseband2power.log").read_text()
    assert "FINISH PAF_PROCESS: 1 integrations, 0 skipped, ok" in log, log[-800:]  # stopped, not failed
    sp = dada.read_dada_file(str(out))[1].view(np.uint32).reshape(-1, g.nout)
    assert sp.shape[0] == 1 and np.array_equal(sp[0], co.power(g, block).view(np.uint32))
    assert not dada.destroy_ring(kin) and not dada.destroy_ring(kout)  # the launcher removed them


_WRITER = """
import sys, time
sys.path.insert(0, {pkg!r})
import numpy as np
from paf_b2p import dada
key, nblk, header, path = int(sys.argv[1], 16), int(sys.argv[2]), sys.argv[3] == "1", sys.argv[4]
data = np.fromfile(path, dtype=np.uint8)
w = dada.Hdu(key, "W")
if header:
    w.write_header(open(path + ".hdr").read())
for b in np.split(data, nblk):
    w.write_block(b.tobytes())
if sys.argv[5] == "hold":
    print("written", flush=True)
    time.sleep(120)  # the transfer stays open until this process is killed
w.close()            # the end of data
"""


@pytest.mark.parametrize("mode,grace,resume", [("single", 1.0, False), ("single_dev", 1.0, False),
                                               ("gathered", 1.0, False), ("single", 0, False),
                                               ("single_dev", 4.0, True)])
def test_stage_notices_a_writer_that_went_away(stages, tmp_path, mode, grace, resume):
    """-W S: a writer killed mid-transfer (SIGKILL: no end of data; the kernel
    undoes its write lock) leaves the stage's transfer open with no writer.
    After S s of that the stage logs "its writer went away", wakes every
    member and exits 1, the spectra of the blocks it had written and whole.
    Without -W it waits (PSRDADA lets a new writer take an open transfer
    on); and a writer that does so within the grace period carries the run
    to its normal end"""
    import signal
    import sys
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=16, npol_out=1, nsamp_int=128)
    rings = 2 if mode == "gathered" else 1
    blocks = [[co.fill_synthetic(g, g.block_bytes, 61, r, b) for b in range(3)] for r in range(rings)]
    hdr = ("HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 16\nNCHUNK 1\nNCHAN_CHUNK 16\nNSAMP_DF 1\n"
           "BYTE_ORDER LE\nTSAMP 0.84375\n")
    base, kout = _key(), _key()
    keys = [base + 0x10 * r for r in range(rings)]
    for k in keys + [kout]:
        dada.destroy_ring(k)
    for k in keys:
        dada.create_ring(k, 6, g.block_bytes)
    dada.create_ring(kout, 8, rings * g.nout * 4)
    script = tmp_path / "writer.py"
    script.write_text(_WRITER.format(pkg=PKG))
    files = []
    for r in range(rings):
        f = tmp_path / f"in{r}.u8"
        np.concatenate([b.reshape(-1).view(np.uint8) for b in blocks[r][:2]]).tofile(f)
        (tmp_path / f"in{r}.u8.hdr").write_text(hdr)
        files.append(f)
    args = ["-f", "header"] + (["-n", "2", "-G", "copy"] if mode == "gathered" else []) \
        + (["-W", str(grace)] if grace else [])
    out = tmp_path / "power.dada"
    procs, writers = [], []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([stages["dev" if mode.endswith("_dev") else "host"], "-a", f"{base:x}", "-b",
                                   f"{kout:x}", "-c", str(tmp_path), "-d", "0"] + args,
                                  stderr=subprocess.PIPE, text=True)]
        for k, f in zip(keys, files):  # two blocks each, the transfers left open
            writers.append(subprocess.Popen([sys.executable, str(script), f"{k:x}", "2", "1", str(f), "hold"],
                                            stdout=subprocess.PIPE, text=True))
        for w in writers:
            assert w.stdout.readline().strip() == "written"
        t_end = time.time() + 30
        while (not out.exists() or out.stat().st_size < 4096 + 2 * rings * g.nout * 4) and time.time() < t_end:
            time.sleep(0.05)
        writers[0].send_signal(signal.SIGKILL)  # ring 0's writer dies mid-transfer
        writers[0].wait()
        t_kill = time.time()
        if resume:  # a new writer takes the open transfer on: one more block, then the end of data
            time.sleep(0.5)
            f3 = tmp_path / "in0b.u8"
            blocks[0][2].reshape(-1).view(np.uint8).tofile(f3)
            assert subprocess.run([sys.executable, str(script), f"{keys[0]:x}", "1", "0", str(f3), "end"],
                                  timeout=30).returncode == 0
        if grace and not resume:
            _, err = procs[1].communicate(timeout=30)
            assert procs[1].returncode == 1, err
            assert time.time() - t_kill >= grace - 0.1  # not before the grace period
            assert f"input ring {keys[0]:x}: its writer went away" in err and "] ERR: " in err, err
        elif resume:
            _, err = procs[1].communicate(timeout=30)
            assert procs[1].returncode == 0, err
        else:  # no -W: still waiting for a writer
            time.sleep(2.0)
            assert procs[1].poll() is None
            procs[1].send_signal(signal.SIGTERM)
            _, err = procs[1].communicate(timeout=30)
            assert procs[1].returncode == 0, err
        _, derr = procs[0].communicate(timeout=30)
        assert procs[0].returncode == 0, derr
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs + writers:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in keys + [kout]:
            dada.destroy_ring(k)
    sp = data.view(np.uint32).reshape(-1, rings, g.nout)
    n = 3 if resume else 2
    assert sp.shape[0] == n, (sp.shape, err[-1500:])
    for b in range(n):
        for r in range(rings):
            assert np.array_equal(sp[b, r], co.power(g, blocks[r][b], nthreads=1).view(np.uint32)), (b, r)
