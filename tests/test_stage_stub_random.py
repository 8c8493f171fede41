"""CPU property test of the stage's orchestration (no GPU): the real
`paf_baseband2power` host code, linked against the CPU test double of
libpafb2p (tests/c/b2p_cpu_stub.c: exact sums, every call finished on
return) and libpafdada's sources, between PSRDADA writers in this process
and `paf_dbdisk`.  Random layouts (int8 / int16 LE, what the stub handles),
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
                                                            "ascii_header.c")]
_SCALE = int(os.environ.get("B2P_HYPOTHESIS_SCALE", "1"))
_SEED = os.environ.get("B2P_HYPOTHESIS_SEED")
_KEY = [0x5a00 + (os.getpid() % 64) * 0x80]
# B2P_STAGE_TSAN=1: the stage built with ThreadSanitizer (halt on the first
# report), so the random cases also hunt data races in its threads
_TSAN = ["-fsanitize=thread", "-fno-omit-frame-pointer"] if os.environ.get("B2P_STAGE_TSAN") else []


@pytest.fixture(scope="module")
def stages(tmp_path_factory):
    d = tmp_path_factory.mktemp("stub_stage")
    out = {}
    for name, defs in (("host", []), ("dev", ["-DB2P_TEST_HOST_RING_AS_DEVICE"])):
        exe = d / f"stage_{name}"
        subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror",
                        *_TSAN, "-I", os.path.join(REPO, "include"), *defs, STAGE, STUB, *DADA_SRC, "-o",
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
    g = npo.Geom(nbit=nbit, nchunk=nchunk, nsamp_df=nsamp_df, nchan_chunk=ncc,
                 npol_out=draw(st.sampled_from([1, 2])), nsamp_int=nframes * nsamp_df,
                 mean=int(draw(st.booleans())))
    nblk = draw(st.integers(1, 10))
    shorter = [draw(st.integers(0, 2)) for _ in range(nmem)] if mode.startswith("gathered") else [0]
    return dict(g=g, mode=mode, nmem=nmem, nbufs=draw(st.integers(2, 6)), nblk=nblk,
                nblks=[max(1, nblk - d) for d in shorter],
                short=mode in ("single", "single_dev", "split") and nframes > 1 and draw(st.booleans()),
                sync=mode in ("single", "gathered") and draw(st.booleans()),
                seed=draw(st.integers(0, 2 ** 32 - 1)))


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
           f"NCHUNK {g.nchunk}\nNCHAN_CHUNK {g.nchan_chunk}\nNSAMP_DF {g.nsamp_df}\nBYTE_ORDER LE\n"
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
    exe = stages["dev" if mode.endswith("_dev") else "host"]
    out = tmp / "power.dada"
    procs, errs = [], []
    try:
        env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
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
    if len(set(nblks)) == 1:  # (the GPU-resident gather also logs the longer transfer's unmatched block)
        assert ("partial integration skipped" in log) == case["short"], (case, log[-600:])


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
