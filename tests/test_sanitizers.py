"""Host-code sanitizers (CPU).  GPU sanitizers are not available on the test
pool; these cover the C code around the kernels:
  * the DADA layer with ASan+UBSan and with TSan: tests/c/ring_stress.c
    (writer + 2 reader threads, EOD, header edits) and tests/c/ring_surface.c
    (deferred start of data, resets, a viewer, tell / seek, read depth 2);
  * the stage's worker threads (paf_baseband2power.c) under TSan, linked
    against a CPU test double of libpafb2p (tests/c/b2p_cpu_stub.c);
  * paf_capture's receive and sorting threads under TSan."""
import os
import subprocess

import pytest

from conftest import REPO

SRC = [os.path.join(REPO, "paf-baseband2power_amd", "csrc", "dada", f)
       for f in ("dada_ring.c", "dada_query.c", "dada_device.c", "ascii_header.c")]
DRIVER = os.path.join(REPO, "tests", "c", "ring_stress.c")


@pytest.mark.parametrize("san,key", [("address,undefined", "7c10"), ("thread", "7c20")])
def test_dada_layer_under_sanitizer(tmp_path, san, key):
    """writer + two readers (depth 1 and 2) through a 3-block ring"""
    exe = tmp_path / "ring_stress"
    cmd = ["gcc", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", f"-fsanitize={san}",
           "-fno-omit-frame-pointer", "-I", os.path.join(REPO, "include"), DRIVER, *SRC,
           "-o", str(exe), "-pthread", "-ldl"]
    subprocess.run(cmd, check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe), key], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "errors 0" in r.stdout
    assert "runtime error" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr


@pytest.mark.parametrize("san,key", [("address,undefined", "7c30"), ("thread", "7c40")])
def test_ring_surface_under_sanitizer(tmp_path, san, key):
    """round 3's libpafdada surface (tests/c/ring_surface.c) under ASan+UBSan
    and TSan: a deferred start of data (ipcio 'w', ipcio_start mid-block,
    ipcio_stop) three times, a writer ipcbuf_reset, a viewer attached during
    a transfer, ipcbuf_hard_reset between transfers, ipcio_tell / seek, two
    readers, one holding two blocks at read depth 2 (set before its read
    lock), every transfer checked byte for byte"""
    exe = tmp_path / "ring_surface"
    subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror",
                    f"-fsanitize={san}", "-fno-omit-frame-pointer", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c", "ring_surface.c"), *SRC, "-o", str(exe), "-pthread",
                    "-ldl", "-lm"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe), key], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "errors 0" in r.stdout
    assert "runtime error" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr


STAGE = os.path.join(REPO, "paf-baseband2power_amd", "csrc", "host", "paf_baseband2power.c")
STUB = os.path.join(REPO, "tests", "c", "b2p_cpu_stub.c")
DADA_SRC = [os.path.join(REPO, "paf-baseband2power_amd", "csrc", "dada", f)
            for f in ("dada_ring.c", "dada_query.c", "dada_device.c", "ascii_header.c", "df_header.c")]


def _stage_tsan(tmp_path, as_device: bool) -> str:
    """paf_baseband2power built with -fsanitize=thread against the CPU test
    double of libpafb2p (tests/c/b2p_cpu_stub.c) and libpafdada's sources;
    as_device: host rings take the GPU-resident paths (test-only
    -DB2P_TEST_HOST_RING_AS_DEVICE), i.e. worker_gather_dev for -n N and
    run_device_pipelined for one sub-band"""
    exe = tmp_path / ("stage_tsan_dev" if as_device else "stage_tsan")
    defs = ["-DB2P_TEST_HOST_RING_AS_DEVICE"] if as_device else []
    subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror",
                    "-fsanitize=thread", "-fno-omit-frame-pointer", "-I", os.path.join(REPO, "include"),
                    *defs, STAGE, STUB, *DADA_SRC, "-o", str(exe), "-pthread", "-ldl", "-lm"], check=True)
    return str(exe)


@pytest.mark.parametrize("mode", ["gathered", "gathered_dev", "split", "single_dev"])
def test_stage_threads_under_tsan(tmp_path, mode):
    """The stage's worker threads under ThreadSanitizer (CPU, no GPU):
      gathered      -n 3 over host rings (worker: one thread per sub-band,
                    barriers per round, the root gathers and writes)
      gathered_dev  -n 3 taking the GPU-resident path (worker_gather_dev:
                    rounds of queued blocks, launches in flight, the root's
                    asynchronous gathers, the real-time drain)
      split         -t 2 (worker_split: shares of one host block, exact
                    partials reduced by the root)
      single_dev    one sub-band on the GPU-resident path (run_device_pipelined)
    Producers are the normal paf_diskdb builds; every spectrum is checked
    against the C oracle, so the threads also moved the right data."""
    import numpy as np
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_c as co
    import b2p_oracle as npo
    from paf_b2p import dada, pipeline
    from test_gpu_pipeline import write_conf
    seed = 20181105
    exe = _stage_tsan(tmp_path, as_device=mode.endswith("_dev"))
    g = npo.Geom(nbit=8, nchan_chunk=64, nsamp_int=1 << 10)
    nblk = 7   # more blocks than the 3-block ring: producers wait, rounds overlap
    nsub = 3 if mode.startswith("gathered") else 1
    hfile = tmp_path / "hdr.txt"
    hfile.write_text("HEADER DADA\nHDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 64\nTSAMP 0.84375\n")
    files, payloads = [], []
    for r in range(nsub):
        p = co.fill_synthetic(g, g.block_bytes * nblk, seed, r, 3)
        f = tmp_path / f"sb{r}.dada"
        dada.write_dada_file(str(f), "x 1\n", p)
        files.append(str(f))
        payloads.append(p)
    kin = 0x6a10 + (os.getpid() % 64) * 0x100 + ["gathered", "gathered_dev", "split", "single_dev"].index(mode) * 0x40
    conf = tmp_path / "p.conf"
    write_conf(conf, 1 << 10, 1, 256, 64, kin, kin + 0x8000, str(hfile))
    env_keep = dict(os.environ)
    os.environ["TSAN_OPTIONS"] = "halt_on_error=1 second_deadlock_stack=1"
    # the CPU double's asynchronous stream model: work completes up to 0.5 ms
    # after it is enqueued, so fences, held blocks and gathers meet late work
    os.environ["B2P_STUB_DELAY_US"] = "500"
    try:
        if nsub > 1:
            outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, files, nsub=nsub, gather=True,
                                timeout=240, stage_exe=exe)
        else:
            outs = pipeline.run(str(conf), str(tmp_path / "out"), 0, files[0], split=2 if mode == "split" else 1,
                                timeout=240, stage_exe=exe)
    finally:
        os.environ.clear()
        os.environ.update(env_keep)
    hdr, data = dada.read_dada_file(outs[0])
    sp = data.view(np.float32).reshape(-1, nsub, g.nout)
    assert sp.shape[0] == nblk
    for i in range(nblk):
        for r in range(nsub):
            blk = payloads[r][i * g.block_bytes:(i + 1) * g.block_bytes]
            assert np.array_equal(sp[i, r].view(np.uint32), co.power(g, blk).view(np.uint32)), (i, r)
    log = open(str(tmp_path / "out" / "paf_baseband2power.log")).read()
    assert "WARNING: ThreadSanitizer" not in log
    assert f"FINISH PAF_PROCESS: {nblk} integrations, 0 skipped, ok" in log, log[-2000:]
    if mode == "gathered_dev":
        assert "queued blocks in rounds" in log
    if mode == "split":
        assert "reduce of 2 time shares" in log


def test_capture_receive_threads_under_tsan(tmp_path):
    """paf_capture's receive threads and the sorting thread (slot rings with
    C11 acquire/release, the stop flag) under ThreadSanitizer, in record
    mode (-o: no GPU).  The HIP library is replaced at link time by stubs of
    the b2p_* entry points the capture references; record mode calls none."""
    import re
    import sys
    import time
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from test_capture import make_stream
    from paf_b2p import dada
    host = os.path.join(REPO, "paf-baseband2power_amd", "csrc", "host", "paf_capture.c")
    inc = ["-I", os.path.join(REPO, "include")]
    obj = tmp_path / "cap.o"
    subprocess.run(["gcc", "-c", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", "-fsanitize=thread",
                    *inc, host, "-o", str(obj)], check=True)
    und = subprocess.run(["nm", "-u", str(obj)], capture_output=True, text=True, check=True).stdout
    b2p = sorted({ln.split()[-1] for ln in und.splitlines() if ln.split()[-1].startswith("b2p_")
                  and not ln.split()[-1].startswith("b2p_df_")})
    assert "b2p_assemble" in b2p
    stub = tmp_path / "stub.c"
    stub.write_text("".join(f"int {s}(void) {{ return -5; }}\n" for s in b2p))
    dsrc = [os.path.join(REPO, "paf-baseband2power_amd", "csrc", "dada", f)
            for f in ("dada_ring.c", "dada_query.c", "dada_device.c", "ascii_header.c", "df_header.c")]
    exe = tmp_path / "paf_capture_tsan"
    subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", "-fsanitize=thread", *inc,
                    str(obj), str(stub), *dsrc, "-o", str(exe), "-pthread", "-ldl", "-lm"], check=True)
    g, _, df, ck = make_stream(tmp_path, nblk=6)
    port = 24000 + (os.getpid() % 500) * 8
    out, outc = tmp_path / "r.df", tmp_path / "r.chunks"
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    cap = subprocess.Popen([str(exe), "-o", str(out), "-O", str(outc), "-P", str(port), "-N", "3",
                            "-R", "3", "-m", "freq:1300", "-t", "1"], stderr=subprocess.PIPE, text=True,
                           env=env)
    time.sleep(1.0)
    snd = subprocess.run([os.path.join(dada.BIN_DIR, "paf_dfsend"), "-i", str(df), "-k", str(ck),
                          "-P", str(port), "-N", "3", "-T", "3", "-r", "200"], capture_output=True, text=True)
    assert snd.returncode == 0, snd.stderr
    _, err = cap.communicate(timeout=120)
    assert cap.returncode == 0, err[-3000:]
    assert "WARNING: ThreadSanitizer" not in err, err[-3000:]
    n = os.path.getsize(df) // 7232
    assert re.search(rf"capture: {n} frames received \(0 not frames\)", err), err[-2000:]
    assert "3 receive thread(s) over 3 port(s)" in err


def test_staging_and_addressing_model_under_asan(tmp_path):
    """the library's own index arithmetic (csrc/b2p_plan.h: launch shape,
    lane channels, row ownership, ragged row, staging chunks) compiled on
    the CPU under ASan+UBSan and replayed over 300 random layouts, CU
    counts, knobs, staging sizes and push cuts (tests/c/plan_model.cpp):
    host spans and staging buffers are exact-size allocations, every load
    is in bounds, every vector is read exactly once, every output slot is
    < nout, and the sums equal the C oracle's"""
    obj = tmp_path / "orc.o"
    exe = tmp_path / "plan_model"
    san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]
    subprocess.run(["gcc", "-O1", "-g", *san, "-c", os.path.join(REPO, "oracle", "b2p_oracle.c"),
                    "-I", os.path.join(REPO, "oracle"), "-o", str(obj)], check=True)
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-Wextra", "-Wno-unknown-pragmas", *san,
                    "-I", os.path.join(REPO, "oracle"), "-I", os.path.join(REPO, "paf-baseband2power_amd", "csrc"),
                    os.path.join(REPO, "tests", "c", "plan_model.cpp"), str(obj), "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(exe), "300", "20181105"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "plan model: 300 cases ok" in r.stdout, r.stdout


def test_read_depth_survives_a_view_under_asan(tmp_path):
    """a handle that sets read depth 2, views a block (view position 1) and
    then locks for reading still holds two blocks at once: the depth lives
    in viewbuf's top byte, apart from the view position (advisor, round 4:
    it used to read back as the old position's low byte;
    tests/c/ring_depth_view.c)"""
    exe = tmp_path / "ring_depth_view"
    subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-D_GNU_SOURCE", "-Wall", "-Wextra", "-Werror",
                    "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c", "ring_depth_view.c"), *SRC, "-o", str(exe), "-pthread",
                    "-ldl", "-lm"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(exe), "7c50"], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "errors 0" in r.stdout


@pytest.mark.parametrize("as_device", [False, True])
def test_stage_stop_signal_under_tsan(tmp_path, as_device):
    """SIGTERM to the stage while its -n 2 members wait on their rings, under
    ThreadSanitizer: the flag the handler sets is read by every member
    thread (a C11 atomic since round 6: as a volatile sig_atomic_t it was a
    data race TSan reported), the waits give up, the output transfer ends,
    exit 0 with every spectrum so far"""
    import signal
    import sys
    import time
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_c as co
    import b2p_oracle as npo
    from paf_b2p import dada
    exe = _stage_tsan(tmp_path, as_device=as_device)
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=16, npol_out=1, nsamp_int=128)
    base = 0x6e00 + (os.getpid() % 64) * 0x40 + (0x20 if as_device else 0)
    keys, kout = [base, base + 0x10], base + 4
    for k in keys + [kout]:
        dada.destroy_ring(k)
    for k in keys:
        dada.create_ring(k, 4, g.block_bytes)
    dada.create_ring(kout, 8, 2 * g.nout * 4)
    blocks = [co.fill_synthetic(g, g.block_bytes, 29, r, 0) for r in range(2)]
    out = tmp_path / "power.dada"
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1", B2P_STUB_DELAY_US="300")
    procs, writers = [], []
    try:
        procs = [subprocess.Popen([os.path.join(dada.BIN_DIR, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([exe, "-a", f"{base:x}", "-b", f"{kout:x}", "-c", str(tmp_path), "-d", "0",
                                   "-f", "int8:16", "-n", "2", "-G", "copy"], stderr=subprocess.PIPE, text=True,
                                  env=env)]
        for k, b in zip(keys, blocks):  # one block each; the transfers stay open
            w = dada.Hdu(k, "W")
            writers.append(w)
            w.write_header("HDR_SIZE 4096\nTSAMP 0.84375\n")
            w.write_block(b.tobytes())
        t_end = time.time() + 30
        while (not out.exists() or out.stat().st_size < 4096 + 2 * g.nout * 4) and time.time() < t_end:
            time.sleep(0.05)
        time.sleep(0.3)
        procs[1].send_signal(signal.SIGTERM)
        _, err = procs[1].communicate(timeout=30)
        _, derr = procs[0].communicate(timeout=30)
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
    assert "WARNING: ThreadSanitizer" not in err, err[-4000:]
    assert procs[1].returncode == 0 and procs[0].returncode == 0, (err[-1500:], derr)
    sp = dada.read_dada_file(str(out))[1].view(np.uint32).reshape(-1, 2, g.nout)
    assert sp.shape[0] == 1
    for r in range(2):
        assert np.array_equal(sp[0, r], co.power(g, blocks[r]).view(np.uint32))
