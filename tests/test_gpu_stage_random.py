"""Property test of the stage end to end: `paf_baseband2power` between a
PSRDADA writer (this process for host rings, `paf_diskdb` processes for
GPU-resident rings) and `paf_dbdisk`, on layouts the input header
describes (NBIT, NCHAN, NCHUNK, NCHAN_CHUNK, NSAMP_DF, BYTE_ORDER; the
reference's TFTFP family), with random ring depths, block counts, output
pols, sum or mean, GPU-resident or host rings, pipelined or one block at a
time (-S), and sometimes a short last block (end of data mid-integration:
skipped).  Every output spectrum equals the oracle's of its block, bit for
bit, and the output header describes it.

B2P_HYPOTHESIS_SCALE / B2P_HYPOTHESIS_SEED scale or reseed the run
(tests/test_gpu_random_layouts.py)."""
import os
import subprocess

import numpy as np
import pytest
from hypothesis import HealthCheck, example, given, seed, settings
from hypothesis import strategies as st

import b2p_oracle as npo
import oracle_c as co
from paf_b2p import dada
from test_gpu_device_ring import BIN, _wait, fresh_key

pytestmark = pytest.mark.gpu
_SCALE = int(os.environ.get("B2P_HYPOTHESIS_SCALE", "1"))
_SEED = os.environ.get("B2P_HYPOTHESIS_SEED")
# B2P_STAGE_WRITER=inproc: every GPU-resident ring is written from THIS
# process (hipIpcOpenMemHandle + hipMemcpy into the imported blocks), as in
# round 4's seed-9090 hunt, instead of from paf_diskdb processes
_INPROC = os.environ.get("B2P_STAGE_WRITER") == "inproc"


@st.composite
def cases(draw):
    nbit = draw(st.sampled_from([8, 16]))
    be = draw(st.booleans()) if nbit == 16 else False
    word = 4 * nbit // 8
    nchunk = draw(st.integers(1, 16))
    ncc = draw(st.integers(1, 64))
    base = 1
    while (base * ncc * word) % 16:
        base *= 2
    nsamp_df = base * draw(st.integers(1, 2))
    npol_out = draw(st.sampled_from([1, 2]))
    frame = nchunk * nsamp_df * ncc * word
    nframes = draw(st.integers(1, max(1, (2 << 20) // frame)))
    g = npo.Geom(nbit=nbit, big_endian=int(be), nchunk=nchunk, nsamp_df=nsamp_df, nchan_chunk=ncc,
                 npol_out=npol_out, nsamp_int=nframes * nsamp_df, mean=int(draw(st.booleans())))
    device = draw(st.booleans())
    return dict(g=g, nbufs=draw(st.integers(2, 6)), nblk=draw(st.integers(1, 12)),
                short=nframes > 1 and draw(st.booleans()), device=device, sync=device and draw(st.booleans()),
                seed=draw(st.integers(0, 2 ** 32 - 1)))


def _diskdb_writer(tmp, key, hdr, blocks, short_bytes=None):
    """write blocks (plus an optional short tail) to a DADA file and start a
    paf_diskdb process that feeds it into ring `key`: GPU-resident rings are
    written from their own process, as in production, so this test process
    never imports a ring block's IPC handle"""
    name = f"in_{key:x}.dada"
    parts = [b.reshape(-1).view(np.uint8) for b in blocks]
    if short_bytes is not None:
        parts.append(parts[0][:short_bytes])
    dada.write_dada_file(str(tmp / name), "FILE_HEADER_IS_SKIPPED 1\n", np.concatenate(parts))
    (tmp / f"hdr_{key:x}.txt").write_text(hdr)
    return subprocess.Popen([os.path.join(BIN, "paf_diskdb"), "-a", f"{key:x}", "-b", str(tmp), "-c", name,
                             "-d", str(tmp / f"hdr_{key:x}.txt"), "-e", "1"], stderr=subprocess.PIPE)


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=24 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(cases())
def test_stage_random_layouts_rings_and_flags(gpu, tmp_path_factory, case):
    g, nblk = case["g"], case["nblk"]
    tmp = tmp_path_factory.mktemp("stage")
    blocks = [co.fill_synthetic(g, g.block_bytes, case["seed"], 3, b) for b in range(nblk)]
    hdr = (f"HDR_SIZE 4096\nNBIT {g.nbit}\nNDIM 2\nNPOL 2\nNCHAN {g.nchunk * g.nchan_chunk}\n"
           f"NCHUNK {g.nchunk}\nNCHAN_CHUNK {g.nchan_chunk}\nNSAMP_DF {g.nsamp_df}\n"
           f"BYTE_ORDER {'BE' if g.big_endian else 'LE'}\nTSAMP 0.84375\n")
    kin, kout = fresh_key(), fresh_key()
    dada.create_ring(kin, case["nbufs"], g.block_bytes, device=0 if case["device"] else -1)
    dada.create_ring(kout, 4, g.nout * 4)
    out = tmp / "power.dada"
    procs = []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp), "-d", "0", "-f", "header", "-p", str(g.npol_out)]
                                  + (["-m"] if g.mean else []) + (["-S"] if case["sync"] else []),
                                  stderr=subprocess.PIPE)]
        if case["device"] and not _INPROC:  # end of data part-way through an integration: a short tail
            procs.append(_diskdb_writer(tmp, kin, hdr, blocks, g.frame_bytes if case["short"] else None))
        else:
            with dada.Hdu(kin, "W") as w:
                w.write_header(hdr)
                for b in blocks:
                    w.write_block(b.tobytes())
                if case["short"]:  # end of data part-way through an integration
                    w.write_block(blocks[0][: g.frame_bytes].tobytes())
        _wait(procs, timeout=120)
        ohdr, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
    sp = data.view(np.uint32).reshape(-1, g.nout)
    assert sp.shape[0] == nblk, case
    for b in range(nblk):
        assert np.array_equal(sp[b], co.power(g, blocks[b], nthreads=8).view(np.uint32)), (case, b)
    assert dada.header_get(ohdr, "NBIT", "%d") == 32
    assert dada.header_get(ohdr, "NPOL", "%d") == g.npol_out
    assert dada.header_get(ohdr, "NCHAN", "%d") == g.nchunk * g.nchan_chunk
    log = open(str(tmp / "paf_baseband2power.log")).read()
    assert f"FINISH PAF_PROCESS: {nblk} integrations" in log, log[-600:]
    assert ("partial integration skipped" in log) == case["short"], log[-600:]


def _run_stage(tmp, g, keys, rings_blocks, stage_args, device, nbufs, out_nsub, short=(), inproc=False):
    """create one input ring per key, start paf_dbdisk and the stage, write
    each ring's blocks (host rings: from a thread of this process each;
    GPU-resident rings: from a paf_diskdb process each, or with inproc from
    a thread of this process each, through the imported IPC handles), and
    return (output header, spectra [n, out_nsub, nout] as uint32, stage
    log)"""
    import threading
    hdr = (f"HDR_SIZE 4096\nNBIT {g.nbit}\nNDIM 2\nNPOL 2\nNCHAN {g.nchunk * g.nchan_chunk}\n"
           f"NCHUNK {g.nchunk}\nNCHAN_CHUNK {g.nchan_chunk}\nNSAMP_DF {g.nsamp_df}\n"
           f"BYTE_ORDER {'BE' if g.big_endian else 'LE'}\nTSAMP 0.84375\n")
    kout = fresh_key()
    for k in keys:
        dada.destroy_ring(k)
        dada.create_ring(k, nbufs, g.block_bytes, device=0 if device else -1)
    dada.create_ring(kout, 4, out_nsub * g.nout * 4)
    out = tmp / "power.dada"
    procs, errs = [], []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{keys[0]:x}", "-b",
                                   f"{kout:x}", "-c", str(tmp), "-d", "0", "-f", "header"] + stage_args,
                                  stderr=subprocess.PIPE)]

        def writer(k, blocks, sh):
            try:
                with dada.Hdu(k, "W") as w:
                    w.write_header(hdr)
                    for b in blocks:
                        w.write_block(b.tobytes())
                    if sh:
                        w.write_block(blocks[0][: g.frame_bytes].tobytes())
            except Exception as e:  # noqa: BLE001 -- reported below
                errs.append(e)
        inproc = inproc or _INPROC
        if device and not inproc:  # GPU-resident rings: one paf_diskdb process per ring
            procs += [_diskdb_writer(tmp, k, hdr, bl, g.frame_bytes if k in short else None)
                      for k, bl in zip(keys, rings_blocks)]
        ths = [] if device and not inproc else [threading.Thread(target=writer, args=(k, bl, k in short))
                                                for k, bl in zip(keys, rings_blocks)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(120)
        assert not errs, errs
        _wait(procs, timeout=120)
        ohdr, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in list(keys) + [kout]:
            dada.destroy_ring(k)
    return ohdr, data.view(np.uint32).reshape(-1, out_nsub, g.nout), open(str(tmp / "paf_baseband2power.log")).read()


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=10 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(cases(), st.integers(2, 3), st.lists(st.integers(0, 2), min_size=3, max_size=3))
# round 5's one failing example (profiles/r05_gpu_suite_gather_flake.txt:
# the stage exited 1 with nothing on stderr), pinned: -n 2 on device rings
# written by paf_diskdb, transfers of 1 and 2 blocks, nbufs 6, async rounds
@example(case=dict(g=npo.Geom(nbit=8, big_endian=0, nchunk=11, nsamp_df=8, nchan_chunk=53, npol_out=2,
                              nsamp_int=536, mean=1), nbufs=6, nblk=2, short=False, device=True, sync=False,
                   seed=1440), nsub=2, shorter=[2, 0, 0])
def test_stage_random_gathered_subbands(gpu, tmp_path_factory, case, nsub, shorter):
    """-n 2 / 3: sub-band r on ring key + 0x10 r with its own data; the
    transfers may end at different blocks -- the stage stops at the shortest,
    every output block holds each sub-band's spectrum of the same round"""
    g = case["g"]
    tmp = tmp_path_factory.mktemp("gather")
    nblks = [max(1, case["nblk"] - shorter[r]) for r in range(nsub)]
    base = fresh_key()
    keys = [base + 0x10 * r for r in range(nsub)]
    blocks = [[co.fill_synthetic(g, g.block_bytes, case["seed"], r, b) for b in range(nblks[r])]
              for r in range(nsub)]
    args = ["-n", str(nsub), "-p", str(g.npol_out)] + (["-m"] if g.mean else []) + (["-S"] if case["sync"] else [])
    # rings that outlive the stage take every block they are given: the
    # writer of a longer transfer must not wait on a reader that has left
    nbufs = case["nbufs"] if len(set(nblks)) == 1 else max(case["nbufs"], max(nblks) + 1)
    ohdr, sp, log = _run_stage(tmp, g, keys, blocks, args, case["device"], nbufs, nsub)
    n = min(nblks)
    assert sp.shape[0] == n, (case, nblks, log[-600:])
    for b in range(n):
        for r in range(nsub):
            assert np.array_equal(sp[b, r], co.power(g, blocks[r][b], nthreads=8).view(np.uint32)), (case, b, r)
    assert dada.header_get(ohdr, "NSUBBAND", "%d") == nsub


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=10 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(cases(), st.integers(2, 3), st.lists(st.integers(0, 2), min_size=3, max_size=3))
def test_stage_random_gathered_subbands_inproc_writers(gpu, tmp_path_factory, case, nsub, shorter):
    """as test_stage_random_gathered_subbands, on GPU-resident rings only,
    written by 2-3 threads of THIS long-lived process through the imported
    IPC handles (dada.Hdu.write_block -> ipcbuf copy-in -> hipMemcpy into a
    hipIpcOpenMemHandle block), concurrently with the stage reading them --
    the pattern whose failures round 4 routed around.  Every ring is
    destroyed after its example; the holder frees its blocks only once
    every importer has detached (dada_internal.h, the ordering rule)"""
    g = case["g"]
    tmp = tmp_path_factory.mktemp("gather_inproc")
    nblks = [max(1, case["nblk"] - shorter[r]) for r in range(nsub)]
    base = fresh_key()
    keys = [base + 0x10 * r for r in range(nsub)]
    blocks = [[co.fill_synthetic(g, g.block_bytes, case["seed"], r, b) for b in range(nblks[r])]
              for r in range(nsub)]
    args = ["-n", str(nsub), "-p", str(g.npol_out)] + (["-m"] if g.mean else []) + (["-S"] if case["sync"] else [])
    nbufs = case["nbufs"] if len(set(nblks)) == 1 else max(case["nbufs"], max(nblks) + 1)
    ohdr, sp, log = _run_stage(tmp, g, keys, blocks, args, True, nbufs, nsub, inproc=True)
    n = min(nblks)
    assert sp.shape[0] == n, (case, nblks, log[-600:])
    for b in range(n):
        for r in range(nsub):
            assert np.array_equal(sp[b, r], co.power(g, blocks[r][b], nthreads=8).view(np.uint32)), (case, b, r)
    assert dada.header_get(ohdr, "NSUBBAND", "%d") == nsub


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=10 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(cases(), st.integers(2, 4))
def test_stage_random_time_split(gpu, tmp_path_factory, case, nsplit):
    """-t 2..4 on a host ring: each block's frames cut into nsplit equal
    shares over as many contexts (all on the one test GPU), exact partials
    reduced; spectra equal one GPU's (the oracle's) bit for bit"""
    g0 = case["g"]
    frames = g0.nsamp_int // g0.nsamp_df
    frames = max(nsplit, frames - frames % nsplit)
    g = npo.Geom(**{**g0.asdict(), "nsamp_int": frames * g0.nsamp_df})
    tmp = tmp_path_factory.mktemp("split")
    key = fresh_key()
    blocks = [co.fill_synthetic(g, g.block_bytes, case["seed"], 5, b) for b in range(case["nblk"])]
    args = ["-t", str(nsplit), "-p", str(g.npol_out)] + (["-m"] if g.mean else [])
    short = (key,) if case["short"] else ()
    ohdr, sp, log = _run_stage(tmp, g, [key], [blocks], args, False, case["nbufs"], 1, short=short)
    assert sp.shape[0] == case["nblk"], (case, log[-600:])
    for b in range(case["nblk"]):
        assert np.array_equal(sp[b, 0], co.power(g, blocks[b], nthreads=8).view(np.uint32)), (case, b)
    assert dada.header_get(ohdr, "NSPLIT", "%d") == nsplit
    assert f"reduce of {nsplit} time shares" in log


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=8 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(st.integers(1, 64), st.integers(1, 8), st.integers(2, 5), st.floats(0.0, 0.3),
       st.floats(0.05, 1.0), st.sampled_from([0, 249_990, 249_999]), st.integers(0, 2 ** 31))
def test_dfdb_random_streams_to_spectra(gpu, tmp_path_factory, block_ndf, nblk, nbufs, loss, shuffle,
                                        ref_idf, s):
    """paf_dfgen stream (0-30 % of frames lost, arrival shuffled within up
    to one block, the 27-s wrap near the start or not) -> paf_dfdb (GPU
    assembly into a device ring, block by block) -> paf_baseband2power:
    every block the stream has frames for comes out, and output b is the
    oracle's spectrum of block b as the oracle places the stream's frames
    (lost frames read as zeros).  Before paf_dfdb followed the frames'
    timestamps, a lossy stream lost its last blocks and, further in, frames
    drifted out of the batches assembled into their block."""
    tmp = tmp_path_factory.mktemp("dfdb")
    nchunk = 48
    g = npo.Geom(nbit=16, big_endian=1, nchunk=nchunk, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=block_ndf * 128)
    per_block = block_ndf * nchunk
    payload = co.fill_synthetic(g, g.block_bytes * nblk, s, 2, 5)
    src = tmp / "bmf.dada"
    dada.write_dada_file(str(src), "NBIT 16\n", payload)
    df, ck = tmp / "s.df", tmp / "s.chunks"
    ref_sec = 27 * 40
    lost = int(loss * 1000)  # paf_dfgen -l: frames lost per mille
    window = max(1, int(shuffle * per_block))
    subprocess.run([os.path.join(BIN, "paf_dfgen"), "-i", str(src), "-o", str(df), "-n", str(nchunk),
                    "-c", str(ck), "-x", str(ref_idf), "-s", str(ref_sec), "-r", str(s % 1000),
                    "-w", str(window), "-l", str(lost)], check=True, capture_output=True)
    kin, kout = fresh_key(), fresh_key()
    from test_gpu_device_ring import HDR, _run_chain
    sp, log = _run_chain(tmp, kin, kout,
                         [os.path.join(BIN, "paf_dfdb"), "-a", f"{kin:x}", "-b", HDR, "-c", str(df),
                          "-k", str(ck), "-n", str(nchunk), "-x", str(ref_idf), "-s", str(ref_sec)],
                         "bmf", g.nout, nbufs, g.block_bytes)
    dfs = np.fromfile(df, dtype=np.uint8).reshape(-1, npo.DF_BYTES)
    chunk = np.fromfile(ck, dtype=np.uint8)
    h = npo.df_decode(dfs)
    rel = np.trunc(h["idf"].astype(np.float64) + (h["sec"].astype(np.float64) - ref_sec) / 1.08e-4 - ref_idf)
    assert sp.shape[0] == int(rel.max()) // block_ndf + 1, log[-600:]    # every block with frames
    idf, sec = ref_idf, ref_sec
    for b in range(sp.shape[0]):
        want = np.zeros(g.block_bytes, np.uint8)
        co.assemble(dfs, chunk, idf, sec, want, block_ndf, nchunk)
        assert np.array_equal(sp[b].view(np.uint32), co.power(g, want, nthreads=8).view(np.uint32)), \
            (block_ndf, nblk, nbufs, lost, window, ref_idf, s, b)
        gi = idf + block_ndf
        idf, sec = gi % 250000, sec + (gi // 250000) * 27


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=6 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large, HealthCheck.filter_too_much,
                                 HealthCheck.function_scoped_fixture])
@given(st.integers(1, 48), st.integers(1, 64), st.integers(1, 6), st.floats(0.0, 0.3), st.floats(0.05, 1.5),
       st.sampled_from([1000, 249_990]), st.integers(0, 2 ** 31))
def test_capture_random_streams_to_spectra(gpu, tmp_path_factory, nchunk, block_ndf, nblk, loss, shuffle,
                                           ref_idf, s):
    """UDP (3 loopback ports) -> paf_capture (host sort by timestamp, GPU
    assembly into a device ring) -> paf_baseband2power, for random chunk
    counts, block lengths, 0-30 % of frames lost at the source and arrival
    shuffled within up to 1.5 blocks (less than the temp buffer's 256 frame
    times, so nothing arrives too late to be placed): every output is the
    oracle's spectrum of its block as the oracle places the sent stream.
    A run where the loopback itself dropped a frame says nothing about the
    capture and is discarded (hypothesis.assume)."""
    import threading
    from hypothesis import assume
    tmp = tmp_path_factory.mktemp("cap")
    g = npo.Geom(nbit=16, big_endian=1, nchunk=nchunk, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=block_ndf * 128)
    per_block = block_ndf * nchunk
    window = max(1, min(int(shuffle * per_block), 200 * nchunk))
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
    assume(len(dfs) > 0)                      # every frame lost at the source: nothing to capture
    h = npo.df_decode(dfs)
    rel = np.trunc(h["idf"].astype(np.float64) + (h["sec"].astype(np.float64) - ref_sec) / 1.08e-4 - ref_idf)
    # the capture ends with the stream: blocks after the last frame's are not made
    n_out = min(nblk, int(rel.max()) // block_ndf + 1)
    hdr = tmp / "hdr.txt"
    hdr.write_text(f"HDR_SIZE 4096\nNBIT 16\nNDIM 2\nNPOL 2\nNCHAN {nchunk * 7}\nNCHUNK {nchunk}\n"
                   "NCHAN_CHUNK 7\nNSAMP_DF 128\nBYTE_ORDER BE\nTSAMP 0.84375\n")
    kin, kout = fresh_key(), fresh_key()
    dada.create_ring(kin, 4, g.block_bytes, device=0)
    dada.create_ring(kout, 8, g.nout * 4)
    port = 27000 + (os.getpid() % 400) * 8
    out = tmp / "power.dada"
    procs, cap_err = [], []
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b",
                                   f"{kout:x}", "-c", str(tmp), "-d", "0"], stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([os.path.join(BIN, "paf_capture"), "-a", f"{kin:x}", "-f", str(hdr),
                                   "-c", str(block_ndf), "-n", str(nblk), "-P", str(port), "-N", "3",
                                   "-m", "freq:1300", "-x", str(ref_idf), "-s", str(ref_sec), "-t", "1",
                                   "-d", "0"], stderr=subprocess.PIPE, text=True)]
        ready = threading.Event()

        def drain():  # the capture's log; ready once its receive threads run
            for ln in procs[2].stderr:
                cap_err.append(ln)
                if "receive thread(s) over" in ln:
                    ready.set()
        th = threading.Thread(target=drain, daemon=True)
        th.start()
        assert ready.wait(60), "".join(cap_err)[-800:]
        snd = subprocess.run([os.path.join(BIN, "paf_dfsend"), "-i", str(df), "-k", str(ck), "-P",
                              str(port), "-N", "3", "-r", "100"], capture_output=True, text=True)
        assert snd.returncode == 0, snd.stderr
        assert procs[2].wait(120) == 0, "".join(cap_err)[-800:]
        th.join(10)
        for p in procs[1::-1]:
            _, e = p.communicate(timeout=120)
            assert p.returncode == 0, e[-800:]
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
    log = "".join(cap_err)
    import re
    m = re.search(r"capture: (\d+) frames received", log)
    assert m, log[-800:]
    assume(int(m.group(1)) == len(dfs))      # the loopback delivered every frame sent
    sp = data.view(np.uint32).reshape(-1, g.nout)
    assert sp.shape[0] == n_out, log[-800:]
    idf, sec = ref_idf, ref_sec
    for b in range(n_out):
        want = np.zeros(g.block_bytes, np.uint8)
        co.assemble(dfs, chunk, idf, sec, want, block_ndf, nchunk)
        assert np.array_equal(sp[b], co.power(g, want, nthreads=8).view(np.uint32)), \
            (nchunk, block_ndf, nblk, loss, window, ref_idf, s, b, log[-600:])
        gi = idf + block_ndf
        idf, sec = gi % 250000, sec + (gi // 250000) * 27


@(seed(int(_SEED)) if _SEED else (lambda f: f))
@settings(max_examples=10 * _SCALE, deadline=None, derandomize=_SEED is None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large,
                                 HealthCheck.function_scoped_fixture])
@given(cases(), st.floats(0.0, 0.99))
def test_diskdb_random_files_to_spectra(gpu, tmp_path_factory, case, tail):
    """paf_diskdb (a DADA file: 4096-B header skipped, the template's header
    passed on, diskdb.cu:69,79-93) -> host or GPU-resident ring -> the stage:
    random layouts, ring depths and block counts, and a file that ends part-
    way through a block (that partial integration is skipped)"""
    g, nblk = case["g"], case["nblk"]
    tmp = tmp_path_factory.mktemp("diskdb")
    frames_tail = int(tail * (g.nsamp_int // g.nsamp_df))
    payload = co.fill_synthetic(g, g.block_bytes * nblk + frames_tail * g.frame_bytes, case["seed"], 6, 1)
    src = tmp / "obs.dada"
    dada.write_dada_file(str(src), "FILE_HEADER_IS_SKIPPED 1\n", payload)
    hdr = tmp / "header.txt"
    hdr.write_text(f"HDR_SIZE 4096\nNBIT {g.nbit}\nNDIM 2\nNPOL 2\nNCHAN {g.nchunk * g.nchan_chunk}\n"
                   f"NCHUNK {g.nchunk}\nNCHAN_CHUNK {g.nchan_chunk}\nNSAMP_DF {g.nsamp_df}\n"
                   f"BYTE_ORDER {'BE' if g.big_endian else 'LE'}\nTSAMP 0.84375\n")
    kin, kout = fresh_key(), fresh_key()
    from test_gpu_device_ring import _run_chain
    args = ["-p", str(g.npol_out)] + (["-m"] if g.mean else [])
    sp, log = _run_chain(tmp, kin, kout,
                         [os.path.join(BIN, "paf_diskdb"), "-a", f"{kin:x}", "-b", str(tmp), "-c", "obs.dada",
                          "-d", str(hdr), "-e", "1"],
                         "header", g.nout, case["nbufs"], g.block_bytes,
                         device=0 if case["device"] else -1, stage_args=args)
    assert sp.shape[0] == nblk, log[-600:]
    for b in range(nblk):
        blk = payload[b * g.block_bytes:(b + 1) * g.block_bytes]
        assert np.array_equal(sp[b].view(np.uint32), co.power(g, blk, nthreads=8).view(np.uint32)), (case, b)
    stage_log = open(str(tmp / "paf_baseband2power.log")).read()
    assert ("partial integration skipped" in stage_log) == (frames_tail > 0), stage_log[-600:]
