"""Property test of the stage end to end: `paf_baseband2power` between a
PSRDADA writer (this process) and `paf_dbdisk`, on layouts the input header
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
from hypothesis import HealthCheck, given, seed, settings
from hypothesis import strategies as st

import b2p_oracle as npo
import oracle_c as co
from paf_b2p import dada
from test_gpu_device_ring import BIN, _wait, fresh_key

pytestmark = pytest.mark.gpu
_SCALE = int(os.environ.get("B2P_HYPOTHESIS_SCALE", "1"))
_SEED = os.environ.get("B2P_HYPOTHESIS_SEED")


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


def _run_stage(tmp, g, keys, rings_blocks, stage_args, device, nbufs, out_nsub, short=()):
    """create one input ring per key, start paf_dbdisk and the stage, write
    each ring's blocks from its own thread (the stage reads every ring each
    round), and return (output header, spectra [n, out_nsub, nout] as uint32,
    stage log)"""
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
        ths = [threading.Thread(target=writer, args=(k, bl, k in short)) for k, bl in zip(keys, rings_blocks)]
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
