"""The drop-in stage, on the HIP library, when an input ring is destroyed
under it (`dada_db -k KEY -d` while it waits for the next block).

The CPU double of the library runs the same case in every threading mode
(tests/test_stage_stub_random.py::test_stage_input_ring_removed_under_it);
here the stage is the shipped binary on the GPU.  The removal is not an end
of data: the stage names the ring in an ERR line on stderr, wakes every other
member, ends the output transfer (paf_dbdisk closes its file, exit 0) and
exits 1, after writing the spectra of the blocks it had, each equal to the C
oracle's.

A GPU-resident ring's holder keeps its blocks while the stage (and this
process, its writer) still have them open: `dada_db -d` waits for them, then
removes the ring's keys and reports them (EBUSY); the holder frees the
blocks once the last of them has detached (device rings)."""
import os
import subprocess
import time

import numpy as np
import pytest

import b2p_oracle as npo
import oracle_c as co
from paf_b2p import dada
from test_gpu_device_ring import BIN, fresh_key

pytestmark = pytest.mark.gpu
_T0 = time.time()


def _phase(what: str) -> None:
    """a timestamped line per phase (pytest -s shows them): where a stuck run stopped"""
    print(f"[{time.time() - _T0:8.2f}] {what}", flush=True)


@pytest.mark.parametrize("mode", ["single", "gathered", "split", "single_dev", "gathered_dev"])
def test_stage_input_ring_removed_under_it_gpu(gpu, tmp_path, mode):
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=16, npol_out=1, nsamp_int=128)
    device = 0 if mode.endswith("_dev") else -1
    nmem = 2 if mode in ("gathered", "gathered_dev", "split") else 1
    rings = nmem if mode.startswith("gathered") else 1
    onsub = nmem if mode.startswith("gathered") else 1
    nblk = 2
    blocks = [[co.fill_synthetic(g, g.block_bytes, 71, r, b) for b in range(nblk)] for r in range(rings)]
    hdr = ("HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 16\nNCHUNK 1\nNCHAN_CHUNK 16\nNSAMP_DF 1\n"
           "BYTE_ORDER LE\nTSAMP 0.84375\n")
    kout, base = fresh_key(), fresh_key()
    keys = [base + 0x10 * r for r in range(rings)]
    for k in keys:
        dada.destroy_ring(k)
        dada.create_ring(k, 4, g.block_bytes, device=device)
    dada.create_ring(kout, 8, onsub * g.nout * 4)
    args = ["-f", "header"] + (["-n", str(nmem), "-G", "copy"] if mode.startswith("gathered") else []) \
        + (["-t", str(nmem), "-G", "copy"] if mode == "split" else [])
    out = tmp_path / "power.dada"
    want_bytes = 4096 + nblk * onsub * g.nout * 4
    procs, writers = [], []
    _phase(f"{mode}: rings made")
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{base:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp_path), "-d", "0"] + args, stderr=subprocess.PIPE, text=True)]
        for k, bl in zip(keys, blocks):  # the transfers stay open: the stage waits for a third block
            w = dada.Hdu(k, "W")
            writers.append(w)
            w.write_header(hdr)
            for b in bl:
                w.write_block(b.tobytes())
        _phase("blocks written")
        t_end = time.time() + 60
        while time.time() < t_end and procs[1].poll() is None and (
                not out.exists() or out.stat().st_size < want_bytes):
            time.sleep(0.05)
        time.sleep(0.3)
        assert procs[1].poll() is None, procs[1].communicate()[1]  # waiting for the next block
        _phase(f"spectra out ({out.stat().st_size if out.exists() else 0} B); destroying ring {keys[0]:x}")
        removed = dada.destroy_ring(keys[0])
        _phase(f"destroy returned {removed}")
        if device >= 0:  # the stage and this process still have its blocks open
            assert not removed and "still have the blocks open" in dada.device_error(), dada.device_error()
        _, err = procs[1].communicate(timeout=60)
        _phase(f"stage exited {procs[1].returncode}")
        _, derr = procs[0].communicate(timeout=60)
        _phase(f"paf_dbdisk exited {procs[0].returncode}")
        assert procs[1].returncode == 1, err
        assert procs[0].returncode == 0, derr
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        _phase("closing writers")
        for w in writers:
            try:
                w.close()
            except OSError:
                pass
        _phase("destroying rings")
        for k in keys + [kout]:
            dada.destroy_ring(k)
        _phase("done")
    assert f"reading input ring {keys[0]:x} failed" in err and "] ERR: " in err, err
    sp = data.view(np.uint32).reshape(-1, onsub, g.nout)
    assert sp.shape[0] == nblk, sp.shape
    for b in range(nblk):
        for r in range(onsub):
            assert np.array_equal(sp[b, r], co.power(g, blocks[r][b], nthreads=1).view(np.uint32)), (b, r)


_WRITER = """
import sys, time
sys.path.insert(0, {pkg!r})
import numpy as np
from paf_b2p import dada
key, path = int(sys.argv[1], 16), sys.argv[2]
w = dada.Hdu(key, "W")
w.write_header(open(path + ".hdr").read())
for b in np.split(np.fromfile(path, dtype=np.uint8), 2):
    w.write_block(b.tobytes())
print("written", flush=True)
time.sleep(120)  # the transfer stays open until this process is killed
"""


@pytest.mark.parametrize("device", [-1, 0])
def test_stage_notices_a_dead_writer_gpu(gpu, tmp_path, device):
    """-W 1 on the GPU: the ring's writer is killed mid-transfer (SIGKILL;
    on a GPU-resident ring its imported blocks go with it, the holder keeps
    them for the stage); the stage logs "its writer went away" after the
    grace second and exits 1, both spectra written and equal to the
    oracle's"""
    import signal
    import sys
    g = npo.Geom(nbit=8, nchunk=1, nsamp_df=1, nchan_chunk=16, npol_out=1, nsamp_int=128)
    blocks = [co.fill_synthetic(g, g.block_bytes, 83, 0, b) for b in range(2)]
    kout, kin = fresh_key(), fresh_key()
    dada.create_ring(kin, 4, g.block_bytes, device=device)
    dada.create_ring(kout, 8, g.nout * 4)
    f = tmp_path / "in.u8"
    np.concatenate([b.reshape(-1).view(np.uint8) for b in blocks]).tofile(f)
    (tmp_path / "in.u8.hdr").write_text("HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN 16\nNCHUNK 1\n"
                                        "NCHAN_CHUNK 16\nNSAMP_DF 1\nBYTE_ORDER LE\nTSAMP 0.84375\n")
    script = tmp_path / "writer.py"
    script.write_text(_WRITER.format(pkg=os.path.dirname(BIN)))
    out = tmp_path / "power.dada"
    procs, writer = [], None
    try:
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", str(out)],
                                  stderr=subprocess.PIPE, text=True),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b", f"{kout:x}",
                                   "-c", str(tmp_path), "-d", "0", "-f", "header", "-W", "1"],
                                  stderr=subprocess.PIPE, text=True)]
        writer = subprocess.Popen([sys.executable, str(script), f"{kin:x}", str(f)], stdout=subprocess.PIPE,
                                  text=True)
        assert writer.stdout.readline().strip() == "written"
        t_end = time.time() + 60
        while (not out.exists() or out.stat().st_size < 4096 + 2 * g.nout * 4) and time.time() < t_end:
            time.sleep(0.05)
        writer.send_signal(signal.SIGKILL)
        writer.wait()
        _, err = procs[1].communicate(timeout=60)
        _, derr = procs[0].communicate(timeout=60)
        assert procs[1].returncode == 1, err
        assert procs[0].returncode == 0, derr
        _, data = dada.read_dada_file(str(out))
    finally:
        for p in procs + ([writer] if writer else []):
            if p.poll() is None:
                p.kill()
                p.wait()
        dada.destroy_ring(kin)
        dada.destroy_ring(kout)
    assert f"input ring {kin:x}: its writer went away" in err, err
    sp = data.view(np.uint32).reshape(-1, g.nout)
    assert sp.shape[0] == 2
    for b in range(2):
        assert np.array_equal(sp[b], co.power(g, blocks[b], nthreads=1).view(np.uint32)), b
