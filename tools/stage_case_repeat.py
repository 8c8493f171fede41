#!/usr/bin/env python3
"""Run round 5's one failing stage example N times on the GPU, as the GPU
test runs it, stopping at the first failure with everything it left: the
stage's exit status, its stderr (a failed stage repeats its ERR log lines
there) and its log file.  DESIGN.md item 1.

The case (profiles/r05_gpu_suite_gather_flake.txt): `paf_baseband2power -n 2
-f header -p 2 -m` on two device rings of 6 blocks of 1 249 952 B (int8,
11 x 53 channels, 67 frames of 8 samples), written by two paf_diskdb
processes; sub-band 0's transfer is one block, sub-band 1's two.  Every
output is checked against the C oracle.

  python3 tools/stage_case_repeat.py N [churn=K]   (one JSON line per run, then a summary)

churn=K tests the candidate cause named in DESIGN.md item 1: before each
run, THIS process makes K other device rings one after another, each
written here (its blocks imported into this long-lived process, as the GPU
suite's in-process writers do) and read by a paf_dbdisk, and destroyed just
before the next is made -- the churn the recorded failure ran after.  The
case's own rings are then made at once, without a pause.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "paf-baseband2power_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402

import b2p_oracle as npo  # noqa: E402
import oracle_c as co  # noqa: E402
from paf_b2p import dada  # noqa: E402

BIN = dada.BIN_DIR


def churn(k: int, tmp: str, size: int) -> dict:
    """k device rings made, written here, read by paf_dbdisk and destroyed,
    back to back; the holders' export records"""
    key, rec = 0x7e80, {"rings": 0, "export_retries": 0, "primer_refused": 0}
    sink = os.path.join(tmp, "churn.dada")
    for i in range(k):
        nb = (2, 4, 6)[i % 3]
        dada.destroy_ring(key)
        dada.create_ring(key, nb, size, device=0)
        info = dada.device_ring_info(key)
        rec["rings"] += 1
        rec["export_retries"] += info["export_retries"]
        rec["primer_refused"] += info["primer_refused"]
        if os.path.exists(sink):
            os.remove(sink)
        rd = subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{key:x}", "-o", sink],
                              stderr=subprocess.DEVNULL)
        try:
            with dada.Hdu(key, "W") as w:
                w.write_header("HDR_SIZE 4096\n")
                for _ in range(nb + 1):
                    w.write_block(b"\1" * size)
            rd.wait(60)
        finally:
            if rd.poll() is None:
                rd.kill()
                rd.wait()
            dada.destroy_ring(key)
    return rec


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    k_churn = next((int(a[6:]) for a in sys.argv[2:] if a.startswith("churn=")), 0)
    g = npo.Geom(nbit=8, big_endian=0, nchunk=11, nsamp_df=8, nchan_chunk=53, npol_out=2, nsamp_int=536, mean=1)
    nblks = [1, 2]
    blocks = [[co.fill_synthetic(g, g.block_bytes, 1440, r, b) for b in range(nblks[r])] for r in range(2)]
    want = [co.power(g, blocks[r][0], nthreads=4).view(np.uint32) for r in range(2)]
    tmp = tempfile.mkdtemp(prefix="case_repeat_")
    hdr = (f"HDR_SIZE 4096\nNBIT 8\nNDIM 2\nNPOL 2\nNCHAN {g.nchunk * g.nchan_chunk}\nNCHUNK {g.nchunk}\n"
           f"NCHAN_CHUNK {g.nchan_chunk}\nNSAMP_DF {g.nsamp_df}\nBYTE_ORDER LE\nTSAMP 0.84375\n")
    for r in range(2):
        dada.write_dada_file(os.path.join(tmp, f"in{r}.dada"), "FILE_HEADER_IS_SKIPPED 1\n",
                             np.concatenate([b.reshape(-1).view(np.uint8) for b in blocks[r]]))
        open(os.path.join(tmp, f"hdr{r}.txt"), "w").write(hdr)
    base = 0x7c00
    keys, kout = [base, base + 0x10], base + 2
    fails = 0
    print(json.dumps({"runs": n, "churn": k_churn}), flush=True)
    for run in range(n):
        d = os.path.join(tmp, f"run{run}")
        os.makedirs(d)
        ch = churn(k_churn, tmp, g.block_bytes) if k_churn else None
        for k in keys + [kout]:
            dada.destroy_ring(k)
        for k in keys:
            dada.create_ring(k, 6, g.block_bytes, device=0)
        dada.create_ring(kout, 4, 2 * g.nout * 4)
        out = os.path.join(d, "power.dada")
        t0 = time.time()
        procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o", out],
                                  stderr=subprocess.PIPE),
                 subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{base:x}", "-b", f"{kout:x}",
                                   "-c", d, "-d", "0", "-f", "header", "-n", "2", "-p", "2", "-m"],
                                  stderr=subprocess.PIPE)]
        procs += [subprocess.Popen([os.path.join(BIN, "paf_diskdb"), "-a", f"{keys[r]:x}", "-b", tmp, "-c",
                                    f"in{r}.dada", "-d", os.path.join(tmp, f"hdr{r}.txt"), "-e", "1"],
                                   stderr=subprocess.PIPE) for r in (0, 1)]
        t_end = time.time() + 60
        while any(p.poll() is None for p in procs) and time.time() < t_end:
            if any(p.poll() not in (None, 0) for p in procs):
                break
            time.sleep(0.02)
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        rcs = [p.returncode for p in procs]
        errs = [p.stderr.read().decode(errors="replace")[-600:] for p in procs]
        ok = all(rc == 0 for rc in rcs)
        if ok:
            _, data = dada.read_dada_file(out)
            sp = data.view(np.uint32).reshape(-1, 2, g.nout)
            ok = sp.shape[0] == 1 and all(np.array_equal(sp[0, r], want[r]) for r in range(2))
        for k in keys + [kout]:
            dada.destroy_ring(k)
        log = open(os.path.join(d, "paf_baseband2power.log")).read() if os.path.exists(
            os.path.join(d, "paf_baseband2power.log")) else ""
        rec = {"run": run, "ok": ok, "rcs": dict(zip(["dbdisk", "stage", "diskdb0", "diskdb1"], rcs)),
               "s": round(time.time() - t0, 2)}
        if ch:
            rec["churn"] = ch
        if not ok:
            fails += 1
            rec.update(stderr=errs, stage_log=log[-3000:])
        print(json.dumps(rec), flush=True)
        if not ok:
            break
    print(json.dumps({"runs": run + 1, "failures": fails}), flush=True)
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
