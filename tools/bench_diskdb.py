"""Measure BASELINE.json configs[0]: a 1024x1024-sample integration of
256 chans x 2 pols (int8) fed from a DADA file by paf_diskdb through a host
ring ("report the diskdb-fed C1 plumbing time separately").

Three consumers of the same ring, one leg each:
  sink  reads every block and does nothing: the file -> ring plumbing rate
        (paf_diskdb's fread into the shared-memory block, diskdb.cu:103-121)
  cpu   integrates every block with the oracle's C restatement (OpenMP,
        --threads): the reference-shaped CPU path (there is no reference
        implementation to time)
  gpu   paf_baseband2power -f int8:256 on GPU 0 (host ring: pinned H2D of
        every block, overlapped with the kernel) -> output ring -> paf_dbdisk
The file (--nint integrations, 1 GiB each, synthetic) is written first and
read once before the legs, so it is served from the page cache.  Prints one
JSON line per leg.

  python tools/bench_diskdb.py [--nint 4] [--legs sink,cpu,gpu] [--threads 16] [--readers 1,8] [--page 0,1]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "paf-baseband2power_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import b2p_oracle as npo  # noqa: E402
import oracle_c as co  # noqa: E402
from paf_b2p import dada  # noqa: E402

BIN = dada.BIN_DIR
HDR = os.path.join(os.path.dirname(BIN), "conf", "header_baseband2power.txt")
SEED = 20181105


def run_leg(leg: str, path: str, nint: int, g, threads: int, workdir: str, readers: int, page: bool) -> dict:
    kin, kout = 0x7d00, 0x7d10
    for k in (kin, kout):
        dada.destroy_ring(k)
    bufsz = g.block_bytes
    dada.create_ring(kin, 2, bufsz, page=page)  # dada_db -p: the reference launcher's ring
    procs, out = [], {}
    try:
        seen, acc = [], np.zeros(g.nout, dtype=np.uint64)
        t_first = []

        def consumer():
            with dada.Hdu(kin, "R") as r:
                r.read_header()
                while (b := r.view_block()) is not None:  # in place, no copy
                    if not t_first:
                        t_first.append(time.perf_counter())
                    seen.append(len(b))
                    if leg == "cpu" and len(b) == bufsz:
                        co.integrate(g, b, nthreads=threads, acc=acc)
                    r.release_block(len(b))

        if leg == "gpu":
            stage_log = os.path.join(workdir, "paf_baseband2power.log")
            if os.path.exists(stage_log):  # appended to by every run: this leg's lines only
                os.unlink(stage_log)
            dada.create_ring(kout, 8, g.nout * 4)
            procs.append(subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-W", "-o",
                                           os.path.join(workdir, "power.dada")], stderr=subprocess.PIPE))
            procs.append(subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b",
                                           f"{kout:x}", "-c", workdir, "-d", "0", "-f", f"int8:{g.nchan}"],
                                          stderr=subprocess.PIPE))
        else:
            th = threading.Thread(target=consumer)
            th.start()
        t0 = time.perf_counter()
        dk = subprocess.Popen([os.path.join(BIN, "paf_diskdb"), "-a", f"{kin:x}", "-b", os.path.dirname(path),
                               "-c", os.path.basename(path), "-d", HDR, "-e", "1", "-T", str(readers)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        procs.append(dk)
        dk_out, dk_err = dk.communicate(timeout=600)
        if dk.returncode != 0:
            raise RuntimeError(dk_err.decode(errors="replace")[-800:])
        m = re.search(r"diskdb: (\d+) B in \d+ blocks, ([0-9.]+) s", (dk_out + dk_err).decode(errors="replace"))
        diskdb = {"diskdb_s": float(m.group(2)), "diskdb_GBps": round(int(m.group(1)) / float(m.group(2)) / 1e9, 2)} \
            if m and float(m.group(2)) > 0 else {}
        m = re.search(r"([0-9.]+) s reading \(([0-9.]+) GB/s; ([0-9.]+) s of it in the first pass over the (\d+) "
                      r"ring blocks\), ([0-9.]+) s waiting", (dk_out + dk_err).decode(errors="replace"))
        if m:
            rest_s, rest_b = float(m.group(1)) - float(m.group(3)), (nint - int(m.group(4))) * bufsz
            diskdb.update({"diskdb_read_s": float(m.group(1)), "diskdb_read_GBps": float(m.group(2)),
                           "diskdb_first_pass_s": float(m.group(3)), "diskdb_wait_s": float(m.group(5)),
                           "diskdb_read_GBps_after_first_pass": round(rest_b / rest_s / 1e9, 2) if rest_s > 0 else None})
        m = re.search(r"([0-9.]+) s mapping the ring", (dk_out + dk_err).decode(errors="replace"))
        if m:
            diskdb["diskdb_map_s"] = float(m.group(1))
        if leg == "gpu":
            errs = {}
            for p in procs:
                if p is dk:
                    errs[p] = dk_err
                else:
                    _, errs[p] = p.communicate(timeout=600)
            if any(p.returncode for p in procs):
                raise RuntimeError("\n".join(f"{os.path.basename(p.args[0])} rc={p.returncode}: "
                                             + errs[p].decode(errors="replace")[-800:] for p in procs))
            wall = time.perf_counter() - t0
            log = open(os.path.join(workdir, "paf_baseband2power.log")).read()
            m = re.search(r"FINISH PAF_PROCESS: (\d+) integrations.* ([0-9.]+) s from the first", log)
            n_int, el = (int(m.group(1)), float(m.group(2))) if m else (0, 0.0)
            out = {"integrations": n_int, "consumer_s": el}
            _, payload = dada.read_dada_file(os.path.join(workdir, "power.dada"))
            spec = np.frombuffer(payload, dtype=np.float32).reshape(-1, g.nout)
            out["spectra_equal_oracle"] = spec.shape[0] == nint and all(
                np.array_equal(spec[b].view(np.uint32),
                               co.power(g, co.fill_synthetic(g, g.block_bytes, SEED, 0, b),
                                        nthreads=threads).view(np.uint32)) for b in range(nint))
        else:
            th.join(600)
            wall = time.perf_counter() - t0
            n_int = len(seen)
            el = time.perf_counter() - t_first[0] if t_first else 0.0
            out = {"integrations": n_int, "consumer_s": round(el, 4)}
            if leg == "cpu":  # exact sums over every integration vs the generator's blocks
                ref = np.zeros(g.nout, dtype=np.uint64)
                for b in range(nint):
                    co.integrate(g, co.fill_synthetic(g, g.block_bytes, SEED, 0, b), nthreads=threads, acc=ref)
                out["sums_equal_oracle"] = bool(np.array_equal(acc, ref))
        out.update(diskdb)
        samples = g.nchan * g.npol * g.nsamp_int  # channels x pols x time, as bench.py counts
        out.update({
            "leg": leg, "config": "configs[0]: 256 ch x 2 pol int8, 1 GiB per integration, paf_diskdb -> host ring",
            "wall_s": round(wall, 4),
            "GBps_wall": round(nint * bufsz / wall / 1e9, 2),
            "Msamples_s_wall": round(nint * samples / wall / 1e6, 1),
            "threads": threads if leg == "cpu" else None,
            "diskdb_readers": readers,
            "ring_paged": page,
        })
        return out
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for k in (kin, kout):
            dada.destroy_ring(k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nint", type=int, default=4)
    ap.add_argument("--legs", default="sink,cpu,gpu")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--nchan", type=int, default=256)
    ap.add_argument("--readers", default="8", help="paf_diskdb -T values, comma-separated (one set of legs each)")
    ap.add_argument("--page", default="1", help="ring created with dada_db -p (1) or not (0); comma-separated")
    a = ap.parse_args()
    g = npo.Geom(nbit=8, nchan_chunk=a.nchan)
    workdir = tempfile.mkdtemp(prefix="bench_diskdb_")
    path = os.path.join(workdir, "c1.dada")
    with open(path, "wb") as f:  # header + nint synthetic integrations
        f.write(dada.header_block("NBIT 8\nNCHAN %d\n" % a.nchan))
        for b in range(a.nint):
            co.fill_synthetic(g, g.block_bytes, SEED, 0, b).tofile(f)
    with open(path, "rb") as f:  # into the page cache
        while f.read(64 << 20):
            pass
    try:
        for page in (x == "1" for x in a.page.split(",")):
            for readers in (int(x) for x in a.readers.split(",")):
                for leg in a.legs.split(","):
                    print(json.dumps(run_leg(leg, path, a.nint, g, a.threads, workdir, readers, page)), flush=True)
    finally:
        os.unlink(path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
