"""UDP capture rate on the loopback interface.

A paf_dfgen stream of BMF frames (48 chunks) is sent by paf_dfsend at a set
rate to 6 ports; paf_capture assembles it on the GPU into a dada_db -g ring
that paf_baseband2power integrates.  For each rate the loss and the
capture's own timing are printed (one JSON line per rate).  One BMF NIC
carries 48 chunks x 7232 B every 108 us = 3.2 GB/s (capture.h:20,27,30).

  python tools/bench_capture.py [--ndf 1024] [--blocks 4] [--rates 800,1600,3200]
                                [--rx-threads 1,6] [--send-threads 1]

--rx-threads: paf_capture -R (receive threads; 0 = one per port, the
reference's layout); --send-threads: paf_dfsend -T (one sender thread
saturates near 5 GB/s on loopback).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "paf-baseband2power_amd"))
from paf_b2p import dada  # noqa: E402

BIN = dada.BIN_DIR


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndf", type=int, default=1024)
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--rates", default="800,1600,3200")
    ap.add_argument("--rx-threads", default="0")
    ap.add_argument("--send-threads", type=int, default=1)
    a = ap.parse_args()
    nchunk = 48
    d = tempfile.mkdtemp(prefix="bench_capture_")
    block = a.ndf * nchunk * 7168
    src = os.path.join(d, "in.dada")
    with open(src, "wb") as f:  # payload content does not matter for the rate
        f.write(dada.header_block("NBIT 16\n"))
        chunk = os.urandom(1 << 20)
        for _ in range(block * a.blocks // len(chunk)):
            f.write(chunk)
    df, ck = os.path.join(d, "s.df"), os.path.join(d, "s.chunks")
    subprocess.run([os.path.join(BIN, "paf_dfgen"), "-i", src, "-o", df, "-n", str(nchunk), "-c", ck,
                    "-x", "0", "-s", "27", "-f", "1300", "-r", "5", "-w", str(nchunk * 16)],
                   check=True, capture_output=True)
    os.unlink(src)
    hdr = os.path.join(d, "hdr.txt")
    with open(hdr, "w") as f:
        f.write("HDR_SIZE 4096\nNBIT 16\n")
    runs = [(int(r), int(x)) for x in a.rx_threads.split(",") for r in a.rates.split(",")]
    for i, (rate, rx) in enumerate(runs):
        kin, kout = 0x7e40 + 4 * i, 0x7e80 + 4 * i
        for k in (kin, kout):
            dada.destroy_ring(k)
        dada.create_ring(kin, 4, block, device=0)
        dada.create_ring(kout, 8, 336 * 4)
        port = 26000 + 16 * i
        procs = []
        try:
            procs = [subprocess.Popen([os.path.join(BIN, "paf_dbdisk"), "-k", f"{kout:x}", "-o",
                                       os.path.join(d, "p.dada")], stderr=subprocess.PIPE, text=True),
                     subprocess.Popen([os.path.join(BIN, "paf_baseband2power"), "-a", f"{kin:x}", "-b",
                                       f"{kout:x}", "-c", d, "-d", "0", "-f", "bmf"],
                                      stderr=subprocess.PIPE, text=True),
                     subprocess.Popen([os.path.join(BIN, "paf_capture"), "-a", f"{kin:x}", "-f", hdr,
                                       "-c", str(a.ndf), "-n", str(a.blocks), "-P", str(port), "-N", "6",
                                       "-m", "freq:1300", "-x", "0", "-s", "27", "-t", "1",
                                       "-R", str(rx)],
                                      stderr=subprocess.PIPE, text=True)]
            time.sleep(3)
            snd = subprocess.run([os.path.join(BIN, "paf_dfsend"), "-i", df, "-k", ck, "-P", str(port),
                                  "-N", "6", "-r", str(rate), "-T", str(a.send_threads)],
                                 capture_output=True, text=True)
            errs = [p.communicate(timeout=300)[1] for p in procs[::-1]]
            cap = errs[0]
            m = re.search(r"capture: (\d+) frames received.*?(\d+) frames placed.*?([0-9.]+) s from the first frame",
                          cap)
            s = re.search(r"(\d+) frames in ([0-9.]+) s \(([0-9.]+) MB/s\)", snd.stderr)
            sent = int(s.group(1)) if s else 0
            got, placed, el = (int(m.group(1)), int(m.group(2)), float(m.group(3))) if m else (0, 0, 0)
            print(json.dumps({"path": "UDP loopback -> paf_capture (GPU assembly) -> device ring -> "
                                      "paf_baseband2power", "rate_target_MBps": rate,
                              "rx_threads": rx or 6, "send_threads": a.send_threads,
                              "sent_MBps": float(s.group(3)) if s else None, "frames_sent": sent,
                              "frames_received": got, "frames_placed": placed,
                              "loss_pct": round(100.0 * (sent - got) / sent, 3) if sent else None,
                              "capture_s": el,
                              "captured_GBps": round(got * 7232 / el / 1e9, 2) if el else None,
                              "rc": [p.returncode for p in procs],
                              "capture_summary": next((ln[22:] for ln in cap.splitlines()
                                                       if "capture: " in ln), "")}),
                  flush=True)
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
            dada.destroy_ring(kin)
            dada.destroy_ring(kout)


if __name__ == "__main__":
    main()
