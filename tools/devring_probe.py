#!/usr/bin/env python3
"""How often does creating a GPU-resident ring (dada_db -g) fail, and where?

Creates and destroys device rings of assorted block sizes and depths, N
times each, one after another (as the stage property tests do), and prints
one JSON line: attempts, failures and IPC-export retries per (block size,
depth), and the holder's error text of each distinct failure.  With `use`,
each used ring's line also carries this process's open file descriptors
and mapped size after the ring was closed, so a per-import leak in the HIP
runtime's IPC path shows as steady growth.

  python3 tools/devring_probe.py [ROUNDS] [use] [noprimer] [pause=S] [handles]
    use       open and write every ring
    noprimer  the holders make no primer allocation (DADA_HOLDER_NO_PRIMER=1):
              block 0 is their first allocation, as before round 5
    pause=S   sleep S seconds between a ring's destroy and the next create
              (the previous holder has then long exited)
    handles   read every block's 64-B IPC handle from its segment (no block is
              opened) and report handles that recur across rings
"""
import collections
import json
import os
import re
import subprocess
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "paf-baseband2power_amd"))
from paf_b2p import dada  # noqa: E402

SIZES = [1040, 29952, 1 << 16, 1032192, 3096576, (3 << 20) + 48, 16 << 20]


def _vm() -> dict:
    out = {}
    for line in open("/proc/self/status"):
        k, _, v = line.partition(":")
        if k in ("VmSize", "VmRSS"):
            out[k] = v.strip()
    return out


def _handles(key: int, nbufs: int) -> list:
    """the 64-B IPC handle in each block's segment (key + 0x10000 (10 + i)),
    read through SysV calls without opening the block"""
    import ctypes
    libc = ctypes.CDLL(None, use_errno=True)
    libc.shmat.restype = ctypes.c_void_p
    libc.shmat.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    libc.shmdt.argtypes = [ctypes.c_void_p]
    out = []
    for i in range(nbufs):
        sid = libc.shmget(key + 0x10000 * (10 + i), 0, 0)
        if sid < 0:
            out.append(None)
            continue
        a = libc.shmat(sid, None, 0o10000)  # SHM_RDONLY
        out.append(ctypes.string_at(a, 64).hex())
        libc.shmdt(ctypes.c_void_p(a))
    return out


def main():
    import resource
    print(json.dumps({"rlimit_nofile": resource.getrlimit(resource.RLIMIT_NOFILE),
                      "fds": len(os.listdir("/proc/self/fd"))}), flush=True)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    use = "use" in sys.argv[2:]
    pause = next((float(a[6:]) for a in sys.argv[2:] if a.startswith("pause=")), 0.0)
    env = dict(os.environ)
    if "noprimer" in sys.argv[2:]:
        env["DADA_HOLDER_NO_PRIMER"] = "1"
    want_handles = "handles" in sys.argv[2:]
    seen = {}  # handle -> first (round, case, block)
    recur = []
    print(json.dumps({"use": use, "noprimer": "noprimer" in sys.argv[2:], "pause_s": pause}), flush=True)
    import tempfile
    tmp = tempfile.mkdtemp(prefix="devring_probe_")
    key = 0x7e40
    fails, retries, errs, attempts = collections.Counter(), collections.Counter(), {}, 0
    primer = collections.Counter()  # holders whose primer (first) allocation did not export
    for r in range(rounds):
        for sz in SIZES:
            for nb in (2, 4, 6):
                attempts += 1
                dada.destroy_ring(key)
                if pause:
                    time.sleep(pause)
                try:
                    p = subprocess.run([os.path.join(dada.BIN_DIR, "dada_db"), "-k", f"{key:x}", "-b", str(sz),
                                        "-n", str(nb), "-g", "0"], capture_output=True, text=True, timeout=120,
                                       env=env)
                    if "primer allocation was not exportable" in p.stderr:
                        primer[f"{sz}x{nb}"] += 1
                    m = re.search(r"(\d+) IPC export retr", p.stderr)
                    if m:
                        retries[f"{sz}x{nb}"] += int(m.group(1))
                        # the holder's first failed try: call, error, address range
                        print(json.dumps({"retry": f"{sz}x{nb}", "round": r,
                                          "holder": p.stderr.strip()[-300:]}), flush=True)
                    if p.returncode == 0 and want_handles:
                        for i, h in enumerate(_handles(key, nb)):
                            if h in seen:
                                recur.append({"handle": h, "first": seen[h], "again": [r, f"{sz}x{nb}", i]})
                            else:
                                seen.setdefault(h, [r, f"{sz}x{nb}", i])
                        if r == 0 and sz == SIZES[0] and nb == 2:
                            print(json.dumps({"sample_handles": _handles(key, nb)}), flush=True)
                    if p.returncode != 0:
                        fails[f"{sz}x{nb}"] += 1
                        e = p.stderr.strip()[-200:]
                        errs[e] = errs.get(e, 0) + 1
                    if p.returncode == 0 and use:
                        # use the ring as the tests do: a reader process and
                        # a writer here open every block's IPC handle
                        sink = os.path.join(tmp, "sink.dada")
                        if os.path.exists(sink):
                            os.remove(sink)
                        rd = subprocess.Popen([os.path.join(dada.BIN_DIR, "paf_dbdisk"), "-k", f"{key:x}",
                                               "-o", sink], stderr=subprocess.DEVNULL)
                        try:
                            with dada.Hdu(key, "W") as w:
                                w.write_header("HDR_SIZE 4096\n")
                                for _ in range(nb + 1):
                                    w.write_block(b"\1" * sz)
                        except OSError as e:  # the device-ring error text, then stop
                            rd.kill()
                            print(json.dumps({"error": str(e), "case": f"{sz}x{nb}",
                                              "fds": len(os.listdir("/proc/self/fd"))}), flush=True)
                            raise
                        rd.wait(60)
                        print(json.dumps({"used": f"{sz}x{nb}", "fds": len(os.listdir("/proc/self/fd")),
                                          "vm": _vm()}), flush=True)
                finally:
                    dada.destroy_ring(key)
        print(json.dumps({"round": r, "attempts": attempts, "failures": sum(fails.values()),
                          "retries": sum(retries.values()), "primer_refused": sum(primer.values())}), flush=True)
    if want_handles:
        print(json.dumps({"distinct_handles": len(seen), "recurring": len(recur), "recur_examples": recur[:10]}),
              flush=True)
    print(json.dumps({"attempts": attempts, "failures": sum(fails.values()), "by_case": fails,
                      "retries": sum(retries.values()), "retries_by_case": retries,
                      "primer_refused": sum(primer.values()), "primer_refused_by_case": primer,
                      "errors": errs}), flush=True)


if __name__ == "__main__":
    main()
