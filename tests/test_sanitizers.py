"""Host-code sanitizers (CPU): the DADA layer built with ASan+UBSan and with
TSan, driven by tests/c/ring_stress.c (writer + 2 reader threads, EOD, header
edits).  GPU sanitizers are not available on the test pool; these cover the
C code around the kernels."""
import os
import subprocess

import pytest

from conftest import REPO

SRC = [os.path.join(REPO, "paf-baseband2power_amd", "csrc", "dada", f)
       for f in ("dada_ring.c", "dada_query.c", "dada_device.c", "ascii_header.c")]
DRIVER = os.path.join(REPO, "tests", "c", "ring_stress.c")


@pytest.mark.parametrize("san,key", [("address,undefined", "7c10"), ("thread", "7c20")])
def test_dada_layer_under_sanitizer(tmp_path, san, key):
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
