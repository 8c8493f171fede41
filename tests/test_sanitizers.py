"""Host-code sanitizers (CPU): the DADA layer built with ASan+UBSan and with
TSan, driven by tests/c/ring_stress.c (writer + 2 reader threads, EOD, header
edits).  GPU sanitizers are not available on the test pool; these cover the
C code around the kernels."""
import os
import subprocess

import pytest

from conftest import REPO

SRC = [os.path.join(REPO, "paf-baseband2power_amd", "csrc", "dada", f)
       for f in ("dada_ring.c", "dada_device.c", "ascii_header.c")]
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
